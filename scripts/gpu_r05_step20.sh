# Round 5, step 20: isect_emit with four returning cursor atomics in flight per lane before their
# key stores (HGSR_EMIT_BATCH).  Bit-exact isect tests on the variant, then an interleaved A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s20
HGSR_LIB=horizongs_amd/_lib_eb/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_deferred.py tests/test_gpu_parity_dense.py > gpurun_out/r05s20/tests.log 2>&1 \
  || { tail -30 gpurun_out/r05s20/tests.log; exit 1; }
tail -1 gpurun_out/r05s20/tests.log
TAG=r05s20/ab_eb LIB_B=horizongs_amd/_lib_eb/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
