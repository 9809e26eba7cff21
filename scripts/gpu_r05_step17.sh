# Round 5, step 17: the 3DGS backward's tiles ordered by the ranges it walks (each tile's
# latest contributor + 1, written by the forward; HGSR_BWD_ORDER) instead of by whole-bin counts.
# Parity on the new build (default and variant share the buffer layout), then an interleaved A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s17
for v in lib lib_bo; do
  HGSR_LIB=horizongs_amd/_$v/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity_dense.py tests/test_gpu_parity.py tests/test_gpu_deferred.py > gpurun_out/r05s17/tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/r05s17/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05s17/tests_$v.log
done
TAG=r05s17/ab_bo LIB_B=horizongs_amd/_lib_bo/libhgsr.so CONFIGS="c2 c2-fixed" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
