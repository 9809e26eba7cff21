# Round 5, step 13: rasterization()'s SH colour kernels with the coefficient / gradient rows staged
# through LDS (contiguous float4 runs instead of 108-B lane-strided rows).  SH parity tests on the
# new build, then a c4 (SH2 colour head) A/B against the old kernels (2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s13
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_glue.py \
  tests/test_gpu_decode.py > gpurun_out/r05s13/tests.log 2>&1 || { tail -30 gpurun_out/r05s13/tests.log; exit 1; }
tail -1 gpurun_out/r05s13/tests.log
TAG=r05s13/ab_sh LIB_A=horizongs_amd/_lib_shold/libhgsr.so CONFIGS="c4" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
