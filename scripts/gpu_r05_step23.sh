# Round 5, step 23: raster2d_fwd stepping two records per loop iteration (HGSR_FWD2_U2): their
# loads, hits and exponentials are independent -- more work in flight per wave for a loop that the
# no-packed-fp32 A/B showed to be dependency-bound.  2DGS parity on the build, then a c3 A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s23
HGSR_LIB=horizongs_amd/_lib_u2/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity_dense.py tests/test_gpu_parity.py -k "2dgs or 2d" > gpurun_out/r05s23/tests.log 2>&1 \
  || { tail -30 gpurun_out/r05s23/tests.log; exit 1; }
tail -1 gpurun_out/r05s23/tests.log
TAG=r05s23/ab_u2 LIB_B=horizongs_amd/_lib_u2/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
