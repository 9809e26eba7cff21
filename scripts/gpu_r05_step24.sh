# Round 5, step 24: raster2d_bwd_tp's pass 1 restructured (the per-step body as a lambda: the
# default build) and stepping two records at a time (HGSR_BWD2_U2).  Parity on both, then c3 A/Bs
# against the previous build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s24
for v in lib lib_bu2; do
  HGSR_LIB=horizongs_amd/_$v/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity_dense.py tests/test_gpu_parity.py -k "2dgs or 2d" > gpurun_out/r05s24/tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/r05s24/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05s24/tests_$v.log
done
TAG=r05s24/ab_refac LIB_A=horizongs_amd/_lib_prev/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
TAG=r05s24/ab_bu2 LIB_A=horizongs_amd/_lib_prev/libhgsr.so LIB_B=horizongs_amd/_lib_bu2/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
