# Round 5, step 9: the LDS-DMA record staging issued as inline asm (HGSR_ASM_DMA).  With the
# builtin, the compiler put s_waitcnt vmcnt(0) in front of LDS reads it could not prove disjoint
# from the DMA destination: once per 4-step group in raster3d_bwd (the transpose read), once per
# pixel row in raster2d_bwd_tp's pass 2, and on the first record reads of every batch in
# raster2d_fwd -- each waits for the next batch's prefetch and every outstanding gradient atomic.
# Parity on the asm builds, then interleaved A/Bs against the default build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s9
for v in adma adma2; do
  HGSR_LIB=horizongs_amd/_lib_$v/libhgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity_dense.py tests/test_gpu_parity.py > gpurun_out/r05s9/tests_$v.log 2>&1 || { tail -30 gpurun_out/r05s9/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05s9/tests_$v.log
done
TAG=r05s9/ab_adma LIB_B=horizongs_amd/_lib_adma/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
TAG=r05s9/ab_adma2 LIB_B=horizongs_amd/_lib_adma2/libhgsr.so CONFIGS="c2" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
