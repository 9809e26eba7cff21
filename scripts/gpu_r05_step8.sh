# Round 5, step 8: two ways at the raster backwards' float atomics.
#  - _lib_rec: accumulator rows padded to whole lines (2DGS 96 -> 128 B, 3DGS 48 -> 64 B) so no
#    row's atomics straddle two cache lines;
#  - _lib_merge: raster3d_bwd merges the four waves' partial sums of a batch in LDS and adds them
#    once per (tile, Gaussian), one batch later (HGSR_BWD3_MERGE).
# Parity on each build, then interleaved A/Bs against the default build (camera set, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s8
for v in merge rec; do
  HGSR_LIB=horizongs_amd/_lib_$v/libhgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity_dense.py tests/test_gpu_parity.py > gpurun_out/r05s8/tests_$v.log 2>&1 || { tail -30 gpurun_out/r05s8/tests_$v.log; exit 1; }
  tail -2 gpurun_out/r05s8/tests_$v.log
done
TAG=r05s8/ab_merge LIB_B=horizongs_amd/_lib_merge/libhgsr.so CONFIGS="c2 c2-fixed" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
TAG=r05s8/ab_rec LIB_B=horizongs_amd/_lib_rec/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
