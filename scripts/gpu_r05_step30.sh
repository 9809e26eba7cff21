# Round 5, step 30: probe -- raster2d_bwd_tp's pass 2 without the hit projection (cz, rcp; wrong
# results, frozen scene) vs the default: how much of the backward that VALU costs.
set -o pipefail
TAG=r05s30/p2c LIB_B=horizongs_amd/_lib_p2c/libhgsr.so CONFIGS="c3" REPS=2 BENCH_EXTRA=--freeze bash scripts/gpu_r04_ab.sh
