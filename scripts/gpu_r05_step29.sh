# Round 5, step 29: raster2d_bwd_tp at 4 / 6 waves per SIMD vs the default 5 (c3 A/Bs).
set -o pipefail
TAG=r05s29/w4 LIB_B=horizongs_amd/_lib_w4/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh &&
TAG=r05s29/w6 LIB_B=horizongs_amd/_lib_w6/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh
