# Round 5, step 38: raster2d_fwd with 128-record batches instead of 64 on the camera set (c3 A/B).
set -o pipefail
TAG=r05s38/fb128 LIB_B=horizongs_amd/_lib_fb128/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh
