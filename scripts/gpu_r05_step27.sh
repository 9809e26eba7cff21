# Round 5, step 27: raster3d_bwd batch-top waits that leave the previous batch's atomics in flight
# (HGSR_BWD_LADDER=1, default build) vs vmcnt(0) (_lib_l0): parity tests, then interleaved c2 A/Bs
# on the camera set and on a frozen scene.
set -o pipefail
TAG=r05s27/ab TESTS="tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_run_to_run.py" \
  LIB_A=horizongs_amd/_lib_l0/libhgsr.so CONFIGS="c2" REPS=3 bash scripts/gpu_r04_ab.sh &&
TAG=r05s27/frz LIB_A=horizongs_amd/_lib_l0/libhgsr.so CONFIGS="c2" REPS=2 BENCH_EXTRA=--freeze bash scripts/gpu_r04_ab.sh
