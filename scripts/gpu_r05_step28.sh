# Round 5, step 28: raster3d_fwd reads the next group's list entries ahead (default build) vs
# HEAD (_lib_base): 3DGS parity tests, then interleaved c2 A/Bs (camera set, frozen scene).
set -o pipefail
TAG=r05s28/ab TESTS="tests/test_gpu_parity.py tests/test_gpu_run_to_run.py" \
  LIB_A=horizongs_amd/_lib_base/libhgsr.so CONFIGS="c2" REPS=3 bash scripts/gpu_r04_ab.sh &&
TAG=r05s28/frz LIB_A=horizongs_amd/_lib_base/libhgsr.so CONFIGS="c2" REPS=2 BENCH_EXTRA=--freeze bash scripts/gpu_r04_ab.sh
