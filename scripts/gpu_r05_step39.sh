# Round 5, step 39: raster3d_fwd with 128-record batches instead of 256 on the camera set (c2 A/B,
# the 3DGS parity tests on the variant first).
set -o pipefail
HGSR_LIB=horizongs_amd/_lib_f128/libhgsr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_parity.py -k "3dgs or c2 or last_ids or pair_counter" \
  > gpurun_out/r05s39_tests.txt 2>&1 || { tail -20 gpurun_out/r05s39_tests.txt; exit 1; }
tail -1 gpurun_out/r05s39_tests.txt
TAG=r05s39/f128 LIB_B=horizongs_amd/_lib_f128/libhgsr.so CONFIGS="c2" REPS=3 bash scripts/gpu_r04_ab.sh
