# Round 5, step 14: the raster backwards' LDS transpose buffers (and the 2DGS pass-2 pixel table)
# re-laid out for CDNA4's per-instruction banking (the round-5 LDS counters counted 72M of
# raster3d_bwd's 161M and 173M of raster2d_bwd's 508M LDS cycles as bank conflicts).  Parity on
# the new build, then an interleaved A/B against the previous layout.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s14
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity_dense.py tests/test_gpu_parity.py \
  > gpurun_out/r05s14/tests.log 2>&1 || { tail -30 gpurun_out/r05s14/tests.log; exit 1; }
tail -1 gpurun_out/r05s14/tests.log
TAG=r05s14/ab_banks LIB_A=horizongs_amd/_lib_prev/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "raster3d_bwd" \
  -d gpurun_out/r05s14/d3 -o d3 --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing --no-quality \
  > gpurun_out/r05s14/d3.log 2>&1 && python scripts/pmc_summary.py gpurun_out/r05s14/d3
