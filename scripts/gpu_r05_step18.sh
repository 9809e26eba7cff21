# Round 5, step 18: the trimmed-range backward tile order now in both backwards (default build)
# -- parity, an interleaved A/B against the whole-bin order (c3, c2), then the per-workgroup
# timing probe of the 3DGS raster kernels (scripts/wg_time.py, probe build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s18
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity_dense.py tests/test_gpu_parity.py tests/test_gpu_deferred.py > gpurun_out/r05s18/tests.log 2>&1 \
  || { tail -30 gpurun_out/r05s18/tests.log; exit 1; }
tail -1 gpurun_out/r05s18/tests.log
TAG=r05s18/ab_bo LIB_A=horizongs_amd/_lib_nobo/libhgsr.so CONFIGS="c3 c2" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
HGSR_LIB=horizongs_amd/_lib_wgt/libhgsr.so timeout -k 10 300 python scripts/wg_time.py > gpurun_out/r05s18/wg_time.jsonl 2>&1 \
  || { tail -20 gpurun_out/r05s18/wg_time.jsonl; exit 1; }
cat gpurun_out/r05s18/wg_time.jsonl
