# Round 5, step 12: what the two workgroup barriers per batch cost raster3d_bwd -- a timing
# probe without them (HGSR_PROBE_NOBAR3: wrong results), on a frozen scene so both builds
# render the same views (c2 camera set and fixed camera, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s12
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_run_to_run.py \
  > gpurun_out/r05s12/run_to_run.log 2>&1 || { tail -30 gpurun_out/r05s12/run_to_run.log; exit 1; }
grep -h "^3d\|^2d" gpurun_out/r05s12/run_to_run.log
TAG=r05s12/probe_nobar LIB_B=horizongs_amd/_lib_nobar/libhgsr.so CONFIGS="c2 c2-fixed" REPS=2 BENCH_EXTRA=--freeze \
  bash scripts/gpu_r04_ab.sh || exit $?
