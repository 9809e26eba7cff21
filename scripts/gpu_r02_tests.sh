# Round-2: GPU test suite (incl. the dense / full-size raster parity tests), then the
# default bench line and a --no-timing A/B of the same step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s $PYTEST_ARGS --timeout 300 --timeout-method thread > gpurun_out/r02_gputests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err && \
timeout -k 10 300 python bench.py --no-timing --no-cpu-baseline > gpurun_out/r02_bench_notiming.json 2>&1
st=$?
grep -E "passed|failed|error" gpurun_out/r02_gputests.log | tail -3
exit $st
