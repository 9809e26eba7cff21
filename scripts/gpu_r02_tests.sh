# Round-2: GPU test suite, smoke, then the default bench line (driver command).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s $PYTEST_ARGS --timeout 300 --timeout-method thread > gpurun_out/r02_gputests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err
st=$?
grep -E "passed|failed|error" gpurun_out/r02_gputests.log | tail -3
exit $st
