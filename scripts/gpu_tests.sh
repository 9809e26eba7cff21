# GPU test suite, smoke, then the default bench line (the driver's round-end command).
# Usage: TAG=r03a bash scripts/gpu_tests.sh   (outputs gpurun_out/$TAG_*)
set -o pipefail
TAG=${TAG:-r03}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s $PYTEST_ARGS --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
st=$?
grep -E "passed|failed|error" gpurun_out/${TAG}_gputests.log | tail -3
exit $st
