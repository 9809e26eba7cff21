# GPU test suite, smoke, then the default bench line (the driver's round-end command).
# Usage: TAG=r03a [TESTS="tests/x.py ..."] [KFILTER="not slow"] [PYTEST_ARGS=...] [BENCH_ARGS=...] [NO_BENCH=1] bash scripts/gpu_tests.sh
# Test FAILURES (pytest status 1) still go on to the smoke and the bench; a timeout, abort,
# crash or any other status ends the script there (nothing more touches the GPU).
set -o pipefail
TAG=${TAG:-r03}
TESTS=${TESTS:-tests}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KARG=()
if [ -n "$KFILTER" ]; then KARG=(-k "$KFILTER"); fi
timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -v -s $PYTEST_ARGS "${KARG[@]}" --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
st=$?
grep -E "passed|failed|error" gpurun_out/${TAG}_gputests.log | tail -3
if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "pytest status $st: stopping"; exit $st; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
if [ -n "$NO_BENCH" ]; then exit $st; fi
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
exit $st
