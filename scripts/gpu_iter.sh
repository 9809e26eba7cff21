# Iteration helper: a subset of the GPU tests (-k $TESTS), then bench A/B of library builds ($LIBS).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -k "$TESTS" -x -v --timeout 200 --timeout-method thread > gpurun_out/titer.log 2>&1
st=$?; grep -E "passed|failed|FAILED|Error|error" gpurun_out/titer.log | tail -12; [ $st -eq 0 ] || exit $st
[ -z "$LIBS" ] || timeout -k 10 600 bash scripts/gpu_libs.sh
