# Raster kernel A/B: bench.py under LIBS (each twice, interleaved), plus optional parity subset
# on the working build first (TESTS / KFILTER).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03e}
if [ -n "$KFILTER" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v -s -k "$KFILTER" --timeout 400 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1
  st=$?; grep -E "passed|failed" gpurun_out/${T}_gputests.log | tail -2
  if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
fi
timeout -k 10 900 bash scripts/gpu_libs.sh > gpurun_out/${T}_ab.txt 2>&1 || exit $?
tail -12 gpurun_out/${T}_ab.txt
