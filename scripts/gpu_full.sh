set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu > gpurun_out/tfull.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
st=$?
tail -5 gpurun_out/tfull.log; cat gpurun_out/smoke.log | tail -3
exit $st
