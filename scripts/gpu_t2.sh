set -o pipefail
mkdir -p gpurun_out
true && \
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "not fullsize" > gpurun_out/t2.log 2>&1
st=$?
cat gpurun_out/diag.log; tail -15 gpurun_out/t2.log
exit $st
