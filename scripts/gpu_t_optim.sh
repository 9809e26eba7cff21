# optimizer + training parity tests, default bench and the decode-inclusive bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_training_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/topt.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b3.json 2> gpurun_out/b3.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --anchors 500000 > gpurun_out/ba.json 2> gpurun_out/ba.err
st=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/topt.log | tail -12; cat gpurun_out/b3.json gpurun_out/ba.json; tail -3 gpurun_out/b3.err gpurun_out/ba.err
exit $st
