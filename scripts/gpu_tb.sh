set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/tb_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/tb_bench.log 2> gpurun_out/tb_bench.err
st=$?
tail -3 gpurun_out/tb_tests.log; cat gpurun_out/tb_bench.log; tail -3 gpurun_out/tb_bench.err
exit $st
