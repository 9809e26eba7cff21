# quick GPU iteration: raster parity + training parity + default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_training_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tquick.log 2>&1
st=$?
tail -3 gpurun_out/tquick.log
[ $st -ne 0 ] && exit $st
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bquick.log 2> gpurun_out/bquick.err
st=$?
cat gpurun_out/bquick.log; tail -3 gpurun_out/bquick.err
exit $st
