set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --anchors 500000 --no-cpu-baseline > gpurun_out/bdec.log 2> gpurun_out/bdec.err
st=$?
cat gpurun_out/bdec.log; tail -3 gpurun_out/bdec.err
exit $st
