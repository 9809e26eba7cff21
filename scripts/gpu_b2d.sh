set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gs 2d --no-cpu-baseline > gpurun_out/b2d.log 2> gpurun_out/b2d.err
st=$?
cat gpurun_out/b2d.log; tail -3 gpurun_out/b2d.err
exit $st
