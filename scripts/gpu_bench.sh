set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/prof.log 2>&1
st=$?
cat gpurun_out/bench.log; tail -5 gpurun_out/bench.err
exit $st
