set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-timing $BENCH_ARGS > gpurun_out/prof.log 2>&1
st=$?
python scripts/stats_summary.py gpurun_out/prof/run_kernel_stats.csv 13 > gpurun_out/prof_stats.txt
python scripts/trace_step.py gpurun_out/prof/run_kernel_trace.csv ${MARKER:-project3d_fwd} > gpurun_out/prof_step.txt
rm -f gpurun_out/prof/run_kernel_trace.csv
exit $st
