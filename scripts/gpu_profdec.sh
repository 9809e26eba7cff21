set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/profdec
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profdec -o run --output-format csv -- python bench.py --anchors 500000 --steps 5 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/profdec.log 2>&1
st=$?
python scripts/stats_summary.py gpurun_out/profdec/run_kernel_stats.csv 7
exit $st
