# kernel stats of the decode-inclusive bench (per decode head)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pd
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pd -o pd --output-format csv -- python bench.py --anchors 500000 --steps 10 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/pd.log 2>&1
st=$?
python scripts/stats_summary.py gpurun_out/pd/pd_kernel_stats.csv 13 > gpurun_out/pd_stats.txt
rm -f gpurun_out/pd/pd_kernel_trace.csv
cat gpurun_out/pd_stats.txt | head -40
exit $st
