# Round 6: kernel-trace stats of the c2 and c3 bench lines (which kernels the step spends on).
set -o pipefail
O=gpurun_out/${TAG:-r06pq}
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
R() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; echo "$name ok"; }
R s3 --kernel-trace --stats -d $O/s3 -o s3 --output-format csv -- $B3 && \
R s2 --kernel-trace --stats -d $O/s2 -o s2 --output-format csv -- $B2
st=$?
python scripts/stats_summary.py $O/s3/s3_kernel_stats.csv 13 > $O/s3_stats.txt 2>&1
python scripts/stats_summary.py $O/s2/s2_kernel_stats.csv 13 > $O/s2_stats.txt 2>&1
exit $st
