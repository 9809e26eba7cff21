# Round 6 probe: where split3's time goes (probe builds, wrong results, timing only):
# p1 no slot reduction, p2 no row loads, p3 no per-entry slot loop.
set -o pipefail
O=gpurun_out/${TAG:-r06probe}
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality --freeze"
for v in base p1 p2 p3; do
  L=horizongs_amd/_lib/libhgsr.so; [ $v != base ] && L=horizongs_amd/_lib_$v/libhgsr.so
  HGSR_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/$v -o $v --output-format csv -- $B3 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python scripts/stats_summary.py $O/$v/${v}_kernel_stats.csv 9 > $O/${v}_stats.txt 2>&1
  echo "$v $(grep split3 $O/${v}_stats.txt)"
done
