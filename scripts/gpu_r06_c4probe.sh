# Round 6: why c4 alone (32 steps) runs slower per step than c4 as a secondary line (16 steps
# after the other configs) -- host step times of both shapes, then c4's kernel list.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06c4p}; rm -rf $O; mkdir -p $O
for sw in "32 5" "16 3" "64 5"; do
  set -- $sw
  HGSR_BENCH_STEP_TIMES=1 timeout -k 10 200 python -u bench.py --config c4 --steps $1 --warmup $2 --no-cpu-baseline --no-quality --no-secondary > $O/c4_$1.json 2> $O/c4_$1.err || { tail -20 $O/c4_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('isects_before'), d.get('isects_after'))" $O/c4_$1.json $1
  grep "step ms" $O/c4_$1.err | cut -c1-600
done
B4="python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s4 -o s4 --output-format csv -- $B4 > $O/s4.log 2>&1 || { tail -20 $O/s4.log; exit 1; }
python scripts/stats_summary.py $O/s4/s4_kernel_stats.csv 13 > $O/s4_stats.txt 2>&1
grep -E "total|torch|Cijk|rocclr" $O/s4_stats.txt
