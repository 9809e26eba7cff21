# rocprofv3 kernel stats (rocpd database -> scripts/rocpd_stats.py) of single bench configs,
# plus the torch-glue attribution of each; every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/prof_r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03f}
for c in ${CONFIGS:-c3 c2-anchors}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03/$c -o run -- python3 bench.py --config $c --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_rocprof_$c.log 2>&1 || exit $?
  python3 scripts/rocpd_stats.py gpurun_out/prof_r03/$c/run_results.db > gpurun_out/${T}_stats_$c.csv || exit $?
  timeout -k 10 200 python scripts/glue_ops.py --config $c > gpurun_out/${T}_glue_$c.txt 2>&1 || exit $?
done
echo done
