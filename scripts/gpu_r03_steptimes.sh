# c2 bench six times with per-step host times (where do the slow runs lose their time?)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3 4 5 6; do
  HGSR_BENCH_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r03t_$r.json 2> gpurun_out/r03t_$r.err || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(d['value'], d['ms_per_step'])" gpurun_out/r03t_$r.json
  grep "step ms" gpurun_out/r03t_$r.err
done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))"
