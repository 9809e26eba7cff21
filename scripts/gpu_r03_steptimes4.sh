# c2: per-step host times after moving gc.collect / timing setup before the warmup
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3 4; do
  HGSR_BENCH_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r03t4_$r.json 2> gpurun_out/r03t4_$r.err || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" gpurun_out/r03t4_$r.json
  grep "step ms" gpurun_out/r03t4_$r.err | cut -c1-140
done
