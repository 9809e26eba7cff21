# c2: per-step host times with and without the live kernel timing (events + pair counters)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  HGSR_BENCH_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary "$@" > gpurun_out/r03t3.json 2> gpurun_out/r03t3.err || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(d['value'], d['ms_per_step'])" gpurun_out/r03t3.json
  grep "step ms" gpurun_out/r03t3.err | cut -c1-140
}
for r in 1 2 3; do echo timing; run; echo no-timing; run --no-timing; done
