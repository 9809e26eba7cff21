# c2: per-step host times with a long warmup, and with a GPU pre-heat before the 5 warmup steps
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  HGSR_BENCH_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-secondary "$@" > gpurun_out/r03t2.json 2> gpurun_out/r03t2.err || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" gpurun_out/r03t2.json
  grep "step ms" gpurun_out/r03t2.err
}
for r in 1 2 3 4; do echo warmup5; run --warmup 5; done
echo gc-debug; HGSR_GC_DEBUG=1 run --warmup 5
