# end-of-round evidence: full GPU suite, smoke, the three bench lines, kernel stats + PMC traffic
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_round.sh > gpurun_out/round.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --anchors 500000 --no-cpu-baseline > gpurun_out/bench_anchors.json 2> gpurun_out/bench_anchors.err || exit 1
bash scripts/gpu_profiles.sh > gpurun_out/profiles.log 2>&1 || exit 1
tail -3 gpurun_out/tfull.log; tail -1 gpurun_out/smoke.log
python - <<'PY'
import json
for f in ("gpurun_out/bench3d.json", "gpurun_out/bench2d.json", "gpurun_out/bench_anchors.json"):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel_avg_ms"])
PY
