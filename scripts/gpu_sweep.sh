# Sweep one environment variable over values on one box: bench.py per value, twice, interleaved.
#   VAR=HGSR_TILE_MAP VALUES="0 1 2" bash scripts/gpu_sweep.sh
set -o pipefail
mkdir -p gpurun_out/sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${BENCH_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}
for r in 1 2; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/sweep/$v.$r.json 2>gpurun_out/sweep/$v.$r.err || exit $?
  done
done
python - <<'PY'
import json, os
for v in os.environ["VALUES"].split():
    for r in (1, 2):
        out = []
        for l in open(f"gpurun_out/sweep/{v}.{r}.json"):
            l = l.strip()
            if l.startswith("{"):
                d = json.loads(l)
                out.append(d)
        for d in out:
            k = d["kernels"]
            print(v, r, d.get("config", {}).get("workload", "")[:12], d["value"], d["ms_per_step"],
                  {x: k[x]["avg_ms"] for x in k if "raster" in x or x in ("tile_sort", "isect_emit", "decode_bwd")})
            for s in d.get("secondary", []):
                k = s["kernels"]
                print("   sec", s["workload"][:14], s["value"], s["ms_per_step"],
                      {x: k[x]["avg_ms"] for x in k if "raster" in x})
PY
