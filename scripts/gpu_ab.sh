# A/B on one box: bench.py under two environments (ENV_A / ENV_B, e.g. HGSR_BWD3=quad8) or
# two library builds (LIB_A / LIB_B), each twice, interleaved.
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=${LIB_A:-horizongs_amd/_lib/libhgsr.so}
B=${LIB_B:-horizongs_amd/_lib/libhgsr.so}
ARGS=${BENCH_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}
for r in 1 2; do
  env HGSR_LIB=$A $ENV_A timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab/a$r.json 2>gpurun_out/ab/a$r.err || exit $?
  env HGSR_LIB=$B $ENV_B timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab/b$r.json 2>gpurun_out/ab/b$r.err || exit $?
done
python - <<'PY'
import json
for n in ("a1", "b1", "a2", "b2"):
    d = json.loads(open(f"gpurun_out/ab/{n}.json").read().strip().splitlines()[-1])
    k = d["kernels"]
    r = d.get("roofline") or {}
    print(n, d["value"], d["ms_per_step"], {x: k[x]["avg_ms"] for x in k if "raster" in x or x in ("tile_sort", "isect_emit")},
          {x: r.get(x) for x in ("frac", "frac_executed", "executed_pairs_per_launch")})
PY
