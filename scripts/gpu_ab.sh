# A/B of two builds of the library on the same box: bench.py with HGSR_LIB=A then B, twice.
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=${LIB_A:-horizongs_amd/_lib/libhgsr.so}
B=${LIB_B:-horizongs_amd/_lib_alt/libhgsr.so}
ARGS=${BENCH_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}
for r in 1 2; do
  HGSR_LIB=$A timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab/a$r.json 2>gpurun_out/ab/a$r.err || exit $?
  HGSR_LIB=$B timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab/b$r.json 2>gpurun_out/ab/b$r.err || exit $?
done
python - <<'PY'
import json
for n in ("a1", "b1", "a2", "b2"):
    d = json.loads(open(f"gpurun_out/ab/{n}.json").read().strip().splitlines()[-1])
    k = d["kernels"]
    print(n, d["value"], d["ms_per_step"], {x: k[x]["avg_ms"] for x in k if "raster" in x or x in ("tile_sort", "isect_emit")})
PY
