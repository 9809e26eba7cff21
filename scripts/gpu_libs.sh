# bench.py under several library builds, twice each, interleaved:
#   LIBS="horizongs_amd/_lib_ref horizongs_amd/_lib" bash scripts/gpu_libs.sh
set -o pipefail
mkdir -p gpurun_out/libs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${BENCH_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}
for r in 1 2; do
  n=0
  for L in $LIBS; do
    n=$((n+1))
    HGSR_LIB=$L/libhgsr.so timeout -k 10 300 python bench.py $ARGS > gpurun_out/libs/$n.$r.json 2>gpurun_out/libs/$n.$r.err || exit $?
  done
done
python - <<'PY'
import json, os
libs = os.environ["LIBS"].split()
for r in (1, 2):
    for n, L in enumerate(libs, 1):
        for l in open(f"gpurun_out/libs/{n}.{r}.json"):
            l = l.strip()
            if not l.startswith("{"):
                continue
            d = json.loads(l)
            k = d["kernels"]
            print(L.split("/")[-1], r, d["value"], d["ms_per_step"],
                  {x: k[x]["avg_ms"] for x in k if "raster" in x or x in ("decode_bwd",)})
            for s in d.get("secondary", []):
                k = s["kernels"]
                print("   sec", s["workload"][:14], s["value"], s["ms_per_step"], {x: k[x]["avg_ms"] for x in k if "raster" in x})
PY
