# bench alternative builds (build/<name>/libhgsr.so) back to back: raster kernel times
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  HGSR_LIB=$PWD/build/$v/libhgsr.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 ${BENCH_ARGS} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || exit 1
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/var_{sys.argv[1]}.json").read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[1], d["value"], {n: v["avg_ms"] for n, v in k.items() if "raster" in n or "loss" in n})
PY
done
