# emit phase sweep: bench kernels + PMC WRITE_SIZE of isect_emit for each HGSR_EMIT_PHASES
set -o pipefail
mkdir -p gpurun_out/ph
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"
for p in ${PHASES:-1 2 4 8}; do
  HGSR_EMIT_PHASES=$p timeout -k 10 300 $B > gpurun_out/ph/b$p.json 2>/dev/null || exit $?
  HGSR_EMIT_PHASES=$p timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "isect_emit|tile_sort" -d gpurun_out/ph/w$p -o w --output-format csv -- $B --no-timing > gpurun_out/ph/w$p.log 2>&1 || exit $?
done
python - <<'PY'
import json, csv, glob
import os
for p in [int(x) for x in os.environ.get("PHASES", "1 2 4 8").split()]:
    d = json.loads(open(f"gpurun_out/ph/b{p}.json").read().strip().splitlines()[-1])
    k = d["kernels"]
    ws = {}
    for f in glob.glob(f"gpurun_out/ph/w{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].split("(")[0].split("::")[-1]
            ws.setdefault(n, []).append(float(r["Counter_Value"]))
    print(p, d["ms_per_step"], k["isect_emit"]["avg_ms"], k["tile_sort"]["avg_ms"], {n: round(sum(v)/len(v)/1e3, 1) for n, v in ws.items()})
PY
