# isect_emit band count sweep: PMC WRITE_SIZE (with kernel durations) per HGSR_EMIT_PHASES value.
set -o pipefail
mkdir -p gpurun_out/emit
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for P in ${PHASES:-4 8 16 32}; do
  HGSR_EMIT_PHASES=$P timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "isect_emit|tile_sort" -d gpurun_out/emit/p$P -o run --output-format csv -- python3 bench.py --config ${CONFIG:-c2} --no-secondary --no-cpu-baseline --no-timing --steps 5 --warmup 2 > gpurun_out/emit/p$P.log 2>&1 || exit $?
  python3 - "$P" <<'PY' || exit $?
import csv, glob, sys, collections
P = sys.argv[1]
w = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/emit/p{P}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        w[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024)
t = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/emit/p{P}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        t[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in w:
    tt = t.get(k, [0])
    print(f"phases {P:>3s} {k[:30]:30s} WRITE_SIZE {sum(w[k]) / len(w[k]) / 1e6:8.1f} MB  {sum(tt) / len(tt):7.1f} us (n={len(tt)})")
PY
done
