# rocprofv3 kernel stats of bench.py under each library build in $LIBS (one short run each).
set -o pipefail
mkdir -p gpurun_out/profab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-timing}
n=0
for L in $LIBS; do
  n=$((n+1))
  HGSR_LIB=$L/libhgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profab/$n -o run --output-format csv -- python bench.py $ARGS > gpurun_out/profab/$n.log 2>&1 || exit 1
done
python - <<'PY'
import csv, glob, os
libs = os.environ["LIBS"].split()
for n, L in enumerate(libs, 1):
    f = glob.glob(f"gpurun_out/profab/{n}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    print("==", L)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
