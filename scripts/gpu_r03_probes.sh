# rocprofv3 kernel durations of one bench config (CONFIG, default c2) under several library
# builds (LIBS), one profiled run each; prints the average duration of the kernels matching KPAT.
set -o pipefail
mkdir -p gpurun_out/probes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=${CONFIG:-c2}
for L in $LIBS; do
  n=$(basename $L)_$C
  HGSR_LIB=$L/libhgsr.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/probes/$n -o run -- python3 bench.py --config $C --no-secondary --no-cpu-baseline --no-timing --steps 10 --warmup 3 > gpurun_out/probes/$n.log 2>&1 || exit $?
  python3 scripts/rocpd_stats.py gpurun_out/probes/$n/run_results.db > gpurun_out/probes/$n.csv || exit $?
  python3 - "$n" "${KPAT:-raster3d_bwd|raster3d_fwd}" <<'PY' || exit $?
import csv, re, sys
n, pat = sys.argv[1], re.compile(sys.argv[2])
for r in csv.DictReader(open(f"gpurun_out/probes/{n}.csv")):
    if pat.search(r["Name"]):
        print(f"{n:28s} {float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>4s}  {r['Name'][:70]}")
PY
done
