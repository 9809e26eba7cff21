# Round 4: what bounds isect_emit -- rocprofv3 kernel stats of projection + isect on c2 under the
# normal build and two probe builds (-DHGSR_PROBE_EMIT=1: cursor atomics without key stores; =2: key
# stores to the slice start without atomics).  Probe outputs are wrong by construction; no raster runs.
set -o pipefail
O=gpurun_out/r04s15
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base probe1 probe2; do
  case $v in base) L=horizongs_amd/_lib/libhgsr.so;; probe1) L=horizongs_amd/_lib_probe1/libhgsr.so;;
              probe2) L=horizongs_amd/_lib_probe2/libhgsr.so;; esac
  HGSR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/isect_probe.py \
    > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("isect", "tile_sort")):
        print("%8.1f us  %s" % (float(r["AverageNs"]) / 1e3, r["Name"][:60]))
PY
done
