# Round 6: the big-entry threshold of the slot reduction (HGSR_BIG_SLOTS 32 = product, 64, 128
# builds): split / pieces kernel times at c2 and c3, interleaved on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06bs}; rm -rf $O; mkdir -p $O
for gs in 3d 2d; do
for v in prod b64 b128 prod2; do
  case $v in prod*) L=_lib;; b64) L=_lib_big64;; b128) L=_lib_big128;; esac
  HGSR_LIB=$GRAFT_REPO_ROOT/horizongs_amd/$L/libhgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${gs}_$v -o s --output-format csv -- python bench.py --gs $gs --freeze --steps 16 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality > $O/${gs}_$v.log 2>&1 || { tail -20 $O/${gs}_$v.log; exit 1; }
  python3 -c "
import csv,sys
tot=0; sel=[]
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']; t=float(r['TotalDurationNs'])
    if any(k in n for k in ('split3','split2','reduce_pieces','slot_write')): sel.append((n.split('(')[0][-32:], round(float(r['AverageNs'])/1e3,1)))
print(sys.argv[2], sel)
" $O/${gs}_$v/s_kernel_stats.csv ${gs}_$v
done
done
