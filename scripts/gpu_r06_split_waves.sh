# Round 6: split3 at 5 (product, 96 VGPRs), 6 and 8 waves per SIMD (HGSR_SPLIT3_WAVES builds, a macro since removed; 22 / 88
# VGPRs spilled) -- kernel stats and the c2 line of each, interleaved on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06sw}; rm -rf $O; mkdir -p $O
B3="python bench.py --freeze --steps 16 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
for v in prod w6 w8 prod2 w62; do
  case $v in prod*) L=_lib;; w6*) L=_lib_split_w6;; w8*) L=_lib_split_w8;; esac
  HGSR_LIB=$GRAFT_REPO_ROOT/horizongs_amd/$L/libhgsr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o s --output-format csv -- $B3 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'split3' in n or 'raster3d_bwd' in n: print(sys.argv[2], n.split('(')[0][-40:], round(float(r['AverageNs'])/1e3,1))
" $O/$v/s_kernel_stats.csv $v
done
