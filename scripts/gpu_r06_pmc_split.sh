# Round 6: PMC counters of the split (gradient-slot reduction) kernels, c2 and c3.
set -o pipefail
O=gpurun_out/${TAG:-r06pmcs}
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B2="python bench.py --gs 2d --steps 6 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
K="split|raster3d_bwd|raster2d_bwd"
L="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM"
R() { local name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; echo "$name ok"; }
R l3 --pmc $L --kernel-include-regex "$K" -d $O/l3 -o l3 --output-format csv -- $B3 && \
R f3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/f3 -o f3 --output-format csv -- $B3 && \
R w3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/w3 -o w3 --output-format csv -- $B3 && \
R l2 --pmc $L --kernel-include-regex "$K" -d $O/l2 -o l2 --output-format csv -- $B2
st=$?
for n in l3 f3 w3 l2; do python scripts/pmc_summary.py $O/$n > $O/$n.txt 2>&1; done
exit $st
