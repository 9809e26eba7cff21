# Round 5, step 40: latency counters of the raster kernels -- rocprofv3's derived VmemLatency /
# LdsLatency (accumulated in-flight levels / instructions, each in its own pass) and the LDS-issue
# wait, c2 (raster3d) and c3 (raster2d).  One --pmc pass per run, no other tracing.
set -o pipefail
O=gpurun_out/r05s40
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B2="python bench.py --gs 2d --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-timing --no-quality"
R() { local name=$1; shift; timeout -s KILL 150 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }; echo "$name ok"; }
R v3 --pmc VmemLatency --kernel-include-regex "raster3d" -d $O/v3 -o v3 --output-format csv -- $B3 && \
R l3 --pmc LdsLatency --kernel-include-regex "raster3d" -d $O/l3 -o l3 --output-format csv -- $B3 && \
R w3 --pmc SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --kernel-include-regex "raster3d" -d $O/w3 -o w3 --output-format csv -- $B3 && \
R v2 --pmc VmemLatency --kernel-include-regex "raster2d" -d $O/v2 -o v2 --output-format csv -- $B2 && \
R l2 --pmc LdsLatency --kernel-include-regex "raster2d" -d $O/l2 -o l2 --output-format csv -- $B2 && \
R w2 --pmc SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --kernel-include-regex "raster2d" -d $O/w2 -o w2 --output-format csv -- $B2
st=$?
for p in v3 l3 w3 v2 l2 w2; do [ -d $O/$p ] && python scripts/pmc_summary.py $O/$p > $O/$p.txt 2>&1; done
exit $st
