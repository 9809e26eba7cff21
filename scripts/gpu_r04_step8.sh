# Round 4: PMC limiter counters of the two 2DGS backward kernels on c3 (per-step reduction vs
# transposed inputs), one pass each, plus WRITE_SIZE.
set -o pipefail
O=gpurun_out/r04s8
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing"
L="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
HGSR_BWD2_TP=1 timeout -k 10 300 rocprofv3 --pmc $L --kernel-include-regex "raster2d_bwd" -d $O/tp -o tp --output-format csv -- $B2 > $O/tp.log 2>&1 && \
HGSR_BWD2_TP=0 timeout -k 10 300 rocprofv3 --pmc $L --kernel-include-regex "raster2d_bwd" -d $O/st -o st --output-format csv -- $B2 > $O/st.log 2>&1 && \
HGSR_BWD2_TP=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "raster2d_bwd" -d $O/wtp -o wtp --output-format csv -- $B2 > $O/wtp.log 2>&1 && \
HGSR_BWD2_TP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s2 -o s2 --output-format csv -- $B2 > $O/s2.log 2>&1
st=$?
for d in tp st wtp; do echo == $d; python scripts/pmc_summary.py $O/$d; done
python scripts/stats_summary.py $O/s2/s2_kernel_stats.csv 13 | head -8
exit $st
