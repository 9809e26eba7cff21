# Round 6 evidence of the benched tree (as scripts/gpu_r05_prof.sh; the gradient-slot kernels in the traffic passes): kernel-trace stats (c2, c3, c4), FETCH_SIZE / WRITE_SIZE
# passes (c2, c3), the raster backwards' limiter counters and the decode MFMA-busy counter (c4).
# Each rocprofv3 call is its own pass; --pmc is never combined with other tracing; per-pass
# counter counts stay within the block limits (<= 8 SQ, <= 4 TCC, <= 2 GRBM).
set -o pipefail
O=gpurun_out/${TAG:-r06prof}
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B4="python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
K="raster3d|raster2d|tile_sort|isect|slot|reduce_pieces|project|pack|split|adam|loss|normal|rotate|activate|sh_"
L="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
D="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
R() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; echo "$name ok"; }
R s3 --kernel-trace --stats -d $O/s3 -o s3 --output-format csv -- $B3 && \
R s2 --kernel-trace --stats -d $O/s2 -o s2 --output-format csv -- $B2 && \
R s4 --kernel-trace --stats -d $O/s4 -o s4 --output-format csv -- $B4 && \
R f3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/f3 -o f3 --output-format csv -- $B3 && \
R w3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/w3 -o w3 --output-format csv -- $B3 && \
R f2 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/f2 -o f2 --output-format csv -- $B2 && \
R w2 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/w2 -o w2 --output-format csv -- $B2 && \
R l3 --pmc $L --kernel-include-regex "raster3d_bwd" -d $O/l3 -o l3 --output-format csv -- $B3 && \
R l2 --pmc $L --kernel-include-regex "raster2d_bwd" -d $O/l2 -o l2 --output-format csv -- $B2 && \
R m4 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "decode" \
  -d $O/m4 -o m4 --output-format csv -- $B4 && \
R d3 --pmc $D --kernel-include-regex "raster3d" -d $O/d3 -o d3 --output-format csv -- $B3 && \
R d2 --pmc $D --kernel-include-regex "raster2d" -d $O/d2 -o d2 --output-format csv -- $B2
st=$?
python scripts/stats_summary.py $O/s3/s3_kernel_stats.csv 13 > $O/s3_stats.txt 2>&1
python scripts/stats_summary.py $O/s2/s2_kernel_stats.csv 13 > $O/s2_stats.txt 2>&1
python scripts/stats_summary.py $O/s4/s4_kernel_stats.csv 13 > $O/s4_stats.txt 2>&1
python scripts/pmc_summary.py $O/l3 > $O/l3.txt 2>&1
python scripts/pmc_summary.py $O/l2 > $O/l2.txt 2>&1
python scripts/pmc_summary.py $O/m4 > $O/m4.txt 2>&1
python scripts/pmc_summary.py $O/d3 > $O/d3.txt 2>&1
python scripts/pmc_summary.py $O/d2 > $O/d2.txt 2>&1
exit $st
