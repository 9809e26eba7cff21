# Round-2 evidence pass: step timeline (gap analysis) + VALU / MFMA counters of the
# dominant kernels.  Each rocprofv3 call is its own pass; --pmc never combined with tracing.
set -o pipefail
OUT=gpurun_out/r02prof
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-timing"
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-timing"
BA="python bench.py --anchors 500000 --steps 10 --warmup 3 --no-cpu-baseline --no-timing"
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 -L > $OUT/counters.txt 2>&1 ; \
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t3 -o t3 --output-format csv -- $B3 > $OUT/t3.log 2>&1 && \
python scripts/trace_step.py $OUT/t3/t3_kernel_trace.csv project3d_fwd > $OUT/t3_step.txt && \
rm -f $OUT/t3/t3_kernel_trace.csv && \
timeout -k 10 300 rocprofv3 --pmc $V --kernel-include-regex "raster3d|tile_sort|isect_emit" -d $OUT/v3 -o v3 --output-format csv -- $B3 > $OUT/v3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $V --kernel-include-regex "raster2d" -d $OUT/v2 -o v2 --output-format csv -- $B2 > $OUT/v2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "decode" -d $OUT/m -o m --output-format csv -- $BA > $OUT/m.log 2>&1
st=$?
python scripts/pmc_summary.py $OUT > $OUT/pmc.txt 2>&1
exit $st
