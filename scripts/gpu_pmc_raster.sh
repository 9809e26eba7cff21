# Issue / wait breakdown of the raster kernels: counter list + two SQ passes per config.
# Each rocprofv3 call is its own pass; --pmc never combined with tracing.
set -o pipefail
OUT=gpurun_out/pmcr
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing"
B2="python bench.py --gs 2d --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing"
P1=${P1:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH"}
P2=${P2:-"SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"}
K=${KERNELS:-"raster3d|raster2d"}
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 ; \
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex "$K" -d $OUT/a3 -o p --output-format csv -- $B3 > $OUT/a3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex "$K" -d $OUT/b3 -o p --output-format csv -- $B3 > $OUT/b3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex "$K" -d $OUT/a2 -o p --output-format csv -- $B2 > $OUT/a2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex "$K" -d $OUT/b2 -o p --output-format csv -- $B2 > $OUT/b2.log 2>&1
st=$?
for v in a3 b3 a2 b2; do echo "== $v"; python scripts/pmc_summary.py $OUT/$v; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
exit $st
