# PMC of one kernel under two library builds (LIB_A / LIB_B), one pass per counter set.
#   KERNEL=raster3d_bwd LIB_B=horizongs_amd/_lib_exp/libhgsr.so bash scripts/gpu_pmc_ab.sh
set -o pipefail
OUT=gpurun_out/pmcab
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=${LIB_A:-horizongs_amd/_lib/libhgsr.so}
B=${LIB_B:-horizongs_amd/_lib/libhgsr.so}
K=${KERNEL:-raster3d_bwd}
V1=${COUNTERS:-"SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"}
for v in a b; do
  L=$A; [ $v = b ] && L=$B
  HGSR_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $V1 --kernel-include-regex "$K" -d $OUT/$v -o p --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing > $OUT/$v.log 2>&1 || exit $?
done
for v in a b; do echo "== $v"; python scripts/pmc_summary.py $OUT/$v; done
