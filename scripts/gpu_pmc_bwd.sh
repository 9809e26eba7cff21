# PMC of raster3d_bwd under both variants (q4 default vs HGSR_BWD3=quad8)
set -o pipefail
OUT=gpurun_out/pmcb
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing"
V1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
for v in q4 quad8; do
  HGSR_BWD3=$v timeout -s KILL 120 rocprofv3 --pmc $V1 --kernel-include-regex "raster3d_bwd" -d $OUT/$v -o p --output-format csv -- $B > $OUT/$v.log 2>&1 || exit $?
done
for v in q4 quad8; do echo "== $v"; python scripts/pmc_summary.py $OUT/$v; done
