# SQ + memory counters for the kernels matching $KRE (separate passes; no trace domains)
set -o pipefail
rm -rf gpurun_out/pmc2
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing $BENCH_ARGS"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${KRE}" -d gpurun_out/pmc2/p$i -o p$i --output-format csv -- $B > gpurun_out/pmc2/p$i.log 2>&1 || exit 1
done
python scripts/pmc_summary.py gpurun_out/pmc2
