# SQ counters of the decode backward kernels (decode-inclusive bench)
set -o pipefail
rm -rf gpurun_out/pmcd && mkdir -p gpurun_out/pmcd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --anchors 500000 --steps 2 --warmup 1 --no-cpu-baseline --no-timing"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "decode_bwd" -d gpurun_out/pmcd/a -o a --output-format csv -- $B > gpurun_out/pmcd/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --kernel-include-regex "decode_bwd" -d gpurun_out/pmcd/b -o b --output-format csv -- $B > gpurun_out/pmcd/b.log 2>&1
st=$?
python scripts/pmc_summary.py gpurun_out/pmcd
exit $st
