set -o pipefail
rm -rf gpurun_out/pmc1
mkdir -p gpurun_out/pmc1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "${KRE:-raster3d}" -d gpurun_out/pmc1/a -o a --output-format csv -- $B > gpurun_out/pmc1/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --kernel-include-regex "${KRE:-raster3d}" -d gpurun_out/pmc1/b -o b --output-format csv -- $B > gpurun_out/pmc1/b.log 2>&1
true
