# SQ counters of the raster kernels for alternative builds (build/<name>/libhgsr.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing ${BENCH_ARGS}"
for v in ${VARIANTS}; do
  rm -rf gpurun_out/pmcv_$v; mkdir -p gpurun_out/pmcv_$v
  export HGSR_LIB=$PWD/build/$v/libhgsr.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "${KRE:-raster3d}" -d gpurun_out/pmcv_$v/a -o a --output-format csv -- $B > gpurun_out/pmcv_$v/a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --kernel-include-regex "${KRE:-raster3d}" -d gpurun_out/pmcv_$v/b -o b --output-format csv -- $B > gpurun_out/pmcv_$v/b.log 2>&1 || exit 1
  echo "== $v"; python scripts/pmc_summary.py gpurun_out/pmcv_$v
done
