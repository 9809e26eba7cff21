# Effective clock and activity of the raster kernels under two builds (GRBM_GUI_ACTIVE / 8 / time).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03j}
for K in raster3d_bwd raster3d_fwd; do
  COUNTERS="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" KERNEL=$K LIB_A=horizongs_amd/_lib_ref/libhgsr.so LIB_B=horizongs_amd/_lib_nodma/libhgsr.so timeout -k 10 400 bash scripts/gpu_pmc_ab.sh > gpurun_out/${T}_pmc_$K.txt 2>&1 || exit $?
  cp gpurun_out/pmcab/a/p_kernel_trace.csv gpurun_out/${T}_trace_a_$K.csv 2>/dev/null
  cp gpurun_out/pmcab/b/p_kernel_trace.csv gpurun_out/${T}_trace_b_$K.csv 2>/dev/null
done
echo done
