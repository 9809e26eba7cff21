# Round-3 diagnosis: PMC counters of the raster kernels under the reference and working builds,
# then the given tests on the reference build.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03d}
for K in raster3d_bwd raster3d_fwd; do
  KERNEL=$K LIB_A=horizongs_amd/_lib_ref/libhgsr.so LIB_B=horizongs_amd/_lib/libhgsr.so timeout -k 10 400 bash scripts/gpu_pmc_ab.sh > gpurun_out/${T}_pmc_$K.txt 2>&1 || exit $?
done
if [ -n "$REF_TESTS" ]; then
  HGSR_LIB=horizongs_amd/_lib_ref/libhgsr.so timeout -k 10 700 python -u -m pytest $REF_TESTS -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/${T}_reftests.log 2>&1
  st=$?; grep -E "passed|failed" gpurun_out/${T}_reftests.log | tail -2; exit $st
fi
