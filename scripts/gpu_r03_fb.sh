# 3DGS forward LDS-DMA with 128 / 64-record batches: raster parity on both, then c2 A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in f128 f64; do
  HGSR_LIB=horizongs_amd/_lib_$v/libhgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py -m gpu -x -q -k "not 2d and not 2D and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03q_$v.log 2>&1 || { tail -30 gpurun_out/r03q_$v.log; exit 1; }
  tail -1 gpurun_out/r03q_$v.log
done
LIBS="horizongs_amd/_lib horizongs_amd/_lib_f128 horizongs_amd/_lib_f64" timeout -k 10 600 bash scripts/gpu_libs.sh
