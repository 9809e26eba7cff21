# 3DGS forward with LDS-DMA staging: 3DGS raster parity on that build, then c2 A/B vs the kept build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=horizongs_amd/_lib_dma/libhgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py -m gpu -x -q -k "not 2d and not 2D and not slow" --timeout 300 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1 || { tail -30 gpurun_out/r03n_tests.log; exit 1; }
tail -2 gpurun_out/r03n_tests.log
LIBS="horizongs_amd/_lib horizongs_amd/_lib_dma" timeout -k 10 600 bash scripts/gpu_libs.sh
