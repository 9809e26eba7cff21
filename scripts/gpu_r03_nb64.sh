# 2DGS forward with LDS-DMA staging: 2DGS parity tests on that build, then c3 A/B vs the kept build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=horizongs_amd/_lib_nb64/libhgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_normal.py -m gpu -x -q -k "2d or 2D" --timeout 300 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1 || { tail -30 gpurun_out/r03o_tests.log; exit 1; }
tail -2 gpurun_out/r03o_tests.log
LIBS="horizongs_amd/_lib horizongs_amd/_lib_nb64" BENCH_ARGS="--config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-secondary" timeout -k 10 600 bash scripts/gpu_libs.sh
