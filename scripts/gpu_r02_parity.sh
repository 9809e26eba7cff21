# raster parity tests only (iteration helper)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_normal.py} -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02_parity.log 2>&1
st=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || st=$?
exit $st
