set -o pipefail
mkdir -p gpurun_out
rocminfo | grep -m3 -E "gfx|Marketing" > gpurun_out/rocminfo.txt || true
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "not fullsize" > gpurun_out/t1.log 2>&1
st=$?
tail -30 gpurun_out/t1.log
exit $st
