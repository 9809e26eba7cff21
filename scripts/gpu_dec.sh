# decode parity tests + phase profile (variant build) + decode-inclusive bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_densify.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tdec.log 2>&1
st=$?
tail -3 gpurun_out/tdec.log
[ $st -ne 0 ] && exit $st
HGSR_LIB=$PWD/build/dprof/libhgsr.so timeout -k 10 300 python scripts/decode_prof.py > gpurun_out/dprof.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --anchors 500000 > gpurun_out/ba.json 2> gpurun_out/ba.err
st=$?
cat gpurun_out/dprof.txt | tail -3
python - <<'PY'
import json
d = json.load(open("gpurun_out/ba.json"))
print(d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
exit $st
