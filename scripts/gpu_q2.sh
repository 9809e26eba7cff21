# raster parity (3D + 2D) + both default bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_training_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tquick.log 2>&1
st=$?
tail -3 gpurun_out/tquick.log
[ $st -ne 0 ] && exit $st
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b3.json 2> gpurun_out/b3.err && \
timeout -k 10 300 python bench.py --gs 2d --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b2.json 2> gpurun_out/b2.err
st=$?
python - <<'PY'
import json
for f in ("gpurun_out/b3.json", "gpurun_out/b2.json"):
    try:
        d = json.load(open(f))
        print(f, d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items()})
    except Exception as e:
        print(f, "ERR", e)
PY
exit $st
