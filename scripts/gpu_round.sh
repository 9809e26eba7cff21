# Round check: GPU parity suite, smoke, default bench line (with CPU baseline), 2DGS bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tfull.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench3d.json 2> gpurun_out/bench3d.err && \
timeout -k 10 300 python bench.py --gs 2d --no-cpu-baseline > gpurun_out/bench2d.json 2> gpurun_out/bench2d.err
st=$?
tail -5 gpurun_out/tfull.log; tail -2 gpurun_out/smoke.log; cat gpurun_out/bench3d.json gpurun_out/bench2d.json
exit $st
