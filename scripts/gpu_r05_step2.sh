# Round 5, step 2: the deferred-count / glue tests after the running-max capacity and the knob
# removal, the 2DGS parity tests after deleting the per-step backward, and the camera-set bench.
set -o pipefail
O=gpurun_out/r05s2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_chunks.py tests/test_gpu_decode.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1
st=$?; tail -3 $O/tests.log; if [ $st -ne 0 ]; then grep -E "FAIL|Error" $O/tests.log | head -20; exit $st; fi
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05s2/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["config"]["cameras"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])
for s in d["secondary"]:
    print(s["config"], s["value"], s["ms_per_step"], s["cameras"])
PY
