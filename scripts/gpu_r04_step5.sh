# Round 4: decode backward per-anchor slot lanes (cov sums without LDS atomics) -- decode tests,
# then interleaved A/Bs against the previous build on c4 and c2-anchors.
set -o pipefail
O=gpurun_out/r04s5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_c4_chunk.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s5/ab LIB_A=horizongs_amd/_lib_base/libhgsr.so LIB_B=horizongs_amd/_lib/libhgsr.so CONFIGS="c4 c2-anchors" \
  bash scripts/gpu_r04_ab.sh || exit $?
