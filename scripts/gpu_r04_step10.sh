# Round 4: decode colour-forward stores through an LDS transpose -- decode tests, c4 A/B against
# HEAD's build.
set -o pipefail
O=gpurun_out/r04s10
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_c4_chunk.py tests/test_gpu_explicit.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s10/ab LIB_A=horizongs_amd/_lib_base/libhgsr.so LIB_B=horizongs_amd/_lib/libhgsr.so CONFIGS="c4 c2-anchors" \
  bash scripts/gpu_r04_ab.sh || exit $?
