# Round 4: isect_emit without LDS atomics for single-key (block, bin) slices (HGSR_EMIT_SINGLE) and
# the Gaussians-per-block knob (HGSR_ISECT_PER_BLOCK): bit-exact isect tests, then interleaved A/Bs.
# (The three variants were measured slower and removed from isect.hip; this script is the record.)
set -o pipefail
O=gpurun_out/r04s13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred.py -m gpu -v \
  -k "isect or deferred" --timeout 240 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
HGSR_ISECT_PER_BLOCK=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v \
  -k "isect" --timeout 240 --timeout-method thread > $O/tests_pb1024.log 2>&1
st=$?
tail -n 2 $O/tests_pb1024.log; grep -E "^FAILED|Error:" $O/tests_pb1024.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s13/ab_single ENV_A="HGSR_EMIT_SINGLE=0" ENV_B="HGSR_EMIT_SINGLE=1" CONFIGS="c2 c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s13/ab_pb ENV_A="HGSR_ISECT_PER_BLOCK=2048" ENV_B="HGSR_ISECT_PER_BLOCK=1024" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
HGSR_ISECT_GLOBAL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v \
  -k "isect" --timeout 240 --timeout-method thread > $O/tests_global.log 2>&1
st=$?
tail -n 2 $O/tests_global.log; grep -E "^FAILED|Error:" $O/tests_global.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s13/ab_global ENV_A="HGSR_ISECT_GLOBAL=0" ENV_B="HGSR_ISECT_GLOBAL=1" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
