# Round 4: Gaussians per isect count / emit block (HGSR_ISECT_PER_BLOCK 4096 / 3072 against 2048):
# bit-exact isect tests at 4096, then interleaved c2 A/Bs.
set -o pipefail
O=gpurun_out/r04s17
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_ISECT_PER_BLOCK=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred.py -m gpu -v \
  -k "isect or deferred" --timeout 240 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s17/ab_4096 ENV_A="HGSR_ISECT_PER_BLOCK=2048" ENV_B="HGSR_ISECT_PER_BLOCK=4096" CONFIGS="c2 c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s17/ab_3072 ENV_A="HGSR_ISECT_PER_BLOCK=2048" ENV_B="HGSR_ISECT_PER_BLOCK=3072" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
