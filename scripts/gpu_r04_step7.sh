# Round 4: unroll variants of the transposed-input 2DGS backward (c3 A/Bs, HGSR_BWD2_TP=1 on
# both sides) and the 2DGS tests on the default build.
set -o pipefail
O=gpurun_out/r04s7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_BWD2_TP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "2dgs" \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -gt 1 ]; then exit $st; fi
TAG=r04s7/ab_u41 ENV_A="HGSR_BWD2_TP=1" ENV_B="HGSR_BWD2_TP=1" LIB_B=horizongs_amd/_lib_v41/libhgsr.so CONFIGS="c3" \
  bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s7/ab_u22 ENV_A="HGSR_BWD2_TP=1" ENV_B="HGSR_BWD2_TP=1" LIB_B=horizongs_amd/_lib_v22/libhgsr.so CONFIGS="c3" \
  bash scripts/gpu_r04_ab.sh || exit $?
