# Round 4: the transposed-input 2DGS backward (HGSR_BWD2_TP=1): 2DGS parity tests on it, then an
# interleaved c3 A/B against the per-step reduction kernel.
set -o pipefail
O=gpurun_out/r04s6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_BWD2_TP=1 HGSR_PARITY_REPORT=$O/parity_strict.jsonl timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_parity_dense.py tests/test_gpu_glue.py tests/test_gpu_deferred.py -m gpu -v -k "2dgs or 2d" \
  --timeout 600 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -gt 1 ]; then exit $st; fi
TAG=r04s6/ab_tp ENV_A="HGSR_BWD2_TP=0" ENV_B="HGSR_BWD2_TP=1" CONFIGS="c3" bash scripts/gpu_r04_ab.sh || exit $?
