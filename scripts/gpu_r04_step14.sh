# Round 4: banded isect count / emit (HGSR_ISECT_BANDS: LDS holds one band of tile rows' counters /
# cursors, so more blocks fit a CU): bit-exact isect tests at 3 and 4 bands, then interleaved A/Bs.
set -o pipefail
O=gpurun_out/r04s14
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for nb in 3 4; do
  HGSR_ISECT_BANDS=$nb timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred.py -m gpu -v \
    -k "isect or deferred" --timeout 240 --timeout-method thread > $O/tests_b$nb.log 2>&1
  st=$?
  tail -n 2 $O/tests_b$nb.log; grep -E "^FAILED|Error:" $O/tests_b$nb.log | head
  if [ $st -ne 0 ]; then exit $st; fi
done
TAG=r04s14/ab_b4 ENV_A="HGSR_ISECT_BANDS=0" ENV_B="HGSR_ISECT_BANDS=4" CONFIGS="c2 c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s14/ab_b2 ENV_A="HGSR_ISECT_BANDS=0" ENV_B="HGSR_ISECT_BANDS=2" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s14/ab_b8 ENV_A="HGSR_ISECT_BANDS=0" ENV_B="HGSR_ISECT_BANDS=8" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
