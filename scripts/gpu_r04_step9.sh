# Round 4: live-step queues -- the 2DGS transposed backward (default) and the 3DGS backward
# (HGSR_BWD3_Q=1): parity tests on both, then interleaved A/Bs (c3, c2).
set -o pipefail
O=gpurun_out/r04s9
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_glue.py \
  tests/test_gpu_deferred.py -m gpu -v -k "2dgs or 2d" --timeout 600 --timeout-method thread > $O/tests2.log 2>&1
st=$?
tail -n 2 $O/tests2.log; grep -E "^FAILED|Error:" $O/tests2.log | head
if [ $st -gt 1 ]; then exit $st; fi
HGSR_BWD3_Q=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py -m gpu -v \
  -k "3dgs or raster3d or rasterization or c1" --timeout 600 --timeout-method thread > $O/tests3.log 2>&1
st=$?
tail -n 2 $O/tests3.log; grep -E "^FAILED|Error:" $O/tests3.log | head
if [ $st -gt 1 ]; then exit $st; fi
TAG=r04s9/ab_tp ENV_A="HGSR_BWD2_TP=0" ENV_B="HGSR_BWD2_TP=1" CONFIGS="c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s9/ab_q ENV_A="HGSR_BWD3_Q=0" ENV_B="HGSR_BWD3_Q=1" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
