# Round 4, first GPU pass: MFMA/VALU micro, the new tests, the MFMA-backward parity subset, then
# interleaved A/Bs (MFMA pass 2 of the 3DGS / 2DGS backward).  Stops at the first failing GPU step.
set -o pipefail
mkdir -p gpurun_out/r04s1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s1
timeout -k 5 60 scripts/micro/mfma_valu > $O/mfma_valu.txt 2>&1 || exit $?
cat $O/mfma_valu.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_parity.py \
  tests/test_gpu_normal.py tests/test_gpu_decode.py -m gpu -x -q --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
HGSR_BWD3_MFMA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_dense.py tests/test_gpu_parity.py -m gpu -x -q \
  -k "3dgs and not c2 or raster3d or rasterization" --timeout 240 --timeout-method thread > $O/tests_mfma.log 2>&1 \
  || { tail -60 $O/tests_mfma.log; exit 1; }
tail -2 $O/tests_mfma.log
HGSR_BWD3_MFMA=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_dense.py -m gpu -x -q \
  -k "3dgs and not c2" --timeout 240 --timeout-method thread > $O/tests_mfma2.log 2>&1 \
  || { tail -60 $O/tests_mfma2.log; exit 1; }
tail -2 $O/tests_mfma2.log
HGSR_BWD2_MFMA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_dense.py tests/test_gpu_parity.py \
  tests/test_gpu_glue.py tests/test_gpu_normal.py -m gpu -x -q -k "2dgs and not c3 or normal" --timeout 240 \
  --timeout-method thread > $O/tests_bwd2.log 2>&1 || { tail -60 $O/tests_bwd2.log; exit 1; }
tail -2 $O/tests_bwd2.log
TAG=r04s1/ab_mfma1 ENV_A="HGSR_BWD3_MFMA=0" ENV_B="HGSR_BWD3_MFMA=1" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s1/ab_mfma2 ENV_A="HGSR_BWD3_MFMA=0" ENV_B="HGSR_BWD3_MFMA=2" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s1/ab_bwd2 ENV_A="HGSR_BWD2_MFMA=0" ENV_B="HGSR_BWD2_MFMA=1" CONFIGS="c3" bash scripts/gpu_r04_ab.sh || exit $?
