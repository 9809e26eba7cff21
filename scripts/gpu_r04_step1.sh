# Round 4, first GPU pass: MFMA/VALU micro, the new tests, the MFMA-backward parity subsets, then
# interleaved A/Bs (MFMA pass 2 of the 3DGS / 2DGS backward).  A test FAILURE (pytest status 1)
# is reported and the script goes on; any other non-zero status (crash, abort, timeout) ends it.
set -o pipefail
mkdir -p gpurun_out/r04s1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s1
T() {  # T <log> <env...> -- <pytest args...>
  local log=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 600 python -u -m pytest "$@" -m gpu -q --timeout 240 --timeout-method thread \
    > $O/$log 2>&1
  local st=$?
  tail -n 2 $O/$log
  if [ $st -eq 1 ]; then grep -E "^FAILED|Error:" $O/$log | head -20; fi
  if [ $st -ne 0 ] && [ $st -ne 1 ]; then tail -n 40 $O/$log; exit $st; fi
  return 0
}
timeout -k 5 60 scripts/micro/mfma_valu > $O/mfma_valu.txt 2>&1 || exit $?
cat $O/mfma_valu.txt
T tests.log HGSR_X=0 -- tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_parity.py \
  tests/test_gpu_normal.py tests/test_gpu_decode.py
T tests_mfma.log HGSR_BWD3_MFMA=1 -- tests/test_gpu_parity_dense.py tests/test_gpu_parity.py \
  -k "3dgs and not c2 or raster3d or rasterization"
T tests_bwd2.log HGSR_BWD2_MFMA=1 -- tests/test_gpu_parity_dense.py tests/test_gpu_parity.py \
  tests/test_gpu_glue.py -k "2dgs and not c3"
TAG=r04s1/ab_mfma1 ENV_A="HGSR_BWD3_MFMA=0" ENV_B="HGSR_BWD3_MFMA=1" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s1/ab_bwd2 ENV_A="HGSR_BWD2_MFMA=0" ENV_B="HGSR_BWD2_MFMA=1" CONFIGS="c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s1/ab_mfma2 ENV_A="HGSR_BWD3_MFMA=0" ENV_B="HGSR_BWD3_MFMA=2" CONFIGS="c2" bash scripts/gpu_r04_ab.sh || exit $?
