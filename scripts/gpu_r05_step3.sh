# Round 5, step 3: tests touched this round (deferred / glue / chunks / decode split heads /
# parity incl. the executed-pair counter), then an interleaved A/B of the heaviest-first tile
# order (A: HGSR_TILE_ORDER=0 build, B: the default build) on the camera-set c2 and c3 lines.
set -o pipefail
O=gpurun_out/r05s3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_chunks.py \
  tests/test_gpu_decode.py tests/test_gpu_parity.py tests/test_gpu_parity_dense.py -m gpu -x -v \
  --timeout 400 --timeout-method thread > $O/tests.log 2>&1
st=$?; tail -3 $O/tests.log; if [ $st -ne 0 ]; then grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $st; fi
grep -o "exec_pairs': ([0-9]*, [0-9]*)" $O/tests.log | head
TAG=r05s3/ab_order LIB_A=horizongs_amd/_lib_noorder/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
