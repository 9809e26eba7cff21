# Round 5, step 4: large footprints in the tile binning (BigQ) -- bit-exact isect tests, then an
# interleaved A/B (A: HGSR_BIGRECT off, B: default) on the camera-set c2 / c3 lines; then a
# timing probe of the 2DGS backward without its float atomics (wrong results, time only).
set -o pipefail
O=gpurun_out/r05s4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred.py -m gpu -x -v -k "isect or deferred" \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?; tail -3 $O/tests.log; if [ $st -ne 0 ]; then grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $st; fi
TAG=r05s4/ab_big LIB_A=horizongs_amd/_lib_nobig/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
TAG=r05s4/probe_noatom2 LIB_A=horizongs_amd/_lib/libhgsr.so LIB_B=horizongs_amd/_lib_probe2/libhgsr.so CONFIGS="c3" REPS=1 \
  bash scripts/gpu_r04_ab.sh || exit $?
