# Round 5, step 6: A/B of one barrier per batch in raster3d_bwd (A: default, B: HGSR_BWD3_ONEBAR=1)
# on c2, the 3DGS parity subset on the B build, then the one-GPU rehearsal of the DDP paths.
set -o pipefail
O=gpurun_out/r05s6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=horizongs_amd/_lib_onebar/libhgsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_parity_dense.py -m gpu -x -v -k "3dgs or raster3d or c1 or pair" --timeout 300 --timeout-method thread > $O/tests_onebar.log 2>&1
st=$?; tail -3 $O/tests_onebar.log; if [ $st -ne 0 ]; then grep -E "^E |FAIL|Error" $O/tests_onebar.log | head -30; exit $st; fi
TAG=r05s6/ab_onebar LIB_B=horizongs_amd/_lib_onebar/libhgsr.so CONFIGS="c2 c2-fixed" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
bash scripts/gpu_r05_step5.sh
