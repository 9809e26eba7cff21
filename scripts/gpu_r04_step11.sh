# Round 4: the 2DGS transposed backward with LDS-merged partials (build flag HGSR_BWD2TP_LDS=1)
# against global atomics: 2DGS parity tests on the variant, then an interleaved c3 A/B.
set -o pipefail
O=gpurun_out/r04s11
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=horizongs_amd/_lib_tplds/libhgsr.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_parity_dense.py tests/test_gpu_glue.py -m gpu -v -k "2dgs and not fullsize" --timeout 600 \
  --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -gt 1 ]; then exit $st; fi
TAG=r04s11/ab LIB_B=horizongs_amd/_lib_tplds/libhgsr.so CONFIGS="c3" REPS=3 bash scripts/gpu_r04_ab.sh || exit $?
