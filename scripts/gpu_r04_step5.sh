# Round 4: decode backward slot lanes (A/B vs the previous commit's build), the raster kernels'
# in-loop vmcnt waits removed (A/B vs HEAD's build), the colour kernel at 2 vs 3 waves/SIMD.
# Tests first; any failure ends the script before the benches.
set -o pipefail
O=gpurun_out/r04s5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_c4_chunk.py tests/test_gpu_parity.py \
  tests/test_gpu_parity_dense.py -m gpu -v -k "not fullsize" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s5/ab_cov LIB_A=horizongs_amd/_lib_c1/libhgsr.so LIB_B=horizongs_amd/_lib_base/libhgsr.so CONFIGS="c4 c2-anchors" \
  bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s5/ab_vm LIB_A=horizongs_amd/_lib_base/libhgsr.so LIB_B=horizongs_amd/_lib/libhgsr.so CONFIGS="c2 c3" \
  bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s5/ab_cw LIB_A=horizongs_amd/_lib/libhgsr.so LIB_B=horizongs_amd/_lib_cw2/libhgsr.so CONFIGS="c4" \
  bash scripts/gpu_r04_ab.sh || exit $?
