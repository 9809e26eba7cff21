# Round 5, step 8: accumulator rows padded to whole lines (2DGS 96 -> 128 B, 3DGS 48 -> 64 B)
# so no row's float atomics straddle two cache lines: dense parity on the padded build, then an
# interleaved A/B against the default build (the camera-set bench, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s8
HGSR_LIB=horizongs_amd/_lib_rec/libhgsr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity_dense.py > gpurun_out/r05s8/tests_rec.log 2>&1 || { tail -30 gpurun_out/r05s8/tests_rec.log; exit 1; }
tail -2 gpurun_out/r05s8/tests_rec.log
TAG=r05s8/ab_rec LIB_B=horizongs_amd/_lib_rec/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
