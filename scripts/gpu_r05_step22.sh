# Round 5, step 22: the library built without packed-fp32 instructions (-target-feature
# -packed-fp32-ops).  v_pk_fma/mul/add_f32 issue at half rate on gfx950 (no FLOP gain,
# scripts/micro/pkrate.hip) and the compiler adds v_mov's to pair their operands: the raster
# step loops drop from 132 -> 98 (3DGS fwd group), 382 -> 350 (3DGS bwd group), 62 -> 53 (2DGS
# fwd step), 482 -> 409 (2DGS bwd pass 2) issue slots.  Parity on the build, then A/Bs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s22
HGSR_LIB=horizongs_amd/_lib_nopk/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity_dense.py tests/test_gpu_parity.py > gpurun_out/r05s22/tests.log 2>&1 \
  || { tail -30 gpurun_out/r05s22/tests.log; exit 1; }
tail -1 gpurun_out/r05s22/tests.log
TAG=r05s22/ab_nopk LIB_B=horizongs_amd/_lib_nopk/libhgsr.so CONFIGS="c2 c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
