# Round 5, step 19: raster3d_fwd walking 2 or 4 tiles per workgroup (HGSR_FWD_TPW) -- the
# per-workgroup timing probe (r05s18/wg_time.jsonl) showed ~4.3 resident workgroups per CU of 8
# with workgroups dispatched until the last 15 % of the launch: fewer, longer workgroups test
# whether dispatch, not the CUs, sets the forward's pace.  Parity, then A/Bs (c2, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s19
for v in tpw2 tpw4; do
  HGSR_LIB=horizongs_amd/_lib_$v/libhgsr.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity_dense.py tests/test_gpu_parity.py -k "3d or 3dgs or c2 or isect or c1" > gpurun_out/r05s19/tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/r05s19/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05s19/tests_$v.log
done
TAG=r05s19/ab_tpw2 LIB_B=horizongs_amd/_lib_tpw2/libhgsr.so CONFIGS="c2" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
TAG=r05s19/ab_tpw4 LIB_B=horizongs_amd/_lib_tpw4/libhgsr.so CONFIGS="c2" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
