# Round 5, step 10: 2DGS hits in gsplat's per-pixel form (HGSR_GSPLAT_HIT: h_u = p_x w - u,
# h_v = p_y w - v, x = h_u x h_v; records carry u, v, w) against the plane form.  2DGS parity on
# both builds (strict pass rates against the gsplat-form f32 oracle are in the logs), then an
# interleaved c3 A/B (camera set, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s10
for v in lib lib_gsh; do
  HGSR_LIB=horizongs_amd/_$v/libhgsr.so timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
    tests/test_gpu_parity_dense.py -k "2dgs" > gpurun_out/r05s10/tests_$v.log 2>&1 || { tail -30 gpurun_out/r05s10/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05s10/tests_$v.log
done
TAG=r05s10/ab_gsh LIB_B=horizongs_amd/_lib_gsh/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
