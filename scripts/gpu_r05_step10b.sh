# Round 5, step 10b: the cost of the gsplat-form 2DGS hit (HGSR_GSPLAT_HIT) at c3 -- its parity
# run (step 10) already showed it leaves the strict rates against the gsplat-form f32 oracle
# where they were; this is the timing half (camera set, 2 runs a side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r05s10/ab_gsh LIB_B=horizongs_amd/_lib_gsh/libhgsr.so CONFIGS="c3" REPS=2 bash scripts/gpu_r04_ab.sh || exit $?
