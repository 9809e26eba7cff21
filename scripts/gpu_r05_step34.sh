# Round 5, step 34: the one-GPU DDP rehearsal with two buckets (colours; everything else) instead of
# three: fewer collectives' fixed costs against the means / quats reduce-scatter's overlap.
set -o pipefail
TAG=r05s34 bash scripts/gpu_r05_step5.sh || exit $?
