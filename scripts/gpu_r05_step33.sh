# Round 5, step 33: the one-GPU DDP rehearsal on the kept bucket layout (three buckets in gradient
# order, the colours' one-parameter bucket reduced in place).
set -o pipefail
TAG=r05s33 bash scripts/gpu_r05_step5.sh || exit $?
