# Round 5, step 25: the one-GPU RCCL rehearsal again with the explicit-Gaussian DDP buckets in
# gradient order and the colours' all-gather deferred into the next step's rasterization (gsplat_api
# parameter-ready hook): the path the driver's N > 1 scaling runs take.
set -o pipefail
TAG=r05s25 bash scripts/gpu_r05_step5.sh || exit $?
