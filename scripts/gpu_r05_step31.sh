# Round 5, step 31: the explicit-Gaussian DDP with its buckets in the backward's gradient order
# (colours first: their reduce-scatter under the projection / activation backwards) and the
# deferred colours bucket stepped last -- the one-rank RCCL test, then the one-GPU rehearsal.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_optim.py \
  > gpurun_out/r05s31_optim.txt 2>&1 || { tail -20 gpurun_out/r05s31_optim.txt; exit 1; }
tail -2 gpurun_out/r05s31_optim.txt
TAG=r05s31 bash scripts/gpu_r05_step5.sh || exit $?
