# Round 5, step 32: one-parameter DDP buckets reduce-scatter autograd's gradient tensors in place
# (no scaled copy into a flat buffer; the 1/N on the shard) -- the one-rank RCCL test, then the
# one-GPU rehearsal.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_optim.py \
  > gpurun_out/r05s32_optim.txt 2>&1 || { tail -20 gpurun_out/r05s32_optim.txt; exit 1; }
tail -2 gpurun_out/r05s32_optim.txt
TAG=r05s32 bash scripts/gpu_r05_step5.sh || exit $?
