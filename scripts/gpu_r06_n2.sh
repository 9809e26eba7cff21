# Round 6 (after the in-place gradients and the 64-B records): rehearsal of the driver's N = 2 bench run on a one-GPU box -- two torchrun ranks
# sharing the GPU, collectives over gloo on device tensors (HGSR_BENCH_SHARE_GPU=1): the headline
# c2 DDP line (sharded optimizer), the c2-chunks / c4 / c5 secondaries, max-over-ranks timing and
# the JSON line.  The numbers are not RCCL numbers; the code paths are the N > 1 ones.
set -o pipefail
mkdir -p gpurun_out/r06n2
HGSR_BENCH_SHARE_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 8 --warmup 2 \
  > gpurun_out/r06n2/n2.json 2> gpurun_out/r06n2/n2.err || { tail -30 gpurun_out/r06n2/n2.err; exit 1; }
tail -c 600 gpurun_out/r06n2/n2.json
