# Round 5, step 37: where the N = 4 shared-GPU rehearsal (step 36) stalls -- c2 only, stack dumps
# of every rank each 30 s (scripts/ft_run.py), bounded at 200 s.
set -o pipefail
mkdir -p gpurun_out/r05s37
HGSR_BENCH_SHARE_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29543 scripts/ft_run.py bench.py --gpus 4 --steps 4 --warmup 1 \
  --no-secondary > gpurun_out/r05s37/n4.json 2> gpurun_out/r05s37/n4.err
st=$?
tail -c 400 gpurun_out/r05s37/n4.json
exit $st
