# Round 5: single-GPU rehearsal of the multi-GPU step over RCCL (HGSR_DDP_FORCE=1: a one-rank
# nccl group runs c2 through the sharded optimizer -- reduce-scatter, shard Adam, all-gather --
# and c5 through the bucketed all-reduce with early decode gradients), against the same configs without it.
set -o pipefail
O=gpurun_out/${TAG:-r05s5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
port=29541
for cfg in c2 c5; do
  for v in plain force; do
    if [ $v = force ]; then F=1; else F=0; fi
    port=$((port + 1))
    HGSR_DDP_FORCE=$F timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --config $cfg --mode ddp --steps 20 --warmup 5 \
      --no-cpu-baseline --no-secondary --no-quality > $O/${cfg}_$v.json 2> $O/${cfg}_$v.err || { tail -30 $O/${cfg}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['parallelism'])" $O/${cfg}_$v.json
  done
done
