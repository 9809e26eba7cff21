# Round 6: gradients written in place into the sharded optimizer's buckets (gradbuf) -- the DDP
# GPU tests, then the one-GPU rehearsal of the c2 / c3 DDP step (one-rank RCCL group forced)
# against the same configs without it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06ddp}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp_two_ranks.py tests/test_gpu_optim.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -5 $O/tests.txt; [ $st -eq 0 ] || exit $st
port=29561
for cfg in c2 c3; do
  for v in plain force; do
    if [ $v = force ]; then F=1; else F=0; fi
    port=$((port + 1))
    HGSR_DDP_FORCE=$F timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --config $cfg --mode ddp --steps 30 --warmup 5 \
      --no-cpu-baseline --no-secondary --no-quality > $O/${cfg}_$v.json 2> $O/${cfg}_$v.err || { tail -30 $O/${cfg}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['parallelism'])" $O/${cfg}_$v.json
  done
done
