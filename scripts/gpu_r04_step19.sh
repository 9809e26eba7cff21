# Round 4: where the one-rank DDP path's extra time goes (c2, HGSR_DDP_FORCE=1 vs plain): rocprofv3
# kernel stats of bench.py run as rank 0 of a one-rank nccl group (env rendezvous, no launcher).
set -o pipefail
O=gpurun_out/r04s19
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for v in plain force; do
  if [ $v = force ]; then F=1; P=29561; else F=0; P=29562; fi
  HGSR_DDP_FORCE=$F MASTER_PORT=$P timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 bench.py \
    --gpus 1 --config c2 --mode ddp --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing > $O/$v.log 2>&1 \
    || { tail -30 $O/$v.log; exit 1; }
  tail -c 300 $O/$v.log
done
