# Round 6: c4 A/B in one box -- this tree (SH centres in-kernel) against a HEAD worktree under
# _ab_head/ (batched-GEMM centres), alternated three times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06ab}; rm -rf $O; mkdir -p $O
R=$PWD
for i in 1 2 3; do
  for side in new old; do
    if [ $side = new ]; then d=$R; else d=$R/_ab_head; fi
    (cd $d && timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-quality --no-secondary) > $O/$side$i.json 2> $O/$side$i.err || { tail -20 $O/$side$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$side$i.json $side
  done
done
