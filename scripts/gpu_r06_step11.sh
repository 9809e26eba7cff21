# Round 6, step 11: the SH colour step's means gradient handed to the projection backward
# (v_means_in) -- glue / parity / c4-chunk tests, then c4 A/B against the previous commit in
# a worktree under _ab_head/, alternated three times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s11b}; rm -rf $O; mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_glue.py tests/test_gpu_parity.py tests/test_gpu_c4_chunk.py tests/test_gpu_explicit.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
for i in 1 2 3; do
  for side in new old; do
    if [ $side = new ]; then d=$R; else d=$R/_ab_head; fi
    (cd $d && timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-quality --no-secondary) > $O/$side$i.json 2> $O/$side$i.err || { tail -20 $O/$side$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$side$i.json $side
  done
done
