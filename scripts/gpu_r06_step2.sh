# Round 6, step 2: the two-rank DDP test (no gradient copied into a bucket), then the round-6
# profiles (scripts/gpu_r06_prof.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp_two_ranks.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
TAG=r06prof bash scripts/gpu_r06_prof.sh
