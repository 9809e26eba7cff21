# Round 5, step 16: per-tile intersection counts over the bench's camera set (scripts/tile_stats.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s16
timeout -k 10 300 python scripts/tile_stats.py --gs 3d > gpurun_out/r05s16/tiles_3d.jsonl 2>&1 && \
timeout -k 10 300 python scripts/tile_stats.py --gs 2d > gpurun_out/r05s16/tiles_2d.jsonl 2>&1
st=$?; cat gpurun_out/r05s16/tiles_3d.jsonl; tail -3 gpurun_out/r05s16/tiles_2d.jsonl; exit $st
