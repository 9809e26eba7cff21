# Round 5, final bench: the default bench line (c2 camera set + secondaries + live PSNR quality +
# CPU baseline) of the committed tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05final; mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
