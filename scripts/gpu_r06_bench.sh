# Round 6: the default bench line exactly as the driver runs it (N = 1, secondaries, CPU
# baseline, live PSNR), timed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06bench}; rm -rf $O; mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "wall $(( $(date +%s) - start )) s"
tail -c 3000 $O/bench.json
