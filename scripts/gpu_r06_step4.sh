# Round 6, step 4: raster3d_bwd's wait-site attribution (probe library), then the c2 bench line
# of the product library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s4}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u scripts/micro/wait_probe.py --steps 16 > $O/wait_probe.json 2> $O/wait_probe.err || { tail -20 $O/wait_probe.err; exit 1; }
cat $O/wait_probe.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])" $O/bench_c2.json
