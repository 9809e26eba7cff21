# Round 6, step 8: the backward's piece count cleared by the forward's slot scan (no memset launch)
# -- 3DGS / DDP tests and the c2 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s8}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_ddp_two_ranks.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
for k in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2_$k.json 2> $O/bench_c2_$k.err || { tail -20 $O/bench_c2_$k.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $O/bench_c2_$k.json
done
