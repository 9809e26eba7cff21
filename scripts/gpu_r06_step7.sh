# Round 6, step 7: the raster records packed on a side stream during the intersection count,
# the backward's seed tensor reused -- 3DGS / DDP tests, the c2 bench line, a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s7}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_deferred.py tests/test_gpu_glue.py tests/test_gpu_ddp_two_ranks.py tests/test_gpu_optim.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $O/bench_c2.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2b.json 2> $O/bench_c2b.err || { tail -20 $O/bench_c2b.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $O/bench_c2b.json
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s3 -o s3 --output-format csv -- $B3 > $O/s3.log 2>&1 || { tail -20 $O/s3.log; exit 1; }
python scripts/stats_summary.py $O/s3/s3_kernel_stats.csv 13 > $O/s3_stats.txt 2>&1
head -3 $O/s3_stats.txt
