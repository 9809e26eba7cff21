# Round 6, step 1: deterministic gradient slots -- run-to-run equality, raster parity suites,
# then the c2 / c3 bench lines (no CPU baseline / quality) for the cost.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_deferred.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -5 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-quality --no-secondary > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
tail -c 600 $O/bench_c2.json; echo; tail -c 600 $O/bench_c3.json
