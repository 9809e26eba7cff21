# Round 6, step 3: 64-B records carrying the gradient-slot base (the backward's slot lookup
# shares the record's sector) -- 3DGS parity / run-to-run tests, the c2 bench line, its kernel
# stats and the raster kernels' FETCH / WRITE passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s3}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_deferred.py tests/test_gpu_glue.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --no-secondary > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
tail -c 400 $O/bench_c2.json; echo
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
K="raster3d|pack3|slot|reduce_pieces|split3"
R() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; echo "$name ok"; }
R s3 --kernel-trace --stats -d $O/s3 -o s3 --output-format csv -- $B3 && \
R f3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/f3 -o f3 --output-format csv -- $B3 && \
R w3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/w3 -o w3 --output-format csv -- $B3
st=$?
python scripts/stats_summary.py $O/s3/s3_kernel_stats.csv 13 > $O/s3_stats.txt 2>&1
head -16 $O/s3_stats.txt
exit $st
