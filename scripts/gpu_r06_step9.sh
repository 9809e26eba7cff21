# Round 6, step 9: 128-B 2DGS records carrying the gradient-slot base (written by the training
# forward's pack2, as 3DGS) -- the raster tests, the c3 line, its kernel stats and traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s9}; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_parity_dense.py tests/test_gpu_deferred.py tests/test_gpu_glue.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
for k in 1 2; do
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-quality --no-secondary > $O/bench_c3_$k.json 2> $O/bench_c3_$k.err || { tail -20 $O/bench_c3_$k.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $O/bench_c3_$k.json
done
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
K="raster2d|pack2|slot|reduce_pieces|split2"
R() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; echo "$name ok"; }
R s2 --kernel-trace --stats -d $O/s2 -o s2 --output-format csv -- $B2 && \
R f2 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/f2 -o f2 --output-format csv -- $B2 && \
R w2 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/w2 -o w2 --output-format csv -- $B2
st=$?
python scripts/stats_summary.py $O/s2/s2_kernel_stats.csv 13 > $O/s2_stats.txt 2>&1
head -12 $O/s2_stats.txt
exit $st
