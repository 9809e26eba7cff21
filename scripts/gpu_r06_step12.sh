# Round 6, step 12: the slot prefix's row sums read hgsr_isect_count's tiles_per_gauss -- the
# raster / training / determinism tests, the c2 line and its kernel list.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s12}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_glue.py tests/test_gpu_parity.py tests/test_gpu_run_to_run.py tests/test_gpu_deferred.py tests/test_gpu_c4_chunk.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'])
for s in d.get('secondary') or []: print(s['config'], s['value'], s['ms_per_step'])" $O/bench.json
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s2 -o s2 --output-format csv -- $B > $O/s2.log 2>&1 || { tail -20 $O/s2.log; exit 1; }
python scripts/stats_summary.py $O/s2/s2_kernel_stats.csv 13 > $O/s2_stats.txt 2>&1
grep -E "total|slot_|pack3" $O/s2_stats.txt
