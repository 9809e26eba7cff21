# Round 6, step 10: SH camera centres computed in the SH kernels from the view matrices (no
# batched GEMM + negation per view) -- SH / parity tests, the c4 line and its torch-kernel list.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06s10}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -3 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --no-quality --no-secondary > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'])" $O/bench_c4.json
B4="python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing --no-quality"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s4 -o s4 --output-format csv -- $B4 > $O/s4.log 2>&1 || { tail -20 $O/s4.log; exit 1; }
python scripts/stats_summary.py $O/s4/s4_kernel_stats.csv 10 > $O/s4_stats.txt 2>&1
grep -E "total|torch|Cijk|rocclr|sh_rgb" $O/s4_stats.txt
