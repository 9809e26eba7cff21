# Round 4: raster parity suites with the strict report, then decode-backward evidence at c4
# (rocprofv3 kernel stats of the c4 line; per-phase clocks from the instrumented library).
set -o pipefail
O=gpurun_out/r04s3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -f $O/parity_strict.jsonl
HGSR_PARITY_REPORT=$O/parity_strict.jsonl timeout -k 10 700 python -u -m pytest tests/test_gpu_parity_dense.py \
  tests/test_gpu_parity.py tests/test_gpu_normal.py -m gpu -v -rA --timeout 600 --timeout-method thread \
  > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -gt 1 ]; then exit $st; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4 -o c4 --output-format csv -- python bench.py --config c4 \
  --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
python scripts/stats_summary.py $O/c4/c4_kernel_stats.csv 13 > $O/c4_stats.txt; head -30 $O/c4_stats.txt
HGSR_LIB=horizongs_amd/_lib_prof/libhgsr.so timeout -k 10 300 python scripts/decode_prof.py --config c4 --steps 5 \
  --warmup 2 > $O/decode_prof_c4.txt 2>&1 || { tail -20 $O/decode_prof_c4.txt; exit 1; }
cat $O/decode_prof_c4.txt
