# Round 4: the one-launch colour-head decode backward -- decode tests, then an interleaved c4 A/B
# against the chunked launches, and the c4 kernel stats of the new path.
set -o pipefail
O=gpurun_out/r04s4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_c4_chunk.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s4/ab_col ENV_A="HGSR_DEC_COLBWD=0" ENV_B="HGSR_DEC_COLBWD=1" CONFIGS="c4" bash scripts/gpu_r04_ab.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4 -o c4 --output-format csv -- python bench.py --config c4 \
  --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
python scripts/stats_summary.py $O/c4/c4_kernel_stats.csv 13 > $O/c4_stats.txt; grep -i "decode\|wgrad" $O/c4_stats.txt
