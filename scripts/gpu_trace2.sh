# step timelines (kernel trace, gaps) of the anchors and 2DGS configs
set -o pipefail
OUT=gpurun_out/tr
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/a -o a --output-format csv -- python bench.py --anchors 500000 --steps 10 --warmup 3 --no-cpu-baseline --no-timing > $OUT/a.log 2>&1 && \
python scripts/trace_step.py $OUT/a/a_kernel_trace.csv decode_count > $OUT/a_step.txt && rm -f $OUT/a/a_kernel_trace.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o t --output-format csv -- python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-timing > $OUT/t.log 2>&1 && \
python scripts/trace_step.py $OUT/t/t_kernel_trace.csv project2d_fwd > $OUT/t_step.txt && rm -f $OUT/t/t_kernel_trace.csv
