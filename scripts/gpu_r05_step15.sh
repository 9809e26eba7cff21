# Round 5, step 15: limiter counters of the raster forwards (as the backwards' in gpu_r05_prof.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s15; mkdir -p $O
L="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B3="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing --no-quality"
B2="python bench.py --gs 2d --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-timing --no-quality"
timeout -k 10 200 rocprofv3 --pmc $L --kernel-include-regex "raster3d_fwd" -d $O/f3 -o f3 --output-format csv -- $B3 > $O/f3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc $L --kernel-include-regex "raster2d_fwd" -d $O/f2 -o f2 --output-format csv -- $B2 > $O/f2.log 2>&1 && \
python scripts/pmc_summary.py $O/f3 && python scripts/pmc_summary.py $O/f2
