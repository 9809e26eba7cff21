# PMC passes (one counter group per run, --kernel-trace not combined with sys/runtime trace)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing"
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "raster3d|tile_sort|isect|project3d|pack3|split3" -d gpurun_out/pmc/p$i -o p$i --output-format csv -- $B > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
ls -R gpurun_out/pmc | head -30
