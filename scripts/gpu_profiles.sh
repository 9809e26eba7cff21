# Round profiles: kernel-trace stats (3DGS + 2DGS bench) and HBM traffic PMC passes.
# Each rocprofv3 call is its own pass; --pmc is never combined with other tracing.
set -o pipefail
OUT=gpurun_out/profiles
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing"
B2="python bench.py --gs 2d --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-timing"
K="raster3d|raster2d|tile_sort|isect|project|pack|split|adam|loss|normal|rotate"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/s3 -o s3 --output-format csv -- $B3 > $OUT/s3.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/s2 -o s2 --output-format csv -- $B2 > $OUT/s2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/f3 -o f3 --output-format csv -- $B3 > $OUT/f3.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/w3 -o w3 --output-format csv -- $B3 > $OUT/w3.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $OUT/f2 -o f2 --output-format csv -- $B2 > $OUT/f2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $OUT/w2 -o w2 --output-format csv -- $B2 > $OUT/w2.log 2>&1
st=$?
find $OUT -name "*.csv" | head -40
exit $st
