# raster3d_bwd phase profile (instrumented build) and the default bench line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03g}
HGSR_LIB=horizongs_amd/_lib_rprof/libhgsr.so timeout -k 10 150 python -u scripts/raster_prof.py > gpurun_out/${T}_rprof.txt 2>&1 || exit $?
grep raster3d_bwd -A1 gpurun_out/${T}_rprof.txt
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo done
