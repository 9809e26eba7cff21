# Library A/B (LIBS, each twice, interleaved), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03h}
timeout -k 10 900 bash scripts/gpu_libs.sh > gpurun_out/${T}_ab.txt 2>&1 || exit $?
tail -12 gpurun_out/${T}_ab.txt
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
fi
echo done
