# Attribute the torch glue kernels of the c2 step, then one c2 bench line (no secondaries).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03g}
timeout -k 10 300 python -u scripts/glue_ops.py > gpurun_out/${T}_glue.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo done
