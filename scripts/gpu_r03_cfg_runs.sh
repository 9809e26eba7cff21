# Bench lines of the given configs (CONFIGS) with the working tree's library, two runs each.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in ${CONFIGS:-c4 c3}; do
  for r in 1 2; do
    timeout -k 10 300 python bench.py --config $C --no-secondary --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/run_${C}_$r.json 2> gpurun_out/run_${C}_$r.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/run_${C}_$r.json').read().strip().splitlines()[-1]); print('$C run $r', d['value'], d['ms_per_step'])"
  done
done
