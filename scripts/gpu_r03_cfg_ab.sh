# Bench A/B of one config (CONFIG) between the HEAD build (_lib_base) and the working tree (_lib),
# interleaved, two runs each.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C=${CONFIG:-c4}
for r in 1 2; do
  for L in _lib_base _lib; do
    HGSR_LIB=horizongs_amd/$L/libhgsr.so timeout -k 10 300 python bench.py --config $C --no-secondary --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ab_${C}_${L}_$r.json 2> gpurun_out/ab_${C}_${L}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${C}_${L}_$r.json').read().strip().splitlines()[-1]); print('$C $L run $r', d['value'], d['ms_per_step'])"
  done
done
