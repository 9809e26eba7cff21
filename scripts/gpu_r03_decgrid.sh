# Decode tests, then decode-backward grid A/B (resident-sized vs the fixed 1024 cap),
# interleaved, c2-anchors / c4 / c5.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_c4_chunk.py -m gpu -x -q -k "not slow" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for r in 1 2; do
  for z in new fixed; do
    for c in c2-anchors c4 c5; do
      if [ $z = fixed ]; then export HGSR_DEC_GRID_FIXED=1; else unset HGSR_DEC_GRID_FIXED; fi
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/${T}_$c.$z.$r.json 2> gpurun_out/${T}_$c.$z.$r.err || exit $?
      python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k if 'decode' in x})" gpurun_out/${T}_$c.$z.$r.json "$c $z r$r"
    done
  done
done
