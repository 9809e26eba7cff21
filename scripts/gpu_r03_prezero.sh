# Raster parity tests with the forward-cleared backward rows, then bench A/B (pre-zero on/off,
# interleaved, c2 and c3).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03z}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_dense.py -m gpu -x -q -k "not slow" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for r in 1 2; do
  for z in 1 0; do
    for c in c2 c3; do
      HGSR_RASTER_PREZERO=$z timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/${T}_$c.z$z.$r.json 2> gpurun_out/${T}_$c.z$z.$r.err || exit $?
      python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k if 'raster' in x})" gpurun_out/${T}_$c.z$z.$r.json "$c z$z r$r"
    done
  done
done
