# isect tests (large bins), then tile_sort timing on c5 / c2-anchors / c4 / c2.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "isect" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for c in c5 c2-anchors c4 c2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/${T}_$c.json 2> gpurun_out/${T}_$c.err || exit $?
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; k=d['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k if 'isect' in x or 'sort' in x})" gpurun_out/${T}_$c.json "$c"
done
