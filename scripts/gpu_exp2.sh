# Scratch: (1) 2DGS forward variants (parity on $VLIB, then A/B of $LIBS on the 2DGS bench),
# (2) decode / densify GPU tests and the decode-inclusive bench line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=$VLIB/libhgsr.so timeout -k 10 400 python -u -m pytest tests -m gpu -k "2dgs" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_exp.log 2>&1 || { tail -30 gpurun_out/t_exp.log; exit 1; }
tail -1 gpurun_out/t_exp.log
BENCH_ARGS="--gs 2d --steps 20 --warmup 5 --no-cpu-baseline --no-secondary" timeout -k 10 900 bash scripts/gpu_libs.sh > gpurun_out/libs_x.txt 2>&1 || exit 1
python - <<'PY'
import json, os
libs = os.environ["LIBS"].split()
for n in range(1, len(libs) + 1):
  for r in ('1','2'):
    d=json.loads(open(f'gpurun_out/libs/{n}.{r}.json').read().strip().splitlines()[-1]); k=d['kernels']
    print(libs[n-1].split('/')[-1], r, d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k if 'raster' in x})
PY
timeout -k 10 400 python -u -m pytest tests -m gpu -k "decode or densify or statis" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dec.log 2>&1 || { tail -30 gpurun_out/t_dec.log; exit 1; }
tail -1 gpurun_out/t_dec.log
timeout -k 10 300 python bench.py --anchors 500000 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/anch.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('gpurun_out/anch.json').read().strip().splitlines()[-1]);print('anchors', d['value'], d['ms_per_step'])"
