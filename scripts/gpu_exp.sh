# Scratch experiment driver: parity subset on a variant build ($VLIB, tests -k $TESTS), then lib A/B ($LIBS).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HGSR_LIB=$VLIB/libhgsr.so timeout -k 10 400 python -u -m pytest tests -m gpu -k "$TESTS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_exp.log 2>&1 || { tail -30 gpurun_out/t_exp.log; exit 1; }
tail -2 gpurun_out/t_exp.log
timeout -k 10 600 bash scripts/gpu_libs.sh > gpurun_out/libs_x.txt 2>&1 || exit 1
python - <<'PY'
import json, os
libs = os.environ["LIBS"].split()
for n in range(1, len(libs) + 1):
  for r in ('1','2'):
    d=json.loads(open(f'gpurun_out/libs/{n}.{r}.json').read().strip().splitlines()[-1]); k=d['kernels']
    print(libs[n-1].split('/')[-1], r, d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k if x in ('isect_emit','tile_sort','raster3d_fwd','raster3d_bwd','raster2d_fwd','raster2d_bwd','project3d_bwd','adam','loss_fwd','loss_bwd')})
PY
