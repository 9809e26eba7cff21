# raster3d_bwd time for alternative builds (build/<v>/libhgsr.so) vs the in-tree library
set -o pipefail
mkdir -p gpurun_out
for v in base ${VARIANTS}; do
  if [ "$v" = base ]; then unset HGSR_LIB; else export HGSR_LIB=$PWD/build/$v/libhgsr.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/var_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/var_$v.json')); k=d['kernels']
print('$v', d['value'], {n: k[n]['avg_ms'] for n in k if ('raster' in n or 'project' in n or 'adam' in n or 'isect' in n or 'sort' in n)})"
done
