set -o pipefail
mkdir -p gpurun_out/envab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -k "$TESTS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_exp.log 2>&1 || { tail -30 gpurun_out/t_exp.log; exit 1; }
tail -1 gpurun_out/t_exp.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary $BARGS > gpurun_out/envab/$v.$r.json 2>gpurun_out/envab/$v.$r.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/envab/$v.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$v', d['value'], d['ms_per_step'], {x:k[x]['avg_ms'] for x in k})"
  done
done
