# Round 4: optional GPU tests, then an interleaved bench A/B on one box.
# Usage: TAG=x [TESTS="tests/a.py ..."] [KFILTER=...] ENV_A="K=V" ENV_B="K=V" [CONFIGS="c2 c3"] [REPS=2]
#        [LIB_A=... LIB_B=...] [BENCH_EXTRA=...] bash scripts/gpu_r04_ab.sh
# Any non-zero test / bench status ends the script there (nothing more touches the GPU).
set -o pipefail
TAG=${TAG:-r04ab}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  KARG=()
  if [ -n "$KFILTER" ]; then KARG=(-k "$KFILTER"); fi
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v "${KARG[@]}" --timeout 240 --timeout-method thread \
    > gpurun_out/$TAG/tests.log 2>&1
  st=$?
  tail -3 gpurun_out/$TAG/tests.log
  if [ $st -ne 0 ]; then grep -E "FAIL|Error|error" gpurun_out/$TAG/tests.log | head -20; exit $st; fi
fi
A=${LIB_A:-horizongs_amd/_lib/libhgsr.so}
B=${LIB_B:-horizongs_amd/_lib/libhgsr.so}
for cfg in ${CONFIGS:-c2}; do
  for r in $(seq 1 ${REPS:-2}); do
    for v in a b; do
      if [ $v = a ]; then L=$A; E=$ENV_A; else L=$B; E=$ENV_B; fi
      env HGSR_LIB=$L $E timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 \
        --no-cpu-baseline --no-secondary --no-quality $BENCH_EXTRA > gpurun_out/$TAG/${cfg}_${v}$r.json \
        2> gpurun_out/$TAG/${cfg}_${v}$r.err || { tail -20 gpurun_out/$TAG/${cfg}_${v}$r.err; exit 1; }
    done
  done
done
python - <<'PY'
import glob, json, os
tag = os.environ.get("TAG", "r04ab")
for f in sorted(glob.glob(f"gpurun_out/{tag}/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["value"], d["ms_per_step"],
          {x: k[x]["avg_ms"] for x in k if "raster" in x or x in ("tile_sort", "isect_emit", "isect_count", "decode_bwd")},
          {x: r.get(x) for x in ("kernel_avg_ms", "frac")})
PY
