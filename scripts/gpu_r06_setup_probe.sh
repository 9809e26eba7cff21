# Round 6 experiment (the probe block has since been removed from raster3d.hip): is raster3d_bwd's setup latency exposed?
# product library and with 4 dependent loads added to every workgroup's setup chain.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06sp}; rm -rf $O; mkdir -p $O
for v in prod probe prod2 probe2; do
  case $v in prod*) L=horizongs_amd/_lib/libhgsr.so;; *) L=horizongs_amd/_lib_probe_setup/libhgsr.so;; esac
  HGSR_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u bench.py --freeze --no-cpu-baseline --no-quality --no-secondary > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" $O/$v.json $v
done
