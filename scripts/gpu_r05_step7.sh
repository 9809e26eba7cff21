# Round 5, step 7: where the raster backwards' float atomics stand -- frozen-scene (--freeze: no
# optimizer step, so both builds see the same views) A/B of the default build against a timing
# probe whose backwards form their sums but never add them (wrong results, time only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r05s7/probe_noatom LIB_B=horizongs_amd/_lib_probe2/libhgsr.so CONFIGS="c2 c3" REPS=2 BENCH_EXTRA=--freeze \
  bash scripts/gpu_r04_ab.sh || exit $?
