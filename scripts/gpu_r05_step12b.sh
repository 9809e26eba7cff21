# Round 5, step 12b: the barrier probe again with the float atomics off in both builds (step 12's
# no-barrier build sent stale ids' sums into one hot row and measured that contention instead):
# A = no atomics, B = no atomics and no batch barriers; frozen scene, 2 runs a side.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r05s12/probe_nobar2 LIB_A=horizongs_amd/_lib_noatom/libhgsr.so LIB_B=horizongs_amd/_lib_nobar/libhgsr.so \
  CONFIGS="c2 c2-fixed" REPS=2 BENCH_EXTRA=--freeze bash scripts/gpu_r04_ab.sh || exit $?
