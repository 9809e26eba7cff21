# Round 5, step 21: does the forward's share of the accumulator-row clearing (zero_share, the
# last thing each forward workgroup does) hold its workgroup slots?  Timing probe without it
# (HGSR_PROBE_NOZERO: wrong gradients), frozen scene, 2 runs a side.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r05s21/probe_nozero LIB_B=horizongs_amd/_lib_nz/libhgsr.so CONFIGS="c2" REPS=2 BENCH_EXTRA=--freeze \
  bash scripts/gpu_r04_ab.sh || exit $?
