# Round 4, final evidence of the tree: the whole GPU suite (strict parity report), smoke, the
# default bench line, then the rocprofv3 / PMC passes (scripts/gpu_r04_prof.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r04final} bash scripts/gpu_r04_suite.sh || exit $?
bash scripts/gpu_r04_prof.sh
