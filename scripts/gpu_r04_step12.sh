# Round 4: the deferred intersection count and the folded glue, measured: interleaved A/Bs of
# HGSR_DEFER_ISECT and of HGSR_GRAD_SINK / HGSR_FUSE_FRAME on c2 / c3, and the aten kernels left
# on the step (scripts/glue_ops.py).
set -o pipefail
O=gpurun_out/r04s12
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r04s12/ab_defer ENV_A="HGSR_DEFER_ISECT=0" ENV_B="HGSR_DEFER_ISECT=1" CONFIGS="c2 c3" bash scripts/gpu_r04_ab.sh || exit $?
TAG=r04s12/ab_glue ENV_A="HGSR_GRAD_SINK=0 HGSR_FUSE_FRAME=0" ENV_B="HGSR_GRAD_SINK=1 HGSR_FUSE_FRAME=1" CONFIGS="c2 c3" \
  bash scripts/gpu_r04_ab.sh || exit $?
timeout -k 10 300 python scripts/glue_ops.py --config c2 > $O/glue_c2.txt 2>&1 || { tail -20 $O/glue_c2.txt; exit 1; }
timeout -k 10 300 python scripts/glue_ops.py --config c3 > $O/glue_c3.txt 2>&1 || { tail -20 $O/glue_c3.txt; exit 1; }
tail -n 15 $O/glue_c2.txt $O/glue_c3.txt
