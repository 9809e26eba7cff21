# Decode-backward phase breakdown (instrumented build, see scripts/decode_prof.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2-anchors c4; do
  HGSR_LIB=horizongs_amd/_lib_prof/libhgsr.so timeout -k 10 300 python scripts/decode_prof.py --config $c --steps 5 --warmup 2 > gpurun_out/decode_prof_$c.txt 2>&1 || exit $?
done
