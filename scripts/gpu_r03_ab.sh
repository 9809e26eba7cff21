# Round-3 kernel iteration: the GPU suite on the working build, then an interleaved bench A/B
# of the reference build (LIB_REF) against it.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03c}
KARG=()
if [ -n "$KFILTER" ]; then KARG=(-k "$KFILTER"); fi
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -s "${KARG[@]}" --timeout 400 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1
st=$?
grep -E "passed|failed" gpurun_out/${T}_gputests.log | tail -2
if [ $st -ne 0 ] && [ $st -ne 1 ]; then echo "pytest status $st: stopping"; exit $st; fi
LIBS="${LIB_REF:-horizongs_amd/_lib_ref} horizongs_amd/_lib" timeout -k 10 700 bash scripts/gpu_libs.sh > gpurun_out/${T}_ab.txt 2>&1 || exit $?
cat gpurun_out/${T}_ab.txt | tail -12
exit $st
