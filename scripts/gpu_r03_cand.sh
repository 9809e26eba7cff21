# Candidate library: the raster parity tests against it, then rocprof kernel durations of
# the c2 bench for HEAD (_lib_ref) and the candidate.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03m}
CAND=${CAND:-horizongs_amd/_lib_pA}
HGSR_LIB=$CAND/libhgsr.so timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_parity_dense.py} > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
LIBS="horizongs_amd/_lib_ref $CAND horizongs_amd/_lib_ref $CAND" bash scripts/gpu_r03_probes.sh || exit $?
echo done
