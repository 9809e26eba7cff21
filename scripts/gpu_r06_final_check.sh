# Round 6: the clean-rebuilt library -- the parity, run-to-run, DDP and training-parity tests, smoke.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06fc}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_run_to_run.py tests/test_gpu_parity.py tests/test_gpu_deferred.py tests/test_gpu_ddp_two_ranks.py tests/test_gpu_chunks.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.txt 2>&1
st=$?; tail -2 $O/tests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
