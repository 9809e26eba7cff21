# Round 5, step 11: the whole GPU suite on the tree with the asm staging DMA and 64-B 3DGS rows
# as defaults (incl. the new run-to-run spread test), then smoke.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05s11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05s11/tests.log 2>&1 || { tail -40 gpurun_out/r05s11/tests.log; exit 1; }
tail -3 gpurun_out/r05s11/tests.log
grep -h "run_to_run\|bit_identical" gpurun_out/run_to_run_*.json | head -2
cat gpurun_out/run_to_run_2d.json | head -40
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05s11/smoke.txt 2>&1 || { tail -20 gpurun_out/r05s11/smoke.txt; exit 1; }
tail -2 gpurun_out/r05s11/smoke.txt
