# Round 6: the whole GPU suite (incl. the at-scale PSNR ensembles and the chunk test) + smoke.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06suite}; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gputests.txt 2>&1
st=$?; tail -4 $O/gputests.txt; cp gpurun_out/parity_rates.txt $O/ 2>/dev/null; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
