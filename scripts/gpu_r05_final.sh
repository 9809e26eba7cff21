# Round 5, final: the whole GPU suite (incl. the at-scale PSNR ensembles), smoke, and the default
# bench line of the committed tree; outputs under gpurun_out/r05final.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gputests.txt 2>&1
st=$?; tail -3 $O/gputests.txt; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
