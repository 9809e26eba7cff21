# Round 4: the whole GPU suite (strict-rate report of every raster parity run), smoke, and the
# default bench line, on one box.  A test FAILURE (pytest status 1) is reported and the script
# goes on; a crash, abort or timeout ends it.
set -o pipefail
TAG=${TAG:-r04suite}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -f $O/parity_strict.jsonl
HGSR_PARITY_REPORT=$O/parity_strict.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA \
  --timeout 600 --timeout-method thread ${KFILTER:+-k "$KFILTER"} > $O/gputests.log 2>&1
st=$?
tail -n 3 $O/gputests.log
grep -E "^FAILED|^ERROR" $O/gputests.log | head -20
if [ $st -gt 1 ]; then exit $st; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
