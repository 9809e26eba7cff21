# Round 4: the projection backwards load the grad-sink scale gradient with their first memory round
# trip (it was loaded after the camera loop: project3d_bwd 56.8 -> 81.4 us when the sink landed).
# Projection / glue parity tests, then an interleaved A/B against the previous build (_lib_old).
set -o pipefail
O=gpurun_out/r04s16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_glue.py -m gpu -v \
  -k "proj or glue or sink or scale" --timeout 240 --timeout-method thread > $O/tests.log 2>&1
st=$?
tail -n 2 $O/tests.log; grep -E "^FAILED|Error:" $O/tests.log | head
if [ $st -ne 0 ]; then exit $st; fi
TAG=r04s16/ab LIB_A=horizongs_amd/_lib_old/libhgsr.so CONFIGS="c2 c3" bash scripts/gpu_r04_ab.sh || exit $?
for v in old new; do
  if [ $v = old ]; then L=horizongs_amd/_lib_old/libhgsr.so; else L=horizongs_amd/_lib/libhgsr.so; fi
  HGSR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --config c2 \
    --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
done
