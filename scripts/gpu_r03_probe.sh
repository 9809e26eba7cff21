# Round-3 probe: GPU render dumps for the branch-resolution debug, torch glue attribution,
# decode-backward phases, the default bench line and a rocprofv3 stats pass of the c2 line.
# Every GPU step has its own time limit; any non-zero status ends the script.
set -o pipefail
mkdir -p gpurun_out/prof_r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r03b}
echo "dump"; timeout -k 10 300 python scripts/dump_render.py > gpurun_out/${T}_dump.log 2>&1 || exit $?
echo "glue"; timeout -k 10 200 python scripts/glue_ops.py > gpurun_out/${T}_glue_3dgs.txt 2>&1 || exit $?
echo "decode prof"
for c in c2-anchors c4; do
  HGSR_LIB=horizongs_amd/_lib_prof/libhgsr.so timeout -k 10 300 python scripts/decode_prof.py --config $c --steps 5 --warmup 2 > gpurun_out/${T}_decode_prof_$c.txt 2>&1 || exit $?
done
echo "bench"; timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo "rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03/c2 -o run -- python3 bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_rocprof.log 2>&1 || exit $?
echo done
