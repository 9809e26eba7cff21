# One training step's kernel timeline (rocprofv3 kernel trace, full names, gaps):
#   BARGS="--gs 2d" MARK=project2d_fwd bash scripts/gpu_trace.sh
set -o pipefail
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/a -o a --output-format csv -- python bench.py $BARGS --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-timing > gpurun_out/tr/a.log 2>&1 || exit 1
python - <<'PY'
import csv, os
rows = sorted(csv.DictReader(open("gpurun_out/tr/a/a_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if os.environ["MARK"] in r["Kernel_Name"]]
a, b = st[-2], st[-1]
prev, tot = None, 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    tot += (e - s) / 1e3
    n = r["Kernel_Name"]
    if "hgsr::" in n:
        n = n.split("(")[0]
    print(f"{(e - s) / 1e3:8.1f} us gap {gap:7.1f} grid {r['Grid_Size_X']:>9} {n[:160]}")
print(f"kernel us in step: {tot:.1f}; span {(int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
PY
