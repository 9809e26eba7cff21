"""Print the kernels of the last train step from a rocprofv3 kernel trace, in launch order,
with durations and idle gaps (finds glue launches between the HIP kernels).
Usage: python scripts/trace_step.py gpurun_out/prof/run_kernel_trace.csv [marker_kernel]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "project3d_fwd"
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = (starts[-2], starts[-1]) if len(starts) > 1 else (0, len(rows))
prev = None
tot = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    tot += (e - s) / 1e3
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "at::native::" in n:
        n = "torch:" + n.split("at::native::")[1]
    print(f"{(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {n[:110]}")
print(f"kernel us in step: {tot:.1f}; span {(int(rows[b - 1]['End_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
