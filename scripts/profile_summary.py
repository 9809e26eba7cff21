"""Summarise a gpu_profiles.sh run into profiles/: per-kernel kernel-trace stats and
HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 128-B read
requests at 64 B, so it reports half the bytes of wide reads -> doubled here;
WRITE_SIZE is exact for float atomics and 16-B stores.  Both counters are in KB.
Usage: python scripts/profile_summary.py gpurun_out/profiles r01
"""
import collections
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("hgsr::", "")


out = {}
for gs in ("3", "2"):
    stats = {}
    for r in csv.DictReader(open(f"{src}/s{gs}/s{gs}_kernel_stats.csv")):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    shutil.copy(f"{src}/s{gs}/s{gs}_kernel_stats.csv", f"{dst}/{tag}_rocprof_kernel_stats_{gs}dgs.csv")
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for kind in ("f", "w"):
        for r in csv.DictReader(open(f"{src}/{kind}{gs}/{kind}{gs}_counter_collection.csv")):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    ks = {}
    for k, d in pmc.items():
        f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
        w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
        ks[k] = {"fetch_size_raw_bytes": round(f), "write_size_bytes": round(w),
                 "hbm_bytes_corrected": round(2 * f + w), "avg_us": stats.get(k, {}).get("avg_us")}
    out[f"{gs}dgs"] = ks
json.dump({"source": "scripts/gpu_profiles.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
           "correction": "hbm_bytes_corrected = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halves wide reads)",
           "kernels": out}, open(f"{dst}/{tag}_pmc_traffic.json", "w"), indent=1)
for gs, ks in out.items():
    for k, v in sorted(ks.items(), key=lambda kv: -(kv[1]["avg_us"] or 0)):
        print(gs, f"{k:36s} {v['avg_us'] or 0:9.1f} us  {v['hbm_bytes_corrected'] / 1e6:9.1f} MB/launch")
