"""rocprofv3 kernel statistics from its SQLite output (rocpd `*_results.db`, the default output
format on this image) in the CSV layout of `rocprofv3 --stats` (*_kernel_stats.csv): Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev.
Usage: python scripts/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_rocprof_kernel_stats_X.csv"""
import csv
import math
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    per = {}
    for name, start, end in con.execute("select name, start, end from kernels"):
        per.setdefault(name, []).append(int(end) - int(start))
    total = sum(sum(v) for v in per.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        n, s = len(d), sum(d)
        avg = s / n
        sd = math.sqrt(sum((x - avg) ** 2 for x in d) / n)
        w.writerow([name, n, s, round(avg, 6), round(100.0 * s / total, 4), min(d), max(d), round(sd, 6)])


if __name__ == "__main__":
    main()
