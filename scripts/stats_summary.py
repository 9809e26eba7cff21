import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total GPU ms per step {tot / 1e6 / steps:.3f}")
for r in rows[:30]:
    n = r['Name']
    short = n.split('(')[0]
    if 'at::native' in short:
        short = 'torch:' + (n.split('at::native::')[1][:70] if 'at::native::' in n else short[:70])
    print(f"{short[-75:]:75s} calls/step {float(r['Calls']) / steps:5.1f} avg_us {float(r['AverageNs']) / 1e3:9.2f} ms/step {float(r['TotalDurationNs']) / 1e6 / steps:7.3f}")
