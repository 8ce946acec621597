"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.2f}us {float(r['Percentage']):6.2f}%")
