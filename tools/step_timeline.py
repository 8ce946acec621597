#!/usr/bin/env python3
"""One decode step's kernel timeline from a rocprofv3 kernel trace: gap before each launch (previous
end -> this start), dispatch duration, name, grid.  usage: step_timeline.py TRACE.csv [STEP_INDEX]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
heads = [i for i, r in enumerate(rows) if "dec_screen_final" in r["Kernel_Name"] or "dec_sample_final" in r["Kernel_Name"]]
i0, i1 = heads[k], heads[k + 1]
t0 = prev = int(rows[i0]["End_Timestamp"])
busy = 0
for r in rows[i0 + 1:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"gap {(s - prev) / 1e3:6.2f}  dur {(e - s) / 1e3:7.2f} us  {r['Kernel_Name'][:72]}  grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} wg={r['Workgroup_Size_X']}")
    prev = e
print(f"step {(prev - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {i1 - i0} launches")
