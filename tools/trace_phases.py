#!/usr/bin/env python3
"""Per-phase kernel durations from a rocprofv3 --kernel-trace CSV of one bench run.

The bench's decode phases appear in the trace as runs of the decode MoE gate/up kernel separated by
other work; this splits a kernel's launches into maximal groups whose neighbours are < GAP_US apart
in dispatch order... simpler: it splits at the span_reduce launches (present only in the spans
generate) and at the profile_decode replays (back-to-back launches of the same kernel).
usage: trace_phases.py TRACE.csv KERNEL_SUBSTRING
"""
import csv
import sys

import numpy as np


def main():
    path, name = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = []  # (index, is_target, duration_us, kernel)
    for i, r in enumerate(rows):
        k = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        seq.append((k, d))
    # label each target launch by its context: 'spans' if the next launch is span_reduce, 'chain' if the
    # previous launch is the same kernel (profile_decode back-to-back), else 'decode'
    out = {"decode": [], "spans": [], "chain": []}
    for i, (k, d) in enumerate(seq):
        if name not in k:
            continue
        nxt = seq[i + 1][0] if i + 1 < len(seq) else ""
        prv = seq[i - 1][0] if i > 0 else ""
        if "span_reduce" in nxt:
            out["spans"].append(d)
        elif name in prv or name in nxt:
            out["chain"].append(d)
        else:
            out["decode"].append(d)
    for k, v in out.items():
        if v:
            a = np.array(v)
            print(f"{k:7s} n={len(a):5d} mean={a.mean():8.3f} us  p50={np.median(a):8.3f}  min={a.min():8.3f}  max={a.max():8.3f}")


if __name__ == "__main__":
    main()
