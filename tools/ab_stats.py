#!/usr/bin/env python3
"""Per-variant kernel durations from a rocprofv3 kernel trace of tools/ab_trace.py (or of one bench run).

    ab_stats.py <g_kernel_trace.csv> [<ab_order.json>] [--kernels substr,substr] [--bytes name=MB,...]

The trace is cut into generates at each prefill (a run of causal-prefill attention launches); generate i
takes variant order[i].  For every variant and decode kernel: launches, mean / median duration, the mean
over back-to-back launches (the previous dispatch ended when this one started: its boundary is inside
the duration, as in a graph replay without profiler gaps) and after-gap launches, and GB/s from --bytes.
"""
import csv
import json
import re
import statistics as S
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"^void ", "", n).replace("dsocr::", "")
    return n.split("(")[0]


def main():
    trace = sys.argv[1]
    order = None
    rest = sys.argv[2:]
    if rest and not rest[0].startswith("--"):
        order = json.load(open(rest[0]))["order"]
        rest = rest[1:]
    want = None
    nbytes = {}
    for i, a in enumerate(rest):
        if a == "--kernels":
            want = rest[i + 1].split(",")
        if a == "--bytes":
            for kv in rest[i + 1].split(","):
                k, v = kv.split("=")
                nbytes[k] = float(v) * 1e6
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # generate boundaries: the first causal-prefill attention launch after >= 200 other launches
    starts, last = [], -10**9
    for i, r in enumerate(rows):
        if "attention_fwd2_kernel" in r["Kernel_Name"]:
            if i - last > 200:
                starts.append(i)
            last = i
    starts.append(len(rows))
    per = defaultdict(lambda: defaultdict(lambda: {"all": [], "b2b": [], "gap": []}))
    for g in range(len(starts) - 1):
        name = order[g]["variant"] if order and g < len(order) else f"gen{g}"
        if name.startswith("_"):
            continue
        for i in range(starts[g], starts[g + 1]):
            r, p = rows[i], rows[i - 1]
            k = short(r["Kernel_Name"])
            if want and not any(w in k for w in want):
                continue
            s, e, pe = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(p["End_Timestamp"])
            d = (e - s) / 1e3
            key = f"{k}|{r['Grid_Size_X']}"
            per[name][key]["all"].append(d)
            per[name][key]["b2b" if s - pe <= 500 else "gap"].append(d)
    for name, ks in per.items():
        print(f"== {name}")
        for key, d in sorted(ks.items(), key=lambda kv: -sum(kv[1]["all"])):
            if len(d["all"]) < 20:
                continue
            k = key.split("|")[0]
            mb = next((v for n, v in nbytes.items() if n in k), None)
            m = S.mean(d["all"])
            b2b = S.mean(d["b2b"]) if d["b2b"] else float("nan")
            gap = S.mean(d["gap"]) if d["gap"] else float("nan")
            extra = f"  {mb / (m * 1e-6) / 1e9:7.1f} GB/s frac {mb / (m * 1e-6) / 8e12:.3f}" if mb else ""
            print(f"  {key[:58]:58s} n {len(d['all']):6d} mean {m:7.2f} med {S.median(d['all']):7.2f} "
                  f"b2b {b2b:7.2f} ({len(d['b2b'])}) gap {gap:7.2f} ({len(d['gap'])}){extra}")


if __name__ == "__main__":
    main()
