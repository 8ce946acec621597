"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV: mean device duration per
(kernel, grid) class, for the decode loop (dispatches after the last vision/prefill GEMM).

    python tools/trace_step.py <kernel_trace.csv> [--all]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if "--all" not in sys.argv:
        # keep the decode loop: after the last gemm_x3 (vision / prefill) dispatch
        last = max((i for i, r in enumerate(rows) if "gemm_x3" in r["Kernel_Name"]), default=-1)
        rows = rows[last + 1:]
    stats = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void dsocr::", "").replace("dsocr::", "")
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        stats[(name[:60], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in stats.values())
    print(f"{len(rows)} dispatches, {tot / 1e3:.2f} ms device time")
    for (name, grid), v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{name:60s} grid {grid:>8s} n {len(v):6d} mean {sum(v) / len(v):8.2f}us "
              f"p50 {v[len(v) // 2]:8.2f} total {sum(v) / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
