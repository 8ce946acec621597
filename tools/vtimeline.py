"""Dev tool: per-stream busy time and idle gaps of one steady-state vision pass in a rocprofv3 kernel trace of
tools/prof_vision.py (the pass = the launches between the i-th patch_im2col and the next clip_embed / prefill).
    python tools/vtimeline.py TRACE.csv [pass index, default last]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]]
starts = [i for i, r in enumerate(rows) if "patch_im2col" in r["Kernel_Name"]]
# two im2col launches per pass (global view + tiles): pass k starts at starts[2k]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2 - 1
i0 = starts[2 * k]
seq = []
for r in rows[i0:]:
    if "rmsnorm" in r["Kernel_Name"] or "embed_gather" in r["Kernel_Name"] or "assemble" in r["Kernel_Name"]:
        break
    seq.append(r)
t0 = int(seq[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seq)
print(f"pass {k}: {len(seq)} launches, span {(t1 - t0) / 1e3:.1f} us")
by_q = collections.defaultdict(list)
for r in seq:
    by_q[r["Queue_Id"]].append(r)
for q, rs in by_q.items():
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    end = (max(int(r["End_Timestamp"]) for r in rs) - t0) / 1e3
    print(f"queue {q}: {len(rs)} launches, busy {busy:.1f} us, ends at {end:.1f} us")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rs:
        n = r["Kernel_Name"].replace("dsocr::", "").split("(")[0][:48]
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f"    {d:8.1f} us {c:4d}  {n}")
