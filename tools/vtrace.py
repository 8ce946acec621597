"""Dev: summarise a prof_vision.py kernel trace (last repetition's vision + prefill segment)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'patch_im2col' in r['Kernel_Name']]
last = rows[idx[-1] - 40:]
end = next(i for i, r in enumerate(last) if 'dec_' in r['Kernel_Name'] or 'lmhead' in r['Kernel_Name'])
seg = last[:end]
agg = collections.defaultdict(lambda: [0, 0.0])
per = collections.defaultdict(list)
for r in seg:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[r['Kernel_Name'][:50]][0] += 1
    agg[r['Kernel_Name'][:50]][1] += d
    if 'gemm' in r['Kernel_Name']:
        per[(r['Kernel_Name'][6:24], int(r['Grid_Size_X']) // 256)].append(d)
print('busy ms', round(sum(v[1] for v in agg.values()) / 1e3, 3))
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:8]:
    print(f"{k:50s} {v[0]:5d} {v[1] / 1e3:8.3f} ms")
if len(sys.argv) > 2:
    for k, v in sorted(per.items()):
        print(k, 'n', len(v), 'avg %.1f' % (sum(v) / len(v)))
