"""Per-stream activity segments of a rocprofv3 kernel trace (late part of the run)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Stream_Id'], r['Kernel_Name'][:30]) for r in rows)
T1 = max(e for _, e, _, _ in ev)
T0 = ev[0][0]
start = T0 + (T1 - T0) * float(sys.argv[2] if len(sys.argv) > 2 else 0.85)
sel = [x for x in ev if x[0] >= start]
b = sel[0][0]
seg = collections.defaultdict(list)
for s, e, q, n in sel:
    L = seg[q]
    if L and s - L[-1][1] < 30000:
        L[-1][1] = max(L[-1][1], e)
        L[-1][2] += 1
    else:
        L.append([s, e, 1, n])
for q in sorted(seg):
    print("stream", q)
    for s, e, c, n in seg[q][:10]:
        print(f"   {(s - b) / 1000:9.1f} -> {(e - b) / 1000:9.1f}  ({(e - s) / 1000:7.1f} us, {c} kernels) first={n}")
