"""Occupancy of a rocprofv3 kernel trace: wall time with >= 1 kernel running,
per-stream busy time, and which kernels run while only one is resident
(the exposed ones).  Usage: python tools/timeline.py run_kernel_trace.csv [t0_frac]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev.append((s, e, r["Kernel_Name"][:60], r.get("Stream_Id", r.get("Queue_Id", "?"))))
ev.sort()
t0 = ev[0][0] + (ev[-1][1] - ev[0][0]) * float(sys.argv[2] if len(sys.argv) > 2 else 0.5)
ev = [x for x in ev if x[0] >= t0]
T0, T1 = ev[0][0], max(e for _, e, _, _ in ev)
pts = []
for s, e, n, q in ev:
    pts.append((s, 1, n))
    pts.append((e, -1, n))
pts.sort(key=lambda p: (p[0], p[1]))
active = defaultdict(int)
busy = alone = 0
alone_by = defaultdict(int)
last = T0
depth = 0
for t, d, n in pts:
    dt = t - last
    if depth > 0:
        busy += dt
    if depth == 1:
        k = [k for k, v in active.items() if v > 0][0]
        alone += dt
        alone_by[k] += dt
    active[n] += d
    depth += d
    last = t
wall = T1 - T0
print(f"window {wall/1e6:.2f} ms  busy {busy/wall:.3f}  single-kernel {alone/wall:.3f}")
perq = defaultdict(int)
for s, e, n, q in ev:
    perq[q] += e - s
for q, v in sorted(perq.items()):
    print(f"  queue/stream {q}: kernel time {v/wall:.3f} of wall")
print("exposed (alone on the GPU) by kernel, % of wall:")
for k, v in sorted(alone_by.items(), key=lambda x: -x[1])[:15]:
    print(f"  {100*v/wall:6.2f}  {k}")
