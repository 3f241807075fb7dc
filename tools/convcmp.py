"""Compare two per-conv timing dumps (bench.py --dump-convs): per layer and total."""
import json
import sys

names = {0: 'c128', 1: 'c64', 2: 'g256', 3: 'g128', 6: 'wino', 7: 'x3_128', 8: 'x3_64', 9: 'x6dma', 5: 'head', 4: 'strm'}
a = json.load(open(sys.argv[1]))
b = json.load(open(sys.argv[2]))
ta = tb = 0
for r, s in zip(a, b):
    ta += r['us']
    tb += s['us']
    d = s['us'] - r['us']
    if abs(d) > float(sys.argv[3]) if len(sys.argv) > 3 else True:
        print(f"M={r['M']:7d} N={r['N']:5d} K={r['K']:6d} {names.get(r['kernel'], r['kernel']):5s} {r['us']:8.1f} -> "
              f"{names.get(s['kernel'], s['kernel']):5s} {s['us']:8.1f} us ({d:+.1f})")
print(f"total {ta:.1f} -> {tb:.1f} us")
