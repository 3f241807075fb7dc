"""Aggregate a bench --dump-convs JSON by layer shape: time, launches, TF/s.
Usage: python tools/convagg.py CONVS.json [top]"""
import json
import sys

d = json.load(open(sys.argv[1]))
tot = sum(x['us'] for x in d)
print(f"total {tot:.0f} us over {len(d)} launches")
agg = {}
for x in d:
    key = (x['M'], x['N'], x['K'], x['kernel'], x['ksplit'])
    a = agg.setdefault(key, [0, 0.0, 0.0])
    a[0] += 1
    a[1] += x['us']
    a[2] += 2 * x['M'] * x['N'] * x['K']
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{v[1]:8.1f} us {v[0]:3d}x  M={k[0]:8d} N={k[1]:5d} K={k[2]:5d} kern={k[3]} ks={k[4]}  "
          f"{v[2] / v[1] / 1e6:7.1f} TF")
