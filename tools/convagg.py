"""Aggregate a bench --dump-convs JSON by layer shape (time, launches, TF/s, HBM-bound GB/s)."""
import json
import sys

d = json.load(open(sys.argv[1]))
tot = sum(x['us'] for x in d)
print(f"total {tot:.0f} us over {len(d)} launches")
agg = {}
for x in d:
    key = (x['M'], x['N'], x['K'], x['k'], x['stride'], x['res'], x['kernel'], x['ksplit'])
    a = agg.setdefault(key, [0, 0, 0, 0])
    a[0] += 1
    a[1] += x['us']
    a[2] += 2 * x['M'] * x['N'] * x['K']
    # minimum HBM bytes: input once (M*K/k^2 rows of Cin... approximated by M*K/(k*k)), output, residual
    cin = x['K'] // (x['k'] * x['k'])
    a[3] += 2 * (x['M'] * cin * (x['stride'] ** 2) + x['M'] * x['N'] * (2 if x['res'] else 1))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{v[1]:8.1f} us {v[0]:3d}x  M={k[0]:8d} N={k[1]:5d} K={k[2]:5d} k={k[3]} s={k[4]} res={int(k[5])} "
          f"kern={k[6]} ks={k[7]}  {v[2] / v[1] / 1e6:7.1f} TF  {v[3] / v[1] / 1e3:6.2f} TB/s(min bytes)")
