import csv, sys
f = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6/steps:.2f} ms/step")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r['Name'][:90]
    print(f"{float(r['TotalDurationNs'])/1e3/steps:9.1f} us/step  calls/step {int(r['Calls'])/steps:6.1f}  avg {float(r['AverageNs'])/1e3:8.1f} us  {n}")
