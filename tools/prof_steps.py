"""Per-step kernel time from a rocprofv3 kernel trace (steady state: the
median step, warmup excluded).  Usage: python tools/prof_steps.py TRACE_CSV [N]"""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        if "k_prep(" in r["Kernel_Name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    steps.append(cur)
    steps = [s for s in steps if any("k_conv" in r["Kernel_Name"] for r in s)]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3 for s in steps]
    med = sorted(range(len(steps)), key=lambda i: busy[i])[len(steps) // 2]
    s = steps[med]
    per = collections.defaultdict(lambda: [0.0, 0])
    for r in s:
        k = r["Kernel_Name"]
        per[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        per[k][1] += 1
    print(f"steps {len(steps)}, busy per step (us): {[round(b) for b in busy]}; median step {busy[med]:.1f} us")
    for k, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t:9.1f} us  {n:3d} calls  {k[:100]}")


if __name__ == "__main__":
    main()
