"""Per-kernel HBM bytes per launch from a FETCH_SIZE and a WRITE_SIZE
rocprofv3 pass (KiB; FETCH_SIZE doubled, MI355X_MICROARCH.md 'HBM').
Usage: python tools/inp_pmc.py FETCH_CSV WRITE_CSV [substring ...]"""
import collections
import csv
import sys


def load(path, counter):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            tot[r["Kernel_Name"]] += float(r["Counter_Value"])
            disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return {k: tot[k] * 1024 / len(disp[k]) for k in tot}


def main():
    f, w = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    subs = sys.argv[3:]
    total = 0.0
    for k in sorted(set(f) | set(w)):
        if subs and not any(s in k for s in subs):
            continue
        b = 2 * f.get(k, 0.0) + w.get(k, 0.0)
        total += b
        print(f"{k[:60]:60s} fetch {2 * f.get(k, 0) / 1e6:8.3f} MB  write {w.get(k, 0) / 1e6:8.3f} MB")
    print(f"total {total / 1e6:.3f} MB per launch set")


if __name__ == "__main__":
    main()
