"""Per-dispatch FETCH_SIZE / WRITE_SIZE of the conv kernels in rocprofv3
counter_collection CSVs (FETCH_SIZE doubled on gfx950, MI355X_MICROARCH.md
'HBM'), as GB per launch.  Usage: python tools/pmc_dispatch.py CSV..."""
import collections
import csv
import json
import sys


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "k_conv" not in name and "k_roi" not in name and "k_gemm" not in name:
                continue
            c = r["Counter_Name"]
            v = float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
            per[name[:70]][c].append(v / 1e9)
    out = {k: {c: [round(x, 3) for x in v] for c, v in d.items()} for k, d in per.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
