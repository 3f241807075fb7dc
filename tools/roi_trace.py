"""Per-launch ROIAlign durations from rocprofv3 kernel-trace CSVs: for each
file, the mean / min of every ROIAlign instance's launches grouped by grid
size (the box pooler is the 32 000-workgroup launch), and the total of all
kernels.  Usage: python tools/roi_trace.py TRACE.csv [TRACE.csv ...]"""
import collections
import csv
import sys


def main():
    for path in sys.argv[1:]:
        d = collections.defaultdict(list)
        total = 0.0
        for r in csv.DictReader(open(path)):
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            total += us
            if "roi_align" in r["Kernel_Name"]:
                grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
                d[(r["Kernel_Name"].split("(")[0], grid, int(r["Grid_Size_Y"]))].append(us)
        print(path)
        for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            print(f"  {k[0][:60]:60s} grid {k[1]:6d} x {k[2]}  n {len(v):3d}  mean {sum(v) / len(v):8.1f} us"
                  f"  min {min(v):8.1f}")
        print(f"  all kernels {total / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
