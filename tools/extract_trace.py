"""Summarise an MDX_EXTRACT_TRACE timeline (moseq2-detectron-extract_amd/extract.py
``_Timeline``): per-phase mean/total wall time and the fraction of the loop
each thread was busy.

    python tools/extract_trace.py gpurun_out/extract_trace.json
"""
import json
import sys
from collections import defaultdict


def main():
    doc = json.load(open(sys.argv[1]))
    ev = doc["events"]
    total = doc["total_s"]
    per = defaultdict(list)
    for e in ev:
        per[e["phase"]].append(e["end_s"] - e["start_s"])
    print(f"loop wall {total:.3f} s, {len(per.get('device pass', []))} chunks")
    worker = 0.0
    for name, ds in per.items():
        s = sum(ds)
        if name != "device pass":
            worker += s
        print(f"{name:20s} n={len(ds):4d} mean {1e3 * s / len(ds):8.2f} ms  "
              f"total {s:7.3f} s ({100 * s / total:5.1f} % of loop)")
    print(f"worker busy {worker:.3f} s ({100 * worker / total:.1f} %)")
    # worker idle gaps between chunks: time from finishing chunk k to starting k+1
    starts = sorted(e["start_s"] for e in ev if e["phase"] == "instance selection")
    ends = sorted(e["end_s"] for e in ev if e["phase"] == "writer hand-off")
    gaps = [b - a for a, b in zip(ends, starts[1:])]
    if gaps:
        print(f"worker gap between chunks: mean {1e3 * sum(gaps) / len(gaps):.2f} ms, "
              f"max {1e3 * max(gaps):.2f} ms")


if __name__ == "__main__":
    main()
