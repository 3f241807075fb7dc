"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE collections into HBM
bytes per bench step for the conv kernels (and the top kernels overall).

Usage: python tools/pmc_summary.py FETCH_CSV WRITE_CSV STEPS OUT_JSON
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950 tallies
128-B read requests at 64 B, MI355X_MICROARCH.md 'HBM').
"""
import collections
import csv
import json
import sys


def load(path, counter):
    per = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        per[k] += float(r["Counter_Value"])
        calls[k] += 1
    return per, calls


def main():
    fpath, wpath, steps, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    fetch, fcalls = load(fpath, "FETCH_SIZE")
    write, _ = load(wpath, "WRITE_SIZE")
    kernels = {}
    for k in set(fetch) | set(write):
        b = 2 * fetch.get(k, 0.0) * 1024 + write.get(k, 0.0) * 1024
        kernels[k] = {"hbm_bytes_per_step": b / steps, "fetch_bytes_per_step": 2 * fetch.get(k, 0.0) * 1024 / steps,
                      "write_bytes_per_step": write.get(k, 0.0) * 1024 / steps, "launches_per_step": fcalls[k] / steps}
    conv = [v for k, v in kernels.items() if "k_conv" in k]
    summary = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py steps",
        "steps": steps,
        "hbm_bytes_per_step": sum(v["hbm_bytes_per_step"] for v in conv),
        "conv_launches_per_step": sum(v["launches_per_step"] for v in conv),
        "top_kernels": dict(sorted(((k[:80], v) for k, v in kernels.items()),
                                   key=lambda kv: -kv[1]["hbm_bytes_per_step"])[:15]),
    }
    summary["kernels"] = {k: {"hbm_bytes_per_launch": v["hbm_bytes_per_step"] / max(v["launches_per_step"], 1e-9),
                              "fetch_bytes_per_launch": v["fetch_bytes_per_step"] / max(v["launches_per_step"], 1e-9),
                              "write_bytes_per_launch": v["write_bytes_per_step"] / max(v["launches_per_step"], 1e-9),
                              "launches_per_step": v["launches_per_step"]}
                          for k, v in kernels.items()}
    with open(out, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({k: summary[k] for k in ("hbm_bytes_per_step", "conv_launches_per_step")}))


if __name__ == "__main__":
    main()
