"""Per-kernel SQ / GRBM counter totals from rocprofv3 --pmc counter_collection
CSVs (one or more passes), with the ratios used to read them:
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs), wait
fractions = SQ_WAIT_* / SQ_WAVE_CYCLES.  Usage: python tools/pmc_sq.py CSV..."""
import collections
import csv
import json
import sys

SIMDS = 1024


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((path, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    out = {}
    for k, c in tot.items():
        d = {n: v for n, v in c.items()}
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g * SIMDS)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in c:
                    d[n.lower() + "_frac"] = c[n] / wc
        if c.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_cycles_per_lds_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"]
        d["dispatch_records"] = len(disp[k])
        out[k[:90]] = d
    for k, d in sorted(out.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[:12]:
        print(k, json.dumps({n: (round(v, 4) if isinstance(v, float) else v) for n, v in d.items()}))


if __name__ == "__main__":
    main()
