"""Device occupancy of a rocprofv3 --kernel-trace CSV: over the window that
holds the last `--tail` fraction of the dispatches (the timed steps of a
bench run), the fraction of wall time with no kernel running, with only
non-GEMM kernels running, and with a GEMM (k_conv* / k_gemm*) running, plus
the longest idle gaps and per-kernel-family busy time.
Usage: python tools/trace_gaps.py KERNEL_TRACE.csv [--tail 0.6]"""
import argparse
import collections
import csv


def family(name: str) -> str:
    base = name.split("(")[0].replace("void ", "")
    return base.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=float, default=0.6)
    args = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(args.csv))]
    rows.sort()
    rows = rows[int(len(rows) * (1 - args.tail)):]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    ev = []
    for s, e, n in rows:
        g = n.startswith(("void mdx::k_conv", "mdx::k_conv", "void mdx::k_gemm", "mdx::k_gemm", "void mdx::k_head"))
        ev.append((s, 1, g))
        ev.append((e, -1, g))
    ev.sort(key=lambda x: (x[0], x[1]))
    busy = gemm = 0
    idle = only_other = with_gemm = 0
    gaps = []
    last = t0
    for t, d, g in ev:
        dt = t - last
        if dt > 0:
            if busy == 0:
                idle += dt
                gaps.append(dt)
            elif gemm == 0:
                only_other += dt
            else:
                with_gemm += dt
        last = t
        busy += d
        gemm += d if g else 0
    wall = t1 - t0
    fam = collections.Counter()
    for s, e, n in rows:
        fam[family(n)] += e - s
    print(f"window {wall / 1e6:.2f} ms, {len(rows)} dispatches")
    print(f"idle {100 * idle / wall:.1f} %  only non-GEMM {100 * only_other / wall:.1f} %  "
          f"GEMM running {100 * with_gemm / wall:.1f} %")
    gaps.sort(reverse=True)
    print("longest idle gaps (us):", [round(g / 1e3, 1) for g in gaps[:10]], f"count {len(gaps)}")
    for f, t in fam.most_common(15):
        print(f"{f:40s} {t / 1e6:8.2f} ms summed")


if __name__ == "__main__":
    main()
