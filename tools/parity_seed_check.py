"""Run tests/test_parity_full.py's comparison for several R50 weight seeds on
the GPU and print each case's summary (frames passing the detection / pose
checks, identical selected masks, poses) -- how the parity seed of a dtype
was chosen.  Usage: python tools/parity_seed_check.py DTYPE WINO seed [seed ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import mdx_pkg
    mdx_pkg.load()
    import test_parity_full as T
    from moseq2_detectron_extract_amd._lib import call
    dtype, wino = sys.argv[1], int(sys.argv[2])
    from moseq2_detectron_extract_amd._lib import knob
    old = knob("winograd", wino)
    try:
        for seed in (int(v) for v in sys.argv[3:]):
            T._ORACLE.clear()
            try:
                T._forward_full_frame(50, 32, dtype, wino, 0, seed)
                res = "pass"
            except AssertionError as e:
                res = "fail: " + str(e)[:160]
            out = os.path.join(ROOT, "gpurun_out", f"parity_full_R50_B32_{dtype}" + (f"_wino{wino}" if wino else "") +
                               f"_s{seed}.json")
            summ = json.load(open(out))["summary"] if os.path.exists(out) else None
            print(json.dumps({"seed": seed, "dtype": dtype, "wino": wino, "result": res, "summary": summ}), flush=True)
    finally:
        knob("winograd", old)


if __name__ == "__main__":
    main()
