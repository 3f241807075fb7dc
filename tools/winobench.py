"""Fused Winograd F(4,3) (k_wino_f4) vs the three-launch path on the
R50-FPN Keypoint R-CNN 3x3 layer shapes of a 32-frame batch (fp32): per
layer us of each, and the per-forward total (layer count as in one forward).

    python tools/winobench.py [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mdx_pkg  # noqa: E402
mdx_pkg.load()
from moseq2_detectron_extract_amd._lib import call  # noqa: E402

# (name, N, H, W, Cin, Cout, layers per forward)
LAYERS = [("res2", 32, 112, 128, 64, 64, 3), ("res3", 32, 56, 64, 128, 128, 4), ("res4", 32, 28, 32, 256, 256, 6),
          ("res5", 32, 14, 16, 512, 512, 3), ("fpn_p2", 32, 112, 128, 256, 256, 1),
          ("fpn_p3", 32, 56, 64, 256, 256, 1), ("fpn_p4", 32, 28, 32, 256, 256, 1), ("fpn_p5", 32, 14, 16, 256, 256, 1),
          ("rpn_p2", 32, 112, 128, 256, 256, 1), ("rpn_p3", 32, 56, 64, 256, 256, 1),
          ("rpn_p4", 32, 28, 32, 256, 256, 1), ("rpn_p5", 32, 14, 16, 256, 256, 1), ("rpn_p6", 32, 7, 8, 256, 256, 1),
          ("mask", 128, 14, 14, 256, 256, 4), ("kp_in", 32, 14, 14, 256, 512, 1), ("kp", 32, 14, 14, 512, 512, 7)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows, tot = [], {"fused": 0.0, "unfused": 0.0, "best": 0.0}
    for name, N, H, W, Cin, Cout, cnt in LAYERS:
        if args.only and name not in args.only.split(","):
            continue
        g = torch.Generator().manual_seed(1)
        x = torch.randn(N, H, W, Cin, generator=g).clamp_min(0).cuda()
        w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5).numpy()
        b = torch.randn(Cout, generator=g).cuda()
        out = torch.empty(N, H, W, Cout, device="cuda")
        res = {}
        m6 = call("mdx_winograd_tile", H, W, 6)
        for mode, m in (("unfused", m6), ("unfused4", 4), ("fused", 4)):
            U = np.empty(((m + 2) ** 2, Cout, Cin), np.float32)
            call("mdx_winograd_weights", w.ctypes.data_as(ctypes.c_void_p), Cout, Cin, m, U.ctypes.data_as(ctypes.c_void_p))
            if mode == "fused":
                Up = np.empty_like(U)
                call("mdx_winograd_pack_f4", U.ctypes.data_as(ctypes.c_void_p), Cout, Cin,
                     Up.ctypes.data_as(ctypes.c_void_p))
                Ud = torch.from_numpy(Up).cuda()
                res[mode] = timed(lambda: call("mdx_conv3x3_winograd_fused", P(x), N, H, W, Cin, P(Ud), P(b), Cout, 1,
                                               P(out), stream), args.reps)
                continue
            Ud = torch.from_numpy(U).cuda()
            nb = call("mdx_winograd_workspace_bytes", N, H, W, Cin, Cout, m)
            ws = torch.empty(nb // 4 + 4, dtype=torch.float32, device="cuda")
            res[mode] = timed(lambda: call("mdx_conv3x3_winograd", P(x), N, H, W, Cin, P(Ud), P(b), Cout, 1, m,
                                           P(out), P(ws), nb, stream), args.reps)
            del ws, Ud
        T4 = N * ((H + 3) // 4) * ((W + 3) // 4)
        fl = 2.0 * 36 * T4 * Cin * Cout
        r = {"layer": name, "N": N, "H": H, "W": W, "Cin": Cin, "Cout": Cout, "count": cnt, "m_unfused": m6,
             "wgs_fused": -(-T4 // 32) * (Cout // 32), **{k: round(v, 1) for k, v in res.items()},
             "fused_tflops": round(fl / res["fused"] / 1e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
        tot["fused"] += cnt * res["fused"]
        tot["unfused"] += cnt * res["unfused"]
        tot["best"] += cnt * min(res["fused"], res["unfused"])
    print(json.dumps({"per_forward_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
