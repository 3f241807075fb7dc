"""Wave-quantisation probe for the fp32 pointwise GEMM (k_conv_sb): each
R50 / box-head GEMM shape at its real M and at nearby M whose 128x128 tile
count is a whole number of per-CU rounds (256 CUs), one launch at a time, HIP
events over 10 launches.  If TFLOP/s at the real M is well below the
whole-round M, the loss is balance, not the inner loop.
Usage: python tools/quant_probe.py [ksplit [name,...]]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # name, M, N, K
    ("box_fc1", 32000, 1024, 12544),
    ("box_fc2", 32000, 1024, 1024),
    ("res3_conv1", 114688, 128, 512),
    ("res4_conv1", 28672, 256, 1024),
    ("res4_conv3", 28672, 1024, 256),
    ("res5_conv1", 7168, 512, 2048),
    ("res5_conv3", 7168, 2048, 512),
]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    ksplit = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ws = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kid, ks = ctypes.c_int(), ctypes.c_int()

    def timeit(fn, reps=10):
        for _ in range(3):
            fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, M0, N, K in SHAPES:
        if only and name not in only:
            continue
        tn = (N + 127) // 128
        tiles0 = (M0 + 127) // 128 * tn
        cands = {M0}
        for rounds in (1, 2, 3, 4, 6, 8, 9, 12):
            t = 256 * rounds
            if t % tn == 0 and 0.4 * tiles0 <= t <= 1.6 * tiles0 and t // tn * 128 * K * 4 < (1 << 31):
                cands.add(t // tn * 128)
        w = torch.randn(N, K, device="cuda") / K ** 0.5
        b = torch.randn(N, device="cuda")
        for M in sorted(cands):
            x = torch.randn(M, K, device="cuda")
            out = torch.empty(M, N, device="cuda")

            def go():
                call("mdx_conv2d_splitk", P(x), M, 1, 1, K, P(w), P(b), N, 1, 1, 1, 0, None, 0, 0, 0, 0, P(out),
                     ksplit, P(ws), ws.numel(), None)
            t = timeit(go)
            call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ks))
            fl = 2.0 * M * N * K
            print(json.dumps({"name": name, "M": M, "real": M == M0, "N": N, "K": K,
                              "tiles": (M + 127) // 128 * tn, "kernel": kid.value, "ksplit": ks.value,
                              "us": round(t * 1e6, 1), "tflops": round(fl / t / 1e12, 1)}), flush=True)
            del x, out


if __name__ == "__main__":
    main()
