"""Time mid-size conv layers of the bench workload at several split-K factors
and tile policies.  Usage: python tools/splitkbench.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [
    # N, H, W, Cin, Cout, k, stride, pad
    (32, 28, 32, 256, 256, 3, 1, 1),     # res4 conv2
    (128, 7, 7, 512, 512, 3, 1, 1),      # keypoint head conv
    (32, 56, 64, 128, 128, 3, 1, 1),     # res3 conv2
    (128, 14, 14, 256, 256, 3, 1, 1),    # mask head conv
    (32, 28, 32, 1024, 256, 1, 1, 0),    # res4 conv1
    (32, 14, 16, 512, 2048, 1, 1, 0),    # res5 conv3
    (32, 14, 16, 512, 512, 3, 1, 1),     # res5 conv2
    (32, 112, 128, 256, 256, 3, 1, 1),   # FPN output / RPN conv p2
    (32, 56, 64, 256, 256, 3, 1, 1),     # FPN output / RPN conv p3
    (32000, 1, 1, 12544, 1024, 1, 1, 0),  # box fc1
    (32, 112, 128, 256, 256, 1, 1, 0),   # FPN lateral p2
]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ws = torch.empty(64 << 18, dtype=torch.float32, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for (N, H, W, Cin, Cout, k, s, p) in SHAPES:
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Cin, device="cuda").half()
        w = (torch.randn(Cout, k * k * Cin, device="cuda") / (k * k * Cin) ** 0.5).half()
        b = torch.randn(Cout, device="cuda")
        out = torch.empty(N, OH, OW, Cout, device="cuda").half()
        M = N * OH * OW
        flops = 2.0 * M * Cout * k * k * Cin
        line = f"M={M:6d} N={Cout:5d} K={k * k * Cin:5d}:"
        for mode, ks in ((1, 0), ("prio", 0), ("dma128", 0), ("dma128prio", 0)):
            oldp = call("mdx_conv_set_mfma_prio", 1 if "prio" in str(mode) else 0)
            if mode == "prio":
                mode = 1
            old_d = call("mdx_conv_set_dma128", 2 if str(mode).startswith("dma128") else 0, 0)
            if str(mode).startswith("dma128"):
                mode = 1
            old = call("mdx_conv_set_large_tiles", mode)

            def go():
                call("mdx_conv2d_splitk", P(x), N, H, W, Cin, P(w), P(b), Cout, k, k, s, p, None, 1, 0, 1, 1,
                     P(out), ks, P(ws), ws.numel() * 4, None)
            try:
                for _ in range(3):
                    go()
            except Exception as ex:  # split not allowed for this shape
                call("mdx_conv_set_large_tiles", old)
                call("mdx_conv_set_dma128", old_d, 1536)
                line += f"  ks{ks}: n/a"
                continue
            e0.record()
            for _ in range(20):
                go()
            e1.record()
            torch.cuda.synchronize()
            call("mdx_conv_set_large_tiles", old)
            d = call("mdx_conv_set_dma128", old_d, 1536)
            pr = call("mdx_conv_set_mfma_prio", oldp)
            t = e0.elapsed_time(e1) / 20 * 1e-3
            tag = ("dma128" if d == 2 else ("auto" if ks == 0 else f"ks{ks}")) + ("+ilv" if pr else "")
            line += f"  {tag}:{t * 1e6:6.1f}us/{flops / t / 1e12:4.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
