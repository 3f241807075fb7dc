"""Time single conv launches of chosen shapes under each kernel policy.
Usage: python tools/convbench.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [
    # N, H, W, Cin, Cout, k, stride, pad, residual
    (32, 112, 128, 64, 256, 1, 1, 0, True),     # res2 conv3
    (32, 112, 128, 64, 256, 1, 1, 0, False),    # res2 shortcut
    (32, 112, 128, 256, 256, 1, 1, 0, False),   # fpn lateral p2
    (32, 112, 128, 256, 64, 1, 1, 0, False),    # res2 conv1
    (32, 112, 128, 64, 64, 3, 1, 1, False),     # res2 conv2
    (32, 112, 128, 256, 256, 3, 1, 1, False),   # fpn output p2
    (32, 56, 64, 128, 512, 1, 1, 0, True),      # res3 conv3
    (32000, 1, 1, 12544, 1024, 1, 1, 0, False),  # fc1
    (32, 225, 257, 16, 64, 4, 1, 1, False),     # stem (space-to-depth 4x4)
    (32, 112, 128, 256, 15, 1, 1, 0, False),    # rpn head p2
    (32, 28, 32, 256, 1024, 1, 1, 0, True),     # res4 conv3
]


def main():
    only = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else None
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    from moseq2_detectron_extract_amd._lib import knob
    for kv in sys.argv[2:]:  # field=value of the kernel-selection policy, e.g. dma_f32=2
        name, val = kv.split("=")
        knob(name, int(val))
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ws = torch.empty(64 << 18, dtype=torch.float32, device="cuda")
    copy_src = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    copy_dst = torch.empty_like(copy_src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        copy_dst.copy_(copy_src)
    e0.record()
    for _ in range(10):
        copy_dst.copy_(copy_src)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10
    print(f"torch copy 256 MiB: {t * 1e3:.1f} us = {2 * (256 << 20) / t / 1e9:.2f} TB/s (read+write)")
    for si, (N, H, W, Cin, Cout, k, s, p, res) in enumerate(SHAPES):
        if only is not None and si not in only:
            continue
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Cin, device="cuda").half()
        w = (torch.randn(Cout, k * k * Cin, device="cuda") / (k * k * Cin) ** 0.5).half()
        b = torch.randn(Cout, device="cuda")
        r = torch.randn(N, OH, OW, Cout, device="cuda").half() if res else None
        out = torch.empty(N, OH, OW, Cout, device="cuda").half()
        M = N * OH * OW
        flops = 2.0 * M * Cout * k * k * Cin
        byts = 2.0 * (x.numel() + w.numel() + out.numel() + (r.numel() if res else 0))
        line = f"M={M:7d} N={Cout:5d} K={k * k * Cin:6d} res={int(res)}:"
        for mode, nk in ((0, 0), (2, 0)):
            old = knob("large_tiles", mode)

            def go():
                call("mdx_conv2d_splitk", P(x), N, H, W, Cin, P(w), P(b), Cout, k, k, s, p, P(r), 1, 0, 1, 1,
                     P(out), 0, P(ws), ws.numel() * 4, None)
            for _ in range(3):
                go()
            e0.record()
            for _ in range(10):
                go()
            e1.record()
            torch.cuda.synchronize()
            knob("large_tiles", old)
            t = e0.elapsed_time(e1) / 10 * 1e-3
            line += f"  [{'64' if nk else ('128' if mode == 0 else '256')}] {t * 1e6:7.1f}us {flops / t / 1e12:6.1f}TF {byts / t / 1e12:5.2f}TB/s"
        print(line, flush=True)


if __name__ == "__main__":
    main()
