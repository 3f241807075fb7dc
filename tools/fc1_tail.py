"""Box head fc1 (M ROIs x K 12544 -> N 1024, fp32) through mdx_conv2d_splitk
at several M and split-K counts, HIP events over 5 launches: how much of
fc1's distance from the f32 peak is the last, partly filled round of
workgroups (tile-count quantisation) rather than the K loop itself.
Usage: python tools/fc1_tail.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    K, N = int(os.environ.get("FC_K", 12544)), int(os.environ.get("FC_N", 1024))
    Ms = [int(v) for v in os.environ.get("FC_M", "24576,27648,30720,32000,32768,36864").split(",")]
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    ws = torch.empty(4 * max(Ms) * N * 4, dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kid, ks = ctypes.c_int(), ctypes.c_int()
    for M in Ms:
        x = torch.randn(M, K, device="cuda")
        out = torch.empty(M, N, device="cuda")
        for split in (1, 2, 3, 4):
            def go():
                call("mdx_conv2d_splitk", P(x), M, 1, 1, K, P(w), P(b), N, 1, 1, 1, 0, None, 1, 0, 0, 0, P(out),
                     split, P(ws), ws.numel(), None)
            for _ in range(2):
                go()
            e0.record()
            for _ in range(5):
                go()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 5 * 1e-3
            call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ks))
            print(json.dumps({"M": M, "N": N, "K": K, "ksplit_req": split, "kernel": kid.value, "ksplit": ks.value,
                              "tiles": ((M + 127) // 128) * ((N + 127) // 128), "us": round(t * 1e6, 1),
                              "tflops": round(2.0 * M * N * K / t / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
