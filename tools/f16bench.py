"""fp16 GEMM layers of the fp16 / mixed models: each shape through
mdx_conv2d_splitk under the default policy (the kernel it picks, from
mdx_conv2d_last_plan) beside torch.matmul on the GEMM of the same M, N, K
(hipBLASLt), HIP events.  Usage: python tools/f16bench.py [field=value ...]
(fields of mdx_policy, e.g. large_tiles=0; only=box_fc1,... picks shapes)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [
    # name, N, H, W, Cin, Cout, k, pad
    ("box_fc1", 32000, 1, 1, 12544, 1024, 1, 0),
    ("box_fc2", 32000, 1, 1, 1024, 1024, 1, 0),
    ("fpn_out_p2", 32, 112, 128, 256, 256, 3, 1),
    ("fpn_lat_p2", 32, 112, 128, 256, 256, 1, 0),
    ("res4_conv2", 32, 28, 32, 256, 256, 3, 1),
    ("mask_conv_b64", 256, 14, 14, 256, 256, 3, 1),
    ("kp_conv_b64", 256, 14, 14, 512, 512, 3, 1),
]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call, knob
    only = None
    for kv in sys.argv[1:]:
        name, val = kv.split("=")
        if name == "only":
            only = val.split(",")
            continue
        knob(name, int(val))
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ws = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps=10):
        for _ in range(3):
            fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    for name, N, H, W, Cin, Cout, k, p in SHAPES:
        if only and name not in only:
            continue
        OH, OW = H + 2 * p - k + 1, W + 2 * p - k + 1
        M, K = N * OH * OW, k * k * Cin
        x = (torch.rand(N, H, W, Cin, device="cuda") * 2 - 1).half()
        w = ((torch.rand(Cout, K, device="cuda") * 2 - 1) / K ** 0.5).half()
        b = torch.rand(Cout, device="cuda")
        out = torch.empty(N, OH, OW, Cout, device="cuda").half()
        flops = 2.0 * M * Cout * K

        def ours():
            call("mdx_conv2d_splitk", P(x), N, H, W, Cin, P(w), P(b), Cout, k, k, 1, p, None, 1, 0, 1, 1,
                 P(out), 0, P(ws), ws.numel(), None)
        t = timed(ours)
        kern, ks = ctypes.c_int(), ctypes.c_int()
        call("mdx_conv2d_last_plan", ctypes.byref(kern), ctypes.byref(ks))
        a = (torch.rand(M, K, device="cuda") * 2 - 1).half()
        bt = w.t()
        tt = timed(lambda: torch.matmul(a, bt))
        print(json.dumps({"name": name, "M": M, "N": Cout, "K": K, "kernel": kern.value, "ksplit": ks.value,
                          "us": round(t * 1e6, 1), "tflops": round(flops / t / 1e12, 1),
                          "frac": round(flops / t / 1e12 / 2500, 3), "torch_us": round(tt * 1e6, 1),
                          "torch_tflops": round(flops / tt / 1e12, 1)}), flush=True)
        del a, x, w, out


if __name__ == "__main__":
    main()
