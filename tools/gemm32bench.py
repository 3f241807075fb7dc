"""fp32 convolution GEMMs of the R50-FPN B=32 forward, one launch shape at a
time, HIP events over 10 launches: the direct layers through
mdx_conv2d_splitk and the 3x3 layers through mdx_conv3x3_winograd (the tile
the library's Winograd policy picks per layer, mdx_winograd_tile; the
GEMM timed apart from the transforms by the model's profiling hook is not
available here, so the whole layer is timed).  Knobs: name=value calls
sets that field of the thread's kernel-selection policy (mdx_policy) first.
Usage: python tools/gemm32bench.py [knob=value ...]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# N, H, W, Cin, Cout, k, stride, pad, residual, count per forward
DIRECT = [
    (32, 112, 128, 256, 64, 1, 1, 0, False, 2),    # res2 conv1 (blocks 2-3)
    (32, 112, 128, 64, 256, 1, 1, 0, True, 3),     # res2 conv3
    (32, 56, 64, 512, 128, 1, 1, 0, False, 3),     # res3 conv1
    (32, 56, 64, 128, 512, 1, 1, 0, True, 4),      # res3 conv3
    (32, 28, 32, 1024, 256, 1, 1, 0, False, 5),    # res4 conv1
    (32, 28, 32, 256, 1024, 1, 1, 0, True, 6),     # res4 conv3
    (32, 14, 16, 2048, 512, 1, 1, 0, False, 2),    # res5 conv1
    (32, 14, 16, 512, 2048, 1, 1, 0, True, 3),     # res5 conv3
    (32, 112, 128, 256, 256, 1, 1, 0, False, 1),   # fpn lateral p2
    (32, 56, 64, 512, 256, 1, 1, 0, False, 1),     # fpn lateral p3
    (32, 112, 128, 64, 64, 3, 1, 1, False, 3),     # res2 conv2 (direct 3x3)
    (32000, 1, 1, 12544, 1024, 1, 1, 0, False, 1),  # box head fc1 (1000 ROIs x 32 frames)
    (32000, 1, 1, 1024, 1024, 1, 1, 0, False, 1),   # box head fc2
]
WINO = [  # N, H, W, Cin, Cout, count
    (32, 112, 128, 256, 256, 2),   # fpn output p2 + rpn p2
    (32, 56, 64, 256, 256, 2),     # fpn output p3 + rpn p3
    (32, 56, 64, 128, 128, 4),     # res3 conv2
    (32, 28, 32, 256, 256, 8),     # res4 conv2 x6 + fpn p4 + rpn p4
    (32, 14, 16, 512, 512, 3),     # res5 conv2
    (128, 14, 14, 256, 256, 4),    # mask head
    (128, 7, 7, 512, 512, 7),      # keypoint head
    (32, 112, 128, 64, 64, 0),     # res2 conv2 (direct in the model: Cin < winograd_min_cin), for comparison
]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call, knob, policy as current_policy
    for kv in sys.argv[1:]:
        name, val = kv.split("=")
        knob(name, *[int(v) for v in val.split(",")])
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    policy = current_policy()["winograd"] or 4
    need = max([call("mdx_winograd_workspace_bytes", N, H, W, Ci, Co, call("mdx_winograd_tile", H, W, policy))
                for N, H, W, Ci, Co, _ in WINO] + [1 << 28])
    ws = torch.empty(need, dtype=torch.uint8, device="cuda")
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

    res = {"direct": [], "winograd": []}
    tot = wtot = 0.0
    for N, H, W, Cin, Cout, k, s, p, r, cnt in DIRECT:
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Cin, device="cuda")
        w = torch.randn(Cout, k * k * Cin, device="cuda") / (k * k * Cin) ** 0.5
        b = torch.randn(Cout, device="cuda")
        rr = torch.randn(N, OH, OW, Cout, device="cuda") if r else None
        out = torch.empty(N, OH, OW, Cout, device="cuda")
        M = N * OH * OW
        fl = 2.0 * M * Cout * k * k * Cin

        def go():
            call("mdx_conv2d_splitk", P(x), N, H, W, Cin, P(w), P(b), Cout, k, k, s, p, P(rr), 1, 0, 0, 0, P(out), 0,
                 P(ws), ws.numel(), None)
        t = timeit(go)
        call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ks))
        tot += t * cnt
        res["direct"].append({"M": M, "N": Cout, "K": k * k * Cin, "kernel": kid.value, "ksplit": ks.value,
                              "us": round(t * 1e6, 1), "tflops": round(fl / t / 1e12, 1), "count": cnt})
        print(json.dumps(res["direct"][-1]), flush=True)
    for N, H, W, Cin, Cout, cnt in WINO:
        x = torch.randn(N, H, W, Cin, device="cuda")
        w = torch.randn(Cout, Cin, 3, 3) / (9 * Cin) ** 0.5
        m = call("mdx_winograd_tile", H, W, policy)
        U = torch.empty((m + 2) ** 2 * Cout * Cin)
        call("mdx_winograd_weights", P(w), Cout, Cin, m, P(U))
        U = U.cuda()
        b = torch.randn(Cout, device="cuda")
        out = torch.empty(N, H, W, Cout, device="cuda")
        T = N * ((H + m - 1) // m) * ((W + m - 1) // m)
        gfl = 2.0 * (m + 2) ** 2 * T * Cin * Cout

        def go():
            call("mdx_conv3x3_winograd", P(x), N, H, W, Cin, P(U), P(b), Cout, 1, m, P(out), P(ws), ws.numel(), None)
        t = timeit(go)
        tot += t * cnt
        wtot += t * cnt
        res["winograd"].append({"N": N, "H": H, "W": W, "Cin": Cin, "Cout": Cout, "m": m, "us": round(t * 1e6, 1),
                                "gemm_tflops_if_all_gemm": round(gfl / t / 1e12, 1), "count": cnt})
        print(json.dumps(res["winograd"][-1]), flush=True)
    res["weighted_ms_per_forward"] = round(tot * 1e3, 3)
    res["winograd_layers_ms_per_forward"] = round(wtot * 1e3, 3)
    print(json.dumps({"weighted_ms_per_forward": res["weighted_ms_per_forward"],
                      "winograd_layers_ms_per_forward": res["winograd_layers_ms_per_forward"],
                      "policy": policy, "knobs": sys.argv[1:]}), flush=True)


if __name__ == "__main__":
    main()
