"""Time mdx_gemm_f32 on a few shapes (HIP events, 10 launches after 3);
MDX_PP_VAR selects a variant of the kernel (gemm_pp.hip); --noepi skips
the epilogue stores.
Usage: MDX_PP_VAR=n python tools/ppdiag.py [--zeros] [--noepi]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = [("box_fc1", 32000, 1024, 12544, 1), ("wino6_p2", 13376, 256, 256, 64), ("res4_conv3", 28672, 1024, 256, 1),
          ("big_sq", 8192, 8192, 8192, 1)]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, M, N, K, B in SHAPES:
        if "--zeros" in sys.argv:
            A = torch.zeros(B, M, K, device="cuda")
            W = torch.zeros(B, N, K, device="cuda")
        else:
            A = torch.randn(B, M, K, device="cuda")
            W = torch.randn(B, N, K, device="cuda")
        C = torch.empty(B, M, N, device="cuda")

        def go():
            call("mdx_gemm_f32", P(A), P(W), None, None, 2 if "--noepi" in sys.argv else 0, P(C), M, N, K, B,
                 M * K, N * K, M * N, None)
        for _ in range(3):
            go()
        e0.record()
        for _ in range(10):
            go()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10 * 1e-3
        print(json.dumps({"var": os.environ.get("MDX_PP_VAR", "0"), "noepi": "--noepi" in sys.argv, "name": name,
                          "us": round(t * 1e6, 1), "tflops": round(2.0 * M * N * K * B / t / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
