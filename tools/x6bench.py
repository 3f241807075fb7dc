"""Time mdx_gemm_x6 (+ the activation split) against the fp32 conv path on
the model's GEMM shapes.  Usage: python tools/x6bench.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mdx_pkg  # noqa: E402

mdx_pkg.load()
from moseq2_detectron_extract_amd._lib import call  # noqa: E402

P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


rows = []
for M, N, K in [(32000, 1024, 12544), (32000, 1024, 1024), (28672, 256, 256), (7168, 512, 512), (114688, 256, 256)]:
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(N, device="cuda")
    pa = torch.empty(call("mdx_x6_plane_bytes", M, K), dtype=torch.uint8, device="cuda")
    pb = torch.empty(call("mdx_x6_plane_bytes", N, K), dtype=torch.uint8, device="cuda")
    out = torch.empty(M, N, device="cuda")
    call("mdx_split_x6", P(B), N, K, K, P(pb), None)
    t_split = timeit(lambda: call("mdx_split_x6", P(A), M, K, K, P(pa), None))
    t_x6 = timeit(lambda: call("mdx_gemm_x6", P(pa), P(pb), P(bias), M, N, K, None, 1, P(out), None))
    t_f32 = timeit(lambda: call("mdx_conv2d", P(A), M, 1, 1, K, P(B), P(bias), N, 1, 1, 1, 0, None, 1, 0, 0, 0, P(out), None))
    fl = 2.0 * M * N * K
    r = {"M": M, "N": N, "K": K, "split_us": round(t_split, 1), "x6_us": round(t_x6, 1), "f32_us": round(t_f32, 1),
         "x6_tflops": round(fl / t_x6 / 1e6, 1), "f32_tflops": round(fl / t_f32 / 1e6, 1),
         "split_gbps": round(M * K * 10 / t_split / 1e3, 1)}
    print(json.dumps(r), flush=True)
    del A, B, pa, pb, out
