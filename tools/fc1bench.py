"""Box head fc1 on its own: the fp32 GEMM of the R50-FPN B=32 forward
(32000 pooled ROIs x 12544 -> 1024, + bias + ReLU) through mdx_conv2d_splitk,
HIP events over REPS launches.  Run under rocprofv3 --pmc FETCH_SIZE (or
WRITE_SIZE) to read its HBM bytes per launch apart from every other launch of
the same kernel symbol.  Knobs: field=value[,threshold] sets that field of the thread's kernel-selection policy.
Usage: python tools/fc1bench.py [reps] [knob=value ...]"""
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
    from moseq2_detectron_extract_amd._lib import call, knob
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 10
    for kv in [a for a in sys.argv[1:] if "=" in a]:
        name, val = kv.split("=")
        knob(name, *[int(v) for v in val.split(",")])
    M, N, K = int(os.environ.get("FC1_M", 32000)), 1024, 12544
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * (2.0 / K) ** 0.5
    b = torch.randn(N, device="cuda", generator=g) * 0.02
    out = torch.empty(M, N, device="cuda")
    ws = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")

    def go():
        call("mdx_conv2d_splitk", P(x), M, 1, 1, K, P(w), P(b), N, 1, 1, 1, 0, None, 1, 0, 0, 0, P(out), 0, P(ws),
             ws.numel(), None)

    for _ in range(2):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) * 1e-3 / reps
    kid, ks = ctypes.c_int(), ctypes.c_int()
    call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ks))
    ref = torch.relu(x[:256].double() @ w.double().t() + b.double())
    err = ((out[:256].double() - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"M": M, "N": N, "K": K, "kernel": kid.value, "ksplit": ks.value, "us": round(s * 1e6, 1),
                      "tflops": round(2.0 * M * N * K / s / 1e12, 2), "frac_f32_peak": round(2.0 * M * N * K / s / 157.3e12, 4),
                      "operand_bytes": (M * K + N * K + M * N) * 4, "rel_err_vs_fp64": err}), flush=True)


if __name__ == "__main__":
    main()
