"""The ping-pong fp32 GEMM (mdx_gemm_f32, csrc/gemm_pp.hip) on the R50-FPN
B=32 GEMM shapes: error against an fp64 matmul of the same operands, and
time (HIP events, 10 launches after 3) against the register-staged kernel the
layer uses today (mdx_conv2d_splitk on the same shape as a pointwise layer)
and torch.matmul (hipBLASLt, exact fp32).
Usage: python tools/ppbench.py [--quick] [--no-torch]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name, M, N, K, batch, residual, count per forward
SHAPES = [
    ("box_fc1", 32000, 1024, 12544, 1, False, 1),
    ("box_fc2", 32000, 1024, 1024, 1, False, 1),
    ("wino6_p2", 13376, 256, 256, 64, False, 2),
    ("wino6_p3", 3520, 256, 256, 64, False, 2),
    ("wino6_res3", 3520, 128, 128, 64, False, 4),
    ("wino4_res4", 1792, 256, 256, 36, False, 8),
    ("wino4_res5", 512, 512, 512, 36, False, 3),
    ("wino4_mask", 2048, 256, 256, 36, False, 4),
    ("wino4_kp", 512, 512, 512, 36, False, 7),
    ("p2_lateral", 458752, 256, 256, 1, False, 1),
    ("p3_lateral", 114688, 256, 512, 1, False, 1),
    ("res3_conv1", 114688, 128, 512, 1, False, 3),
    ("res3_conv3", 114688, 512, 128, 1, True, 4),
    ("res4_conv1", 28672, 256, 1024, 1, False, 5),
    ("res4_conv3", 28672, 1024, 256, 1, True, 6),
    ("res5_conv1", 7168, 512, 2048, 1, False, 2),
    ("res5_conv3", 7168, 2048, 512, 1, True, 3),
]
RAGGED = [("ragged_a", 1000, 300, 64, 1, True, 0), ("ragged_b", 257, 257, 32, 3, False, 0),
          ("ragged_c", 300, 520, 96, 1, False, 0), ("tiny", 5, 7, 32, 1, True, 0)]


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    quick = "--quick" in sys.argv
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ws = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
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

    g = torch.Generator(device="cuda").manual_seed(0)
    tot = {"pp": 0.0, "cur": 0.0, "torch": 0.0}
    for name, M, N, K, B, res, cnt in RAGGED + ([] if quick else SHAPES):
        A = torch.randn(B, M, K, device="cuda", generator=g)
        W = torch.randn(B, N, K, device="cuda", generator=g) / K ** 0.5
        bias = torch.randn(N, device="cuda", generator=g)
        R = torch.randn(M, N, device="cuda", generator=g) if res else None
        C = torch.empty(B, M, N, device="cuda")
        relu = 1

        def pp():
            call("mdx_gemm_f32", P(A), P(W), P(bias), P(R), relu, P(C), M, N, K, B, M * K, N * K, M * N, None)
        pp()
        torch.cuda.synchronize()
        # fp64 reference of the same fp32 operands
        ref = torch.matmul(A.double(), W.double().transpose(1, 2)) + bias.double()
        if R is not None:
            ref = ref + R.double()
        ref = ref.clamp_min(0)
        scale = (A.double().abs() @ W.double().abs().transpose(1, 2)).amax().item() + 1e-30
        err = (C.double() - ref).abs().max().item() / scale
        rec = {"name": name, "M": M, "N": N, "K": K, "batch": B, "residual": res, "rel_err": err}
        assert err < 2e-6, rec
        if cnt:
            fl = 2.0 * M * N * K * B
            t = timeit(pp)
            rec.update({"pp_us": round(t * 1e6, 1), "pp_tflops": round(fl / t / 1e12, 1)})
            tot["pp"] += t * cnt

            # the kernel the layer runs on today (single GEMMs only: the model
            # batches the Winograd GEMMs in grid.z, which this entry point
            # does not expose; tools/gemm32bench.py times those layers whole)
            def cur():
                for z in range(B):
                    call("mdx_conv2d_splitk", P(A[z]), M, 1, 1, K, P(W[z]), P(bias), N, 1, 1, 1, 0, P(R), relu, 0, 0,
                         0, P(C[z]), 1, P(ws), ws.numel(), None)
            if B == 1:
                t2 = timeit(cur)
                call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ks))
                rec.update({"cur_us": round(t2 * 1e6, 1), "cur_kernel": kid.value,
                            "cur_tflops": round(fl / t2 / 1e12, 1)})
                tot["cur"] += t2 * cnt
            if "--no-torch" not in sys.argv:
                def tm():
                    torch.matmul(A, W.transpose(1, 2), out=C)
                t3 = timeit(tm)
                rec.update({"torch_us": round(t3 * 1e6, 1), "torch_tflops": round(fl / t3 / 1e12, 1)})
                tot["torch"] += t3 * cnt
        print(json.dumps(rec), flush=True)
        del A, W, C, R
    print(json.dumps({"weighted_ms": {k: round(v * 1e3, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
