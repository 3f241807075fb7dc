"""fp32 GEMM reference points on the MI355X: torch.matmul (hipBLASLt /
rocBLAS) on the model's large GEMM shapes and a square one, TFLOP/s, to size
what a plain library fp32 GEMM reaches on this chip (for the roofline
discussion of k_conv_sb).  Usage: python tools/blasbench.py"""
import json
import time

import torch

SHAPES = [("square_8192", 8192, 8192, 8192), ("box_fc1", 32000, 1024, 12544), ("res4_conv3", 28672, 1024, 256),
          ("res4_conv1", 28672, 256, 1024), ("wino6_p2_gemm", 856064, 256, 256), ("res3_conv3", 114688, 512, 128),
          ("res2_conv3", 458752, 256, 64), ("kp_wino4", 18432, 512, 512)]


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda")
        b = torch.randn(K, N, device="cuda")
        c = a @ b
        torch.cuda.synchronize()
        reps = max(3, min(50, int(2e12 / (2 * M * N * K))))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            torch.matmul(a, b, out=c)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "us": round(us, 1),
                          "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
        del a, b, c
    time.sleep(0.1)


if __name__ == "__main__":
    main()
