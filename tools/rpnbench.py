"""Time mdx_rpn_proposals (top-k, NMS mask + scan, level merge) on the bench
shape: B images, levels p2..p6 of a 448x512 input, 3 anchors, 1000 pre/post
NMS.  HIP events on the launch stream.  Usage: python tools/rpnbench.py [B] [reps]"""
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd._lib import call
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    A = 3
    sizes = [(112, 128), (56, 64), (28, 32), (14, 16), (7, 8)]
    g = torch.Generator().manual_seed(1)
    heads = [torch.cat([torch.randn(B, H, W, A, generator=g) * 2, torch.randn(B, H, W, 4 * A, generator=g) * 0.3],
                       -1).contiguous().cuda() for H, W in sizes]
    cells = []
    for size in (32, 64, 128, 256, 512):
        for ar in (0.5, 1.0, 2.0):
            w_ = math.sqrt(float(size) ** 2 / ar)
            h_ = ar * w_
            cells.append([-w_ / 2, -h_ / 2, w_ / 2, h_ / 2])
    cells = np.array(cells, np.float32)
    boxes = torch.empty(B, 1000, 4, device="cuda")
    scores = torch.empty(B, 1000, device="cuda")
    cnt = torch.empty(B, dtype=torch.int32, device="cuda")
    ws = torch.empty(call("mdx_rpn_workspace_bytes", B, 5, 1000), dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.c_void_p * 5)(*[h.data_ptr() for h in heads])
    ia = lambda v: (ctypes.c_int * len(v))(*v)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    stream = torch.cuda.current_stream()

    def run():
        call("mdx_rpn_proposals", ptrs, ia([s[0] for s in sizes]), ia([s[1] for s in sizes]), ia([4, 8, 16, 32, 64]),
             5, B, A, cells.ctypes.data_as(ctypes.c_void_p), 0.0, 423, 511, 1000, 1000, 0.7, 0.0, math.log(1000 / 16),
             None, P(boxes), P(scores), P(cnt), P(ws), ctypes.c_void_p(stream.cuda_stream))

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    print(f"rpn_proposals B={B}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us  checksum "
          f"{float(scores.double().sum()):.6f} {int(cnt.sum())}", flush=True)


if __name__ == "__main__":
    main()
