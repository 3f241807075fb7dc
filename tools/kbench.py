"""Per-op timing of the frame-side kernels on the bench workload (32 synthetic
512x424 frames), HIP events on the launch stream.  Usage:
    python tools/kbench.py [--reps 20] [--only clean,moments,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import proc, synth

    B = args.batch
    sess = synth.SyntheticSession(B, seed=1000)
    raw = torch.from_numpy(sess.frames(0, B)).cuda()
    prep = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, True)
    prepped = prep(raw)
    cleaned = proc.clean_frames(prepped, iters_tail=3)
    mask = (prepped > 10).to(torch.uint8)
    feats = proc.frame_moments(cleaned, mask, 3.0)
    ang = torch.rad2deg(feats["orientation"]).nan_to_num(0.0)
    cen = feats["centroid"].nan_to_num(200.0)
    prep_noinp = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, False)
    p0, inv = prep_noinp(raw, return_invalid=True)

    from moseq2_detectron_extract_amd._lib import call
    import ctypes

    def clean_mode(m):
        def f():
            old = call("mdx_clean_set_mode", m)
            try:
                proc.clean_frames(prepped, iters_tail=3)
            finally:
                call("mdx_clean_set_mode", old)
        return f

    def moments_nows():
        n, H, W = cleaned.shape
        out = [torch.empty((n, 2), dtype=torch.float64, device="cuda"), torch.empty((n,), dtype=torch.float64,
               device="cuda"), torch.empty((n, 2), dtype=torch.float64, device="cuda")]
        call("mdx_frame_moments", ctypes.c_void_p(cleaned.data_ptr()), ctypes.c_void_p(mask.data_ptr()), n, H, W, 3.0,
             *[ctypes.c_void_p(t.data_ptr()) for t in out], None,
             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

    ops = {
        "clean_perpass": clean_mode(0),
        "clean_stream_auto": clean_mode(1),
        "clean_stream256": clean_mode(2),
        "clean_stream512": clean_mode(3),
        "moments_in_kernel_pack": moments_nows,
        "prep_noinpaint": lambda: prep_noinp(raw),
        "prep_inpaint": lambda: prep(raw),
        "inpaint_only": lambda: proc.fill_invalid_pixels(p0.clone(), inv, _workspace_owner=prep_noinp),
        "clean": lambda: proc.clean_frames(prepped, iters_tail=3),
        "median_only": lambda: proc.clean_frames(prepped, iters_tail=0),
        "moments": lambda: proc.frame_moments(cleaned, mask, 3.0),
        "crop": lambda: proc.crop_and_rotate_frames(prepped, cen, ang, (80, 80), frames2=mask),
    }
    only = [o for o in args.only.split(",") if o]
    res = {}
    for name, fn in ops.items():
        if only and name not in only:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / args.reps * 1e3, 1)
        print(f"{name:16s} {res[name]:9.1f} us", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
