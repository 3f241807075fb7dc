"""Box-head ROIAlign kernels on the bench workload (R50-FPN B=32, synthetic
session frames): serial forwards per mdx_policy.roi_mode, HIP events
around each forward (the ROIAlign difference is the forward-time difference;
the whole model is enqueued from C, so the pooler has no Python hook), and
the box_pooled tensor compared bit for bit against mode 4.
Usage: python tools/roibench.py [fp32|fp16]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import proc, synth
    from moseq2_detectron_extract_amd._lib import call
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    cfg = ModelConfig(score_thresh_test=0.0)
    dt = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    m = Predictor.from_config(cfg, dtype=dt, seed=0, weights="synthetic").model
    sess = synth.SyntheticSession(32, seed=1000)
    raw = torch.from_numpy(sess.frames(0, 32)).cuda()
    prepped = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, True)(raw)
    lut = proc.scale_lut(0, 100)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ref = None
    for mode in (4, 6, 4, 6):
        from moseq2_detectron_extract_amd._lib import knob
        old = knob("roi_mode", mode)
        try:
            for _ in range(2):
                m.forward(prepped, lut)
            e0.record()
            for _ in range(6):
                m.forward(prepped, lut)
            e1.record()
            torch.cuda.synchronize()
            pooled = m.forward(prepped, lut, intermediates=True)["intermediates"]["box_pooled"].clone()
            torch.cuda.synchronize()
        finally:
            knob("roi_mode", old)
        if ref is None:
            ref = pooled
        print(json.dumps({"roi_mode": mode, "forward_ms": round(e0.elapsed_time(e1) / 6, 3),
                          "box_pooled_equal_mode4": bool(torch.equal(pooled, ref))}), flush=True)


if __name__ == "__main__":
    main()
