"""Level assignment and feature-space sizes of the box-head ROIs on the bench
workload (32 synthetic frames, random-init weights).  Usage: python tools/roistats.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import proc, synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    cfg = ModelConfig(score_thresh_test=0.0)
    pred = Predictor.from_config(cfg, dtype="fp16", seed=0)
    sess = synth.SyntheticSession(32, seed=1000)
    raw = torch.from_numpy(sess.frames(0, 32)).cuda()
    prepped = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, True)(raw)
    out = pred.model.forward(prepped, proc.scale_lut(0, 100), intermediates=True)
    inter = out["intermediates"] if "intermediates" in out else out
    props = inter["proposals"].float().cpu().numpy().reshape(-1, 4)
    cnt = inter["proposal_count"].cpu().numpy()
    print("proposals per image:", cnt.min(), cnt.max())
    w = props[:, 2] - props[:, 0]
    h = props[:, 3] - props[:, 1]
    area = np.clip(w * h, 0, None)
    lvl = np.floor(4 + np.log2(np.sqrt(area) / 224 + 1e-8))
    lvl = np.clip(lvl, 2, 5)
    for l in range(2, 6):
        m = lvl == l
        s = 2.0 ** l
        if m.any():
            print(f"level {l}: {m.sum():6d} rois, feature w {np.mean(w[m] / s):5.1f} h {np.mean(h[m] / s):5.1f} "
                  f"(max {np.max(w[m] / s):5.1f} x {np.max(h[m] / s):5.1f})")


if __name__ == "__main__":
    main()
