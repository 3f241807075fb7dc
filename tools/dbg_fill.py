"""Debug: forwards after filling the workspace with different bytes; the first
intermediate (in forward order) that depends on the stale contents."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth, proc
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor

order = ["res2", "res3", "res4", "res5", "p5", "p4", "p3", "p2", "p6", "proposals", "proposal_scores",
         "proposal_count", "box_pooled", "box_pred", "mask_logits"]
for dt in ("fp16", "fp32"):
    s = synth.SyntheticSession(4, seed=5)
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt)
    prep = proc.FramePrep(s.bground_im, s.roi, 0, 100)
    x = prep(torch.from_numpy(s.frames(0, 4)).cuda())
    B, h, w = x.shape
    outs = []
    for byte in (0x00, 0x7f, 0x3c):
        pred.model.debug_fill(B, h, w, byte)
        o = pred.model.forward(x, proc.scale_lut(0, 100), intermediates=True)
        torch.cuda.synchronize()
        outs.append(o)
    a = outs[0]
    for j, b in enumerate(outs[1:]):
        bad = []
        for k in order:
            ta, tb = a["intermediates"][k], b["intermediates"][k]
            if not torch.equal(torch.nan_to_num(ta.float(), nan=1e30), torch.nan_to_num(tb.float(), nan=1e30)):
                diff = (ta.float() - tb.float()).abs()
                bad.append((k, int((diff != 0).sum()), int(torch.isnan(tb.float()).sum())))
        for k in ("boxes", "scores", "keypoints", "masks"):
            if not torch.equal(a[k], b[k]):
                bad.append(("out:" + k,))
        print(dt, "fill", j + 1, bad or "identical", flush=True)
