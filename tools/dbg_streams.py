"""Debug: model outputs of the same batch on the default stream, on a fresh
side stream, and twice on one side stream; which outputs differ."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor

dt = sys.argv[1] if len(sys.argv) > 1 else "fp16"
s = synth.SyntheticSession(12, seed=5)
raw = torch.from_numpy(s.frames(0, 12)).cuda()
pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt)
ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(batch_size=4))
prepped, cleaned = ex.front(raw[:4])
torch.cuda.synchronize()
keys = ("boxes", "scores", "ndet", "keypoints")


def run(stream):
    with torch.cuda.stream(stream):
        o = pred.model.forward(prepped, ex.lut, intermediates=True)
    torch.cuda.synchronize()
    return o


base = run(torch.cuda.current_stream())
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
for name, st in (("sideA", sa), ("sideA_again", sa), ("sideB", sb), ("default_again", torch.cuda.current_stream())):
    o = run(st)
    diffs = {}
    for k in keys + ("masks",):
        a, b = base[k].float(), o[k].float()
        diffs[k] = float((a - b).abs().max()) if a.numel() else 0.0
    for k, v in base["intermediates"].items():
        if torch.is_tensor(v) and v.is_floating_point():
            d = (v.float() - o["intermediates"][k].float()).abs().max().item()
            if d != 0:
                diffs["I:" + k] = d
    print(name, {k: v for k, v in diffs.items() if v != 0} or "identical", flush=True)
