"""Debug: serial step_device vs OverlappedExtractor, per stage (front, model
outputs, tail) and batch; which tensors differ."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor

dt = sys.argv[1] if len(sys.argv) > 1 else "fp16"
nms = int(sys.argv[2]) if len(sys.argv) > 2 else 2
knob = sys.argv[3] if len(sys.argv) > 3 else ""
from moseq2_detectron_extract_amd._lib import call
if knob == "nolarge":
    call("mdx_conv_set_large_tiles", 0)
elif knob == "nostream":
    call("mdx_conv_set_stream1x1", 0, 65536)
elif knob == "dma128":
    call("mdx_conv_set_dma128", 2, 0)
s = synth.SyntheticSession(12, seed=5)
raw = torch.from_numpy(s.frames(0, 12)).cuda()
pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt)
ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(batch_size=4))
batches = [raw[i:i + 4] for i in range(0, 12, 4)]
rec = {"front": [], "inf": []}
orig_front, orig_infer = ex.front, ex.infer


def front(r):
    p, c = orig_front(r)
    rec["front"].append((p, c))
    return p, c


def infer(p):
    o = orig_infer(p)
    rec["inf"].append(o)
    return o


ex.front, ex.infer = front, infer
want = [ex.step_device(b) for b in batches]
torch.cuda.synchronize()
wf, wi = rec["front"], rec["inf"]
rec["front"], rec["inf"] = [], []
pipe = OverlappedExtractor(ex, nms)
got = [r for r in (pipe.submit(b) for b in batches) if r is not None]
got.extend(pipe.flush())
torch.cuda.synchronize()


def d(a, b):
    if a.dtype == torch.bool or not a.is_floating_point():
        return int((a != b).sum())
    return float(torch.nan_to_num((a.double() - b.double()).abs(), nan=0.0).max())


for i in range(3):
    out = {}
    out["prepped"] = d(wf[i][0], rec["front"][i][0])
    out["cleaned"] = d(wf[i][1], rec["front"][i][1])
    for k, v in wi[i].items():
        if torch.is_tensor(v):
            out["inf:" + k] = d(v, rec["inf"][i][k])
        elif k == "masks":
            out["inf:masks"] = sum(d(a, b) for a, b in zip(v, rec["inf"][i][k]))
    for k in ("depth_frames", "mask_frames", "centroid", "angle", "keypoints"):
        out[k] = d(want[i][k], got[i][k])
    print(dt, nms, knob, "batch", i, {k: v for k, v in out.items() if v} or "identical", flush=True)
