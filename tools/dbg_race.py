"""Debug: a forward on stream A while another forward (or a background
kernel loop: modes conv / gn / torch) runs on stream B, repeated; the earliest
intermediate of A (forward order) that differs from a serial run of the same
batch.  This located the packed-FP32 GroupNorm nondeterminism (see
_build.DEVICE_FLAGS): python tools/dbg_race.py fp16 24 same."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth, proc
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor

dt = sys.argv[1] if len(sys.argv) > 1 else "fp16"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mode = sys.argv[3] if len(sys.argv) > 3 else "same"   # same | other (second handle) | conv (background conv)
order = ["res2", "res3", "res4", "res5", "fpn_lateral5", "fpn_inner5", "fpn_output5", "p5",
         "fpn_lateral4", "fpn_inner4", "fpn_output4", "p4", "fpn_inner3", "p3", "fpn_inner2", "p2", "p6", "proposals", "proposal_scores",
         "proposal_count", "box_pooled", "box_pred", "mask_logits"]
if os.environ.get("MDX_DEBUG_SHADOW"):
    order = order[:4] + ["shadow_gnws5", "gnws5"] + [f"{k}{l}" for l in (5, 4, 3, 2) for k in ("fpn_lateral", "shadow_inner", "fpn_inner",
                                                                     "fpn_output", "shadow_p", "p")]
s = synth.SyntheticSession(8, seed=5)
pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt, weights="synthetic")
prep = proc.FramePrep(s.bground_im, s.roi, 0, 100)
x = prep(torch.from_numpy(s.frames(0, 8)).cuda())
xa, xb = x[:4].contiguous(), x[4:].contiguous()
lut = proc.scale_lut(0, 100)
m = pred.model
# other: a second handle on stream B (DBG_OTHER_DT: its dtype, default the same)
mb = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=os.environ.get("DBG_OTHER_DT", dt),
                           weights="synthetic").model if mode == "other" else m
import ctypes
from moseq2_detectron_extract_amd._lib import call
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
tdt = torch.float16 if dt == "fp16" else torch.float32
bx = torch.randn(8, 112, 128, 256).to(tdt).cuda()
bw = (torch.randn(256, 2304) * 0.02).to(tdt).cuda()
bo = torch.empty(8, 112, 128, 256, dtype=tdt, device="cuda")
gg, gb = torch.ones(256, device="cuda"), torch.zeros(256, device="cuda")
gws = torch.empty(1 << 22, dtype=torch.float32, device="cuda")


def background(n):
    for _ in range(n):
        if mode == "conv":
            call("mdx_conv2d", P(bx), 8, 112, 128, 256, P(bw), None, 256, 3, 3, 1, 1, None, 0, 0, int(dt == "fp16"),
                 int(dt == "fp16"), P(bo), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        elif mode == "gn":
            call("mdx_groupnorm", P(bx), 8, 112, 128, 256, 32, 1e-5, P(gg), P(gb), None, 0,
                 int(dt == "fp16"), P(bo), P(gws), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        elif mode == "torch":
            bo.copy_(bx)
            bo.mul_(1.5)
        else:
            mb.forward(xb, lut)


# DBG_SET="fn:arg[:arg],fn:arg": planner knobs set before the runs (bisecting the kernels involved)
for spec in filter(None, os.environ.get("DBG_SET", "").split(",")):
    fn, *args = spec.split(":")
    print("set", fn, args, "->", call(fn, *[int(v) for v in args]))
ref = m.forward(xa, lut)
torch.cuda.synchronize()
ref["intermediates"] = {k: m.tensor(k) for k in order}
torch.cuda.synchronize()
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
with torch.cuda.stream(sa):
    m.reserve(4, *xa.shape[1:])
with torch.cuda.stream(sb):
    mb.reserve(4, *xb.shape[1:])
torch.cuda.synchronize()
hist = {}
for r in range(reps):
    if os.environ.get("DBG_FILL"):
        with torch.cuda.stream(sa):
            m.debug_fill(4, *xa.shape[1:], int(os.environ["DBG_FILL"], 0))
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    sa.wait_event(ev); sb.wait_event(ev)
    # B first so that A's kernels overlap B's in varying phase
    with torch.cuda.stream(sb):
        background(r % 3 + (int(os.environ.get("DBG_BG", "3")) if mode in ("conv", "gn", "torch") else 0))
    with torch.cuda.stream(sa):
        oa = m.forward(xa, lut)
    with torch.cuda.stream(sb):
        background(1 + (int(os.environ.get("DBG_BG", "3")) if mode in ("conv", "gn", "torch") else 0))
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        inter = {k: m.tensor(k) for k in order}
    torch.cuda.synchronize()
    first = None
    diffs = []
    for k in order:
        a, b = ref["intermediates"][k], inter[k]
        if k in ("proposals", "proposal_scores", "box_pred"):
            b = b.reshape(a.shape) if b.numel() == a.numel() else b
        if k == "proposal_count":
            b = b.view(-1)
        if k == "input":
            continue
        if a.shape != b.shape:
            b = b.reshape(a.shape)
        if not torch.equal(torch.nan_to_num(a.float(), nan=7e7), torch.nan_to_num(b.float(), nan=7e7)):
            d = (a.float() - b.float()).abs()
            diffs.append(k)
            if first is not None:
                continue
            first = (k, int((d != 0).sum()), float(d.max()))
            if k.endswith("gnws5"):
                # level-5 GN workspace: [stats 2*N*G][partials 3*N*G*nch]
                idx = (d.flatten() != 0).nonzero().flatten()
                print("   gnws5 differing floats:", idx.numel(), "first indices", idx[:12].tolist(), flush=True)
                dump = os.environ.get("DBG_DUMP")
                if dump and not os.path.exists(dump):
                    # the GN's input and both workspaces, for the CPU restatement
                    # of the partial / final kernels (tools/gn_emulate.py)
                    import numpy as np
                    np.savez(dump, lat_ref=ref["intermediates"]["fpn_lateral5"].cpu().numpy(),
                             lat_rep=inter["fpn_lateral5"].cpu().numpy(),
                             ws_ref=a.cpu().numpy(), ws_rep=b.cpu().numpy(), rep=r)
            if os.environ.get("DBG_DETAIL") and d.dim() == 4 and d.shape[1] > 1 and d.shape[3] % 32 == 0:
                Bn, Hh, Ww, Cc = d.shape
                grp = (d != 0).reshape(Bn, Hh * Ww, 32, Cc // 32)  # GN groups of C/32 channels
                per = grp.float().mean(dim=(1, 3))                # fraction differing per (image, group)
                bad = (per > 0).nonzero().tolist()
                pix = (d != 0).any(dim=3).reshape(Bn, -1).sum(1).tolist()
                print("   detail", k, "img/grp with diffs:", len(bad), bad[:12], "frac", [round(float(per[i, j]), 3) for i, j in bad[:12]],
                      "pixels differing per image", pix, "ref max", float(a.float().abs().max()), flush=True)
    print(dt, mode, "rep", r, first or "identical", "all differing:", diffs[:12],
          "boxes_equal", bool(torch.equal(oa["boxes"], ref["boxes"])), flush=True)
    hist[first[0] if first else None] = hist.get(first[0] if first else None, 0) + 1
print("summary", dt, mode, hist, flush=True)
if os.environ.get("MDX_DEBUG_SHADOW"):
    # where in the level-5 GN workspace: [stats 2*N*G][partials 3*N*G*nch]
    N, G = 4, 32
    a = ref["intermediates"]["shadow_gnws5"].flatten()
    with torch.cuda.stream(sa):
        b = m.tensor("shadow_gnws5").flatten()
    torch.cuda.synchronize()
    d = (a != b).nonzero().flatten().cpu().numpy()
    print("last rep gnws5 differing floats:", d.size, "stats part" if d.size and d[0] < 2 * N * G else "",
          d[:20].tolist(), flush=True)
