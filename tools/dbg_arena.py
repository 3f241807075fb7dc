"""Debug: snapshot a forward's whole workspace after a serial run and after a
run concurrent with another handle's forward (both from the same fill);
report the differing byte ranges and the named buffers they fall in."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth, proc
from moseq2_detectron_extract_amd._lib import call
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor

dt = sys.argv[1] if len(sys.argv) > 1 else "fp16"
s = synth.SyntheticSession(8, seed=5)
pa = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt)
pb = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dt)
prep = proc.FramePrep(s.bground_im, s.roi, 0, 100)
x = prep(torch.from_numpy(s.frames(0, 8)).cuda())
xa, xb = x[:4].contiguous(), x[4:].contiguous()
lut = proc.scale_lut(0, 100)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
m, mb = pa.model, pb.model
S = lambda st: ctypes.c_void_p(st.cuda_stream)  # noqa: E731
names = ["input_s2d", "res2", "res3", "res4", "res5"] + [f"fpn_{k}{l}" for l in (5, 4, 3, 2)
                                                          for k in ("lateral", "inner", "output")] + \
        ["p5", "p4", "p3", "p2", "p6", "proposals", "proposal_scores", "proposal_count", "box_pooled", "box_pred",
         "mask_logits"]


def snap(concurrent):
    with torch.cuda.stream(sa):
        m.debug_fill(4, *xa.shape[1:], 0x5a)
    with torch.cuda.stream(sb):
        mb.debug_fill(4, *xb.shape[1:], 0x5a)
    torch.cuda.synchronize()
    ev = torch.cuda.Event(); ev.record(torch.cuda.current_stream())
    sa.wait_event(ev); sb.wait_event(ev)
    if concurrent:
        with torch.cuda.stream(sb):
            mb.forward(xb, lut)
    with torch.cuda.stream(sa):
        m.forward(xa, lut)
    if concurrent:
        with torch.cuda.stream(sb):
            mb.forward(xb, lut)
    torch.cuda.synchronize()
    cap = ctypes.c_int64()
    call("mdx_model_debug_arena", m._h, S(sa), None, None, ctypes.byref(cap), None, 0)
    buf = torch.empty(cap.value, dtype=torch.uint8, device="cuda")
    call("mdx_model_debug_arena", m._h, S(sa), None, None, None, ctypes.c_void_p(buf.data_ptr()), cap.value)
    torch.cuda.synchronize()
    offs = {}
    for n in names:
        o = ctypes.c_int64()
        with torch.cuda.stream(sa):
            call("mdx_model_debug_arena", m._h, S(sa), n.encode(), ctypes.byref(o), None, None, 0)
            t = m.tensor(n)
        offs[n] = (o.value, t.numel() * t.element_size())
    return buf, offs


ref, offs = snap(False)
ref2, _ = snap(False)
print("serial vs serial differing bytes:", int((ref != ref2).sum()), flush=True)
for rep in range(6):
    got, _ = snap(True)
    diff = (got != ref).nonzero().flatten().cpu().numpy()
    if diff.size == 0:
        print("rep", rep, "identical", flush=True)
        continue
    # group into ranges
    cuts = np.flatnonzero(np.diff(diff) > 4096) + 1
    ranges = [(int(g[0]), int(g[-1]) + 1) for g in np.split(diff, cuts)]
    desc = []
    for a, b in ranges[:12]:
        hits = [n for n, (o, nb) in offs.items() if o >= 0 and a < o + nb and b > o]
        desc.append((a, b - a, hits))
    print("rep", rep, "ranges", len(ranges), desc, flush=True)

# does anything write into A's workspace while ONLY B runs?
with torch.cuda.stream(sa):
    m.debug_fill(4, *xa.shape[1:], 0x5a)
torch.cuda.synchronize()
cap = ctypes.c_int64()
call("mdx_model_debug_arena", m._h, S(sa), None, None, ctypes.byref(cap), None, 0)
before = torch.empty(cap.value, dtype=torch.uint8, device="cuda")
call("mdx_model_debug_arena", m._h, S(sa), None, None, None, ctypes.c_void_p(before.data_ptr()), cap.value)
torch.cuda.synchronize()
for _ in range(4):
    with torch.cuda.stream(sb):
        mb.forward(xb, lut)
torch.cuda.synchronize()
after = torch.empty_like(before)
call("mdx_model_debug_arena", m._h, S(sa), None, None, None, ctypes.c_void_p(after.data_ptr()), cap.value)
torch.cuda.synchronize()
d = (after != before).nonzero().flatten().cpu().numpy()
print("A's workspace bytes changed while only B ran:", d.size, (int(d[0]), int(d[-1])) if d.size else "", flush=True)
# and with the same handle on another stream
for _ in range(4):
    with torch.cuda.stream(sb):
        m.forward(xb, lut)
torch.cuda.synchronize()
after2 = torch.empty_like(before)
call("mdx_model_debug_arena", m._h, S(sa), None, None, None, ctypes.c_void_p(after2.data_ptr()), cap.value)
torch.cuda.synchronize()
d = (after2 != before).nonzero().flatten().cpu().numpy()
print("A's workspace bytes changed while the same handle ran on B:", d.size, (int(d[0]), int(d[-1])) if d.size else "",
      flush=True)
# B's arena base vs A's
for nm, mm, st in (("A", m, sa), ("B(other)", mb, sb), ("A-handle on B", m, sb)):
    o = ctypes.c_int64()
    call("mdx_model_debug_arena", mm._h, S(st), b"res2", ctypes.byref(o), None, None, 0)
    with torch.cuda.stream(st):
        t = mm.tensor("res2")
    print(nm, "res2 offset", o.value, flush=True)
