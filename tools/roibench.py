"""Time the box-head ROIAlign on the bench workload's real proposals and FPN
maps for several LDS staging caps.  Usage: python tools/roibench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import proc, synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    cfg = ModelConfig(score_thresh_test=0.0)
    dt = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    pred = Predictor.from_config(cfg, dtype=dt, seed=0)
    m = pred.model
    sess = synth.SyntheticSession(32, seed=1000)
    raw = torch.from_numpy(sess.frames(0, 32)).cuda()
    prepped = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, True)(raw)
    captured = {}
    orig = m.roi_align

    def cap(feats, props, pcount, R, P, *a, **k):
        if P == cfg.box_pooler_resolution and "box" not in captured:
            captured["box"] = (feats, props, pcount, R, P, a, k)
        return orig(feats, props, pcount, R, P, *a, **k)
    m.roi_align = cap
    m.forward(prepped, proc.scale_lut(0, 100))
    m.roi_align = orig
    feats, props, pcount, R, P, a, k = captured["box"]
    # adaptive sampling grid statistics (gh x gw per bin) by level
    import math
    b = props.reshape(-1, 4).float()
    w, h = (b[:, 2] - b[:, 0]).clamp(min=0), (b[:, 3] - b[:, 1]).clamp(min=0)
    lvl = torch.floor(4 + torch.log2(torch.sqrt(w * h) / 224 + 1e-8)).clamp(2, 5)
    sc = 2.0 ** (-lvl)
    gh = torch.ceil(h * sc / P).clamp(min=1)
    gw = torch.ceil(w * sc / P).clamp(min=1)
    S = (gh * gw)
    print(f"ROIs {b.shape[0]}, samples/bin mean {S.mean().item():.2f}, p50 {S.median().item():.0f}, "
          f"p90 {S.quantile(0.9).item():.0f}, p99 {S.quantile(0.99).item():.0f}, max {S.max().item():.0f}; "
          f"total samples x bins {float((S * P * P).sum()):.3e}; share of the top 5% ROIs "
          f"{float(S.sort(descending=True).values[:len(S) // 20].sum() / S.sum()):.2f}")
    from moseq2_detectron_extract_amd._lib import call
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    outs = {}
    for mode, name in ((0, "slice+LDS window"), (1, "rows x1"), (2, "rows x2"), (3, "rows x4"), (4, "separable"), (5, "separable, row-shared"), (6, "separable, LDS window")):
        old = call("mdx_roi_align_set_mode", mode)
        for _ in range(2):
            out = orig(feats, props, pcount, R, P, *a, **k)
        e0.record()
        for _ in range(5):
            out = orig(feats, props, pcount, R, P, *a, **k)
        e1.record()
        torch.cuda.synchronize()
        call("mdx_roi_align_set_mode", old)
        outs[mode] = out.float()
        print(f"box ROIAlign [{name}]: {e0.elapsed_time(e1) / 5 * 1e3:8.1f} us", flush=True)
    for order in (0, 1):
        oldo = call("mdx_roi_align_set_order", order)
        for _ in range(2):
            out = orig(feats, props, pcount, R, P, *a, **k)
        e0.record()
        for _ in range(5):
            out = orig(feats, props, pcount, R, P, *a, **k)
        e1.record()
        torch.cuda.synchronize()
        call("mdx_roi_align_set_order", oldo)
        print(f"box ROIAlign [separable, xcd_remap={order}]: {e0.elapsed_time(e1) / 5 * 1e3:8.1f} us", flush=True)
    print("max |diff| between kernels:", max((outs[0] - outs[m]).abs().max().item() for m in outs))
    # locality experiment: ROIs of each image ordered by level, then position
    pr = props.reshape(pcount.shape[0], -1, 4)
    cy = (pr[..., 1] + pr[..., 3]) / 2
    cx = (pr[..., 0] + pr[..., 2]) / 2
    wv, hv = (pr[..., 2] - pr[..., 0]).clamp(min=0), (pr[..., 3] - pr[..., 1]).clamp(min=0)
    lv = torch.floor(4 + torch.log2(torch.sqrt(wv * hv) / 224 + 1e-8)).clamp(2, 5)
    key = lv * 1e6 + torch.floor(cy / 32) * 1e3 + cx
    order = key.argsort(dim=1)
    ps = torch.gather(pr, 1, order[..., None].expand(-1, -1, 4)).reshape(props.shape).contiguous()
    for mode in (1, 4):
        old = call("mdx_roi_align_set_mode", mode)
        for _ in range(2):
            out = orig(feats, ps, pcount, R, P, *a, **k)
        e0.record()
        for _ in range(5):
            out = orig(feats, ps, pcount, R, P, *a, **k)
        e1.record()
        torch.cuda.synchronize()
        call("mdx_roi_align_set_mode", old)
        print(f"box ROIAlign [mode {mode}, ROIs sorted by level/position]: {e0.elapsed_time(e1) / 5 * 1e3:8.1f} us",
              flush=True)

if __name__ == "__main__":
    main()
