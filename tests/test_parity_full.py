"""Parity of the BENCHED configuration against the oracle: full 512x424
synthetic frames, the production batch (R50-FPN B=32 -- BASELINE config 2 --
and R101-FPN B=64 -- config 5), fp32 and fp16, through GPUExtractor (prep +
inpaint, scale LUT, the model handle's forward with the planner's production
kernels -- k_convg<8> / split-K / the 32k-ROI pooler grid -- mask NMS +
instance 0, clean, moments, crop).  Frames 0 and one from the middle of the
batch are re-run through the CPU oracle chain (oracle/frameops.c +
oracle/model_ref.py, M/model/predict.py:92 -> M/proc/proc.py:716-717,305-340).

Tolerances (written here, stated in DESIGN.md §4):
  features p2..p6, rel. max error:   fp32 <= 2e-4,  fp16 <= 3e-2
  detections: same count; every oracle box matched by a GPU box of IoU
    >= 0.98 (fp32) / 0.9 (fp16), |score diff| <= 1e-3 (fp32) / 2e-2 (fp16)
  masks of matched detections: differing pixels <= max(4, 3 % (fp32) /
    10 % (fp16) of the union) -- seeded random weights give masks of a few
    pixels up to blob size, where an IoU bound alone says little.  fp16:
    the bound applies to the DECISIVE pixels, those whose oracle pasted
    probability is outside 0.5 +- 0.05 (random weights leave large areas of
    logits near 0, where fp16's ~1e-2 logit error flips the threshold); the
    raw differing-pixel counts are recorded as well
  keypoints of matched detections: >= 90 % (fp32) / 75 % (fp16) within 1 px
  downstream (selected mask -> clean -> moments -> angle -> crop):
    selected mask: the mask bound above; centroid within 0.5 px (fp32) /
    2 px (fp16), angle within 1 deg / 5 deg (mod 180), NaN (no contour)
    on both sides or neither; the crop at the GPU centroid / angle equals
    the oracle crop at the same centroid / angle bit for bit.
The measured numbers are written to gpurun_out/parity_full_<case>.json when
that directory exists (evidence for DESIGN.md)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TOL = {"fp32": dict(feat=2e-4, box_iou=0.98, score=1e-3, mask_px=0.03, kp=0.9, cen=0.5, ang=1.0, margin=0.0),
       "fp16": dict(feat=3e-2, box_iou=0.9, score=2e-2, mask_px=0.10, kp=0.75, cen=2.0, ang=5.0, margin=0.05)}
MASK_PX_FLOOR = 4  # pixels: the seeded-weight masks can be a handful of pixels


def _iou_box(a, b):
    x1 = np.maximum(a[:, None, 0], b[None, :, 0]); y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2]); y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]); ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + ab[None, :] - inter)


def _mask_iou(a, b):
    u = np.logical_or(a, b).sum()
    return 1.0 if u == 0 else np.logical_and(a, b).sum() / u


def _mask_px(a, b, probs=None, margin=0.0):
    """(differing pixels, union pixels); with the oracle's pasted
    probabilities and a margin, only pixels outside 0.5 +- margin count"""
    x = np.logical_xor(a, b)
    if probs is not None and margin > 0:
        x &= np.abs(probs - 0.5) > margin
    return int(x.sum()), int(np.logical_or(a, b).sum())


def _mask_ok(diff_union, frac):
    d, u = diff_union
    return d <= max(MASK_PX_FLOOR, frac * u)


def _close_nan(a, b, tol):
    a, b = np.asarray(a, float), np.asarray(b, float)
    if np.isnan(a).any() or np.isnan(b).any():
        return bool(np.array_equal(np.isnan(a), np.isnan(b)))
    return bool(np.abs(a - b).max() <= tol)


def _ang_diff(a, b):
    d = np.abs(np.mod(a - b, 180.0))
    return np.minimum(d, 180.0 - d)


@pytest.mark.parametrize("depth,B,dtype,wino,split", [(50, 32, "fp32", 4, 0), (50, 32, "fp32", 2, 0),
                                                      (50, 32, "fp32", 0, 0), (50, 32, "fp32", 4, 6),
                                                      (50, 32, "fp16", 0, 0), (101, 64, "fp16", 0, 0)])
def test_forward_full_frame(mdx, depth, B, dtype, wino, split):
    """wino: the fp32 3x3 algorithm (mdx_conv_set_winograd: 4 = F(4x4,3x3),
    2 = F(2x2,3x3), 0 = direct); split: the fp32 layers as exact bf16 plane
    products (mdx_conv_set_fp32_split, 0 = the f32 MFMA kernels); the same
    fp32 tolerances hold for all."""
    from moseq2_detectron_extract_amd._lib import call
    old = call("mdx_conv_set_winograd", wino)
    old_s = call("mdx_conv_set_fp32_split", split)
    try:
        _forward_full_frame(depth, B, dtype, wino, split)
    finally:
        call("mdx_conv_set_winograd", old)
        call("mdx_conv_set_fp32_split", old_s)


def _forward_full_frame(depth, B, dtype, wino, split=0):
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor, synthetic_state_dict
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
    from oracle import frameops as O
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    tol = TOL[dtype]
    cfg = ModelConfig(depth=depth, score_thresh_test=0.0)
    sd = synthetic_state_dict(cfg, 0)
    pred = Predictor.from_config(cfg, weights=sd, dtype=dtype)
    s = synth.SyntheticSession(B, seed=77)
    raw = s.frames(0, B)
    ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(batch_size=B))
    prepped_d, cleaned_d = ex.front(torch.from_numpy(raw).cuda())
    inf = ex.infer(prepped_d)
    gfeat = {k: pred.model.tensor(k).cpu().permute(0, 3, 1, 2).double() for k in ("p2", "p3", "p4", "p5", "p6")}
    tail = ex.tail(prepped_d, cleaned_d, inf)
    torch.cuda.synchronize()
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    np.testing.assert_array_equal(prepped_d.cpu().numpy(), prepped)  # bit-exact frame ops feed both sides
    scaled = O.scale_raw_frames(prepped, 0, 100)
    masks_all = torch.cat([m for m in inf["masks"]]).cpu().numpy()
    stats = {"case": f"R{depth} B={B} {dtype}" + (f" winograd F({wino}x{wino},3x3)" if wino else "") +
             (f" bf16x{split} plane products" if split else ""), "frames": []}
    try:
        _compare(sd, cfg, tol, B, prepped, scaled, inf, gfeat, masks_all, cleaned_d, tail, stats)
    finally:
        out = os.path.join(ROOT, "gpurun_out")
        if os.path.isdir(out):
            name = f"parity_full_R{depth}_B{B}_{dtype}" + (f"_wino{wino}" if wino else "") + (f"_x{split}" if split else "")
            with open(os.path.join(out, name + ".json"), "w") as fh:
                json.dump(stats, fh, indent=1)


def _compare(sd, cfg, tol, B, prepped, scaled, inf, gfeat, masks_all, cleaned_d, tail, stats):
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import model_ref as R
    for i in (0, B // 2 + 1):
        want, inter = R.forward(sd, cfg, scaled[i:i + 1, ..., None])
        w = want[0]
        fe = {}
        for k in ("p2", "p3", "p4", "p5", "p6"):
            g, ww = gfeat[k][i], inter[k][0].double()
            fe[k] = (g - ww).abs().max().item() / (ww.abs().max().item() + 1e-9)
        n = int(inf["ndet"][i])
        wb = w["pred_boxes"].numpy()
        gb = inf["boxes"][i, :n].cpu().numpy()
        rec = {"frame": i, "feat_rel_err": fe, "ndet": [n, len(wb)]}
        stats["frames"].append(rec)
        m = min(n, len(wb))
        iou = _iou_box(wb[:m], gb) if m else np.zeros((0, 0))
        match = iou.argmax(1) if m else np.zeros(0, int)
        rec["box_iou_min"] = float(iou.max(1).min()) if m else 1.0
        gs = inf["scores"][i, :n].cpu().numpy()
        rec["score_diff_max"] = float(np.abs(gs[match] - w["scores"].numpy()[:m]).max()) if m else 0.0
        gm = masks_all[i, :n].astype(bool)
        rec["mask_iou"] = [float(_mask_iou(gm[match[j]], w["pred_masks"][j].numpy())) for j in range(m)]
        wp = w["pred_mask_probs"].numpy()
        rec["mask_px_raw"] = [_mask_px(gm[match[j]], w["pred_masks"][j].numpy()) for j in range(m)]
        rec["mask_px"] = [_mask_px(gm[match[j]], w["pred_masks"][j].numpy(), wp[j], tol["margin"]) for j in range(m)]
        gk = inf["keypoints"][i, :n].cpu().numpy()
        wk = w["pred_keypoints"].numpy()[:m]
        d = np.abs(gk[match][..., :2] - wk[..., :2]).max(-1)
        rec["kp_within_1px"] = float((d < 1.0).mean()) if m else 1.0
        # downstream: the oracle chain on the oracle's own masks
        keep = FR.nms_mask_instances(w["pred_masks"].numpy(), w["scores"].numpy())
        d2w = w["pred_masks"][keep[0]].numpy().astype(np.uint8) if keep else np.zeros(prepped.shape[1:], np.uint8)
        d2g = inf["d2_mask"][i].cpu().numpy()
        rec["sel_mask_iou"] = float(_mask_iou(d2g.astype(bool), d2w.astype(bool)))
        rec["sel_mask_px_raw"] = _mask_px(d2g.astype(bool), d2w.astype(bool))
        rec["sel_mask_px"] = _mask_px(d2g.astype(bool), d2w.astype(bool), wp[keep[0]] if keep else None,
                                      tol["margin"])
        cl = O.clean_frames(prepped[i:i + 1], iters_tail=3)
        rec["cleaned_bit_exact"] = bool(np.array_equal(cleaned_d[i].cpu().numpy(), cl[0]))
        fw = O.get_frame_features(cl, 3, mask=d2w[None])
        cw = fw["centroid"][0]
        aw = np.mod(-np.rad2deg(fw["orientation"][0]), 360)
        cg = tail["centroid"][i].cpu().numpy()
        ag = float(tail["angle"][i])
        rec["centroid"] = [cg.tolist(), cw.tolist()]
        rec["angle"] = [ag, float(aw)]
        rec["centroid_px"] = float(np.abs(cg - cw).max())
        rec["angle_deg_mod180"] = float(_ang_diff(ag, aw))
        # crops: the GPU crop equals the oracle crop at the same centre / angle
        oc = O.crop_and_rotate_frames(prepped[i:i + 1], cg[None], np.array([ag]))
        rec["crop_bit_exact_same_pose"] = bool(np.array_equal(tail["depth_frames"][i].cpu().numpy(), oc[0]))
        ocw = O.crop_and_rotate_frames(prepped[i:i + 1], cw[None], np.array([aw]))
        rec["crop_bit_exact_vs_oracle_pose"] = bool(np.array_equal(tail["depth_frames"][i].cpu().numpy(), ocw[0]))
    for rec in stats["frames"]:
        assert max(rec["feat_rel_err"].values()) <= tol["feat"], rec
        assert rec["ndet"][0] == rec["ndet"][1], rec
        assert rec["box_iou_min"] >= tol["box_iou"], rec
        assert rec["score_diff_max"] <= tol["score"], rec
        assert all(_mask_ok(x, tol["mask_px"]) for x in rec["mask_px"]), rec
        assert rec["kp_within_1px"] >= tol["kp"], rec
        assert rec["cleaned_bit_exact"], rec
        assert _mask_ok(rec["sel_mask_px"], tol["mask_px"]), rec
        assert _close_nan(rec["centroid"][0], rec["centroid"][1], tol["cen"]), rec
        a, b = rec["angle"]
        assert (np.isnan(a) and np.isnan(b)) or (not np.isnan(a) and not np.isnan(b) and
                                                 _ang_diff(a, b) <= tol["ang"]), rec
        assert rec["crop_bit_exact_same_pose"], rec
