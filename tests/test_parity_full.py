"""Parity of the BENCHED configuration against the oracle: full 512x424
synthetic frames, the production batch (R50-FPN B=32 -- BASELINE config 2 --
and R101-FPN B=64 -- config 5), fp32 and fp16, through GPUExtractor (prep +
inpaint, scale LUT, the model handle's forward with the planner's production
kernels -- k_convg<8> / split-K / the 32k-ROI pooler grid -- mask NMS +
instance 0, clean, moments, crop).  EVERY frame of the batch is re-run
through the CPU oracle chain (oracle/frameops.c + oracle/model_ref.py,
M/model/predict.py:92 -> M/proc/proc.py:716-717,305-340); the oracle's
forward of a (depth, batch) is computed once and shared by the cases.

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
  the north_star's integer-exactness claim, at the ORACLE's pose:
    every frame, both dtypes: the crop kernel at the oracle's pose gives the
      oracle's integer crop window (M/proc/proc.py:325-328) and depth crop
      byte for byte, and the mask crop too wherever the selected masks agree.
    fp32: every frame whose selected mask equals the oracle's pixel for pixel
      has the oracle's centroid bit for bit and its angle to ANGLE_ULPS ulp
      (the moments are integer-exact; the orientation's atan2 is the GPU's
      libm, which may round the last bit differently from glibc), and the
      pipeline's depth crop equals the oracle chain's byte for byte.
  conditioning (fp32): a frame is WELL-CONDITIONED when no pixel of the
    oracle's pasted probability map of its selected detection lies within
    NEAR_EPS of the 0.5 paste threshold (M/model/util.py:45-62,
    detector_postprocess; M/proc/proc.py:657-685 takes that mask); there a
    last-bit difference of the fp32 sums cannot flip the thresholded mask.
    On the well-conditioned frames at least MIN_SEL_EXACT have the identical
    selected mask.  On an ill-conditioned frame the pose bounds are excused
    only when flipping its near-threshold pixels moves the ORACLE's own pose
    past them (each pixel alone, and all of them on / off at once: the chain
    clean -> moments -> angle re-run on the oracle side); every excluded or
    excused frame is recorded with its reason.  The R50 fp32 cases run on
    every weight seed of R50_SEEDS with these constants.
    fp16 (BASELINE config 5's precision, vs the fp32 oracle), R50 over
    R50_SEEDS: the detection checks above hold on at least FP16_FRAMES of the
    frames of all seeds together and on at least FP16_FRAMES_MIN of each
    seed's, the pose bounds likewise; at least FP16_CROP_EXACT of the
    non-NaN-pose frames give the oracle's depth crop byte for byte (the rest
    differ because fp16 moves the small seeded-weight masks by a few
    near-threshold pixels, and with them the pose); which detection check
    failed is recorded per frame (box, score, mask, keypoints).
  coverage: at least MIN_POSES frames per case (30 / 32 for R50, 60 / 64 for
    R101) carry a non-NaN pose on both sides (the chain is compared on real
    contours, not NaN against NaN).
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
       "fp16": dict(feat=3e-2, box_iou=0.9, score=2e-2, mask_px=0.10, kp=0.75, cen=2.0, ang=5.0, margin=0.05),
       # BASELINE config 5 as stated: fp32 trunk / RPN / box head (the fp32
       # feature and box bounds), fp16 mask + keypoint heads (the fp16 mask,
       # keypoint and pose bounds)
       "mixed": dict(feat=2e-4, box_iou=0.98, score=1e-3, mask_px=0.10, kp=0.75, cen=2.0, ang=5.0, margin=0.05)}
MASK_PX_FLOOR = 4       # pixels: the seeded-weight masks can be a handful of pixels
MIN_POSES = {50: 30, 101: 60}  # non-NaN poses (both sides) per case, by depth
MIN_SEL_EXACT = 0.9     # fp32: fraction of the WELL-CONDITIONED frames whose selected mask is the oracle's
NEAR_EPS = 1e-4         # fp32: a pasted probability within this of 0.5 makes its frame ill-conditioned
ANGLE_ULPS = 2          # fp32: angle agreement (deg) in units in the last place when the masks agree
FP16_FRAMES = 0.85      # fp16: fraction of all seeds' frames passing the detection checks / the pose bounds
FP16_FRAMES_MIN = 0.75  # fp16: the same per seed
FP16_CROP_EXACT = 0.12  # fp16: fraction of non-NaN-pose frames whose crop equals the oracle chain's
                        # (round-4 records: R50 B=32 4 / 21, R101 B=64 8 / 63)
MIXED_CROP_EXACT = 0.9  # config 5 as stated (fp32 trunk / box head, fp16 mask + keypoint heads): the same
                        # fraction (round-4 record: R101 B=64 62 / 64), and every frame passes the
                        # detection and pose checks
SEED = 77               # synthetic session of the batch
# seeded synthetic weights.  R50: the fp32 cases and the fp16 check run on
# every seed of R50_SEEDS with one set of constants (the seeds whose oracle
# chain carries >= MIN_POSES non-NaN poses, tools/pose_seed_scan.py 50 32).
# R101 with seed 0 selects detections off the animal on 61 of 64 frames (NaN
# poses on both sides, nothing compared downstream); seed 1 selects
# on-animal masks on every frame.
R50_SEEDS = (3, 11, 14, 34, 35)
R101_SEED = 1
ORACLE_CHUNK = 8        # frames per oracle forward (its intermediates of a whole batch would not fit)

_ORACLE = {}


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


def _window(c, a):
    """M/proc/proc.py:317-328: -1s where the crop returns zeros, else python
    int() (truncation toward zero) of centre -+ 40, shifted by the border."""
    cx, cy = float(c[0]), float(c[1])
    if np.isnan(a) or np.isnan(cx) or np.isnan(cy) or cx < 0 or cy < 0:
        return [-1] * 4
    return [int(cx - 40) + 80, int(cx + 40) + 80, int(cy - 40) + 80, int(cy + 40) + 80]


def _oracle(depth, B, wseed):
    """The oracle chain over every frame of the batch (cached per (depth, B,
    weight seed)): prepped / scaled frames, per-frame Instances fields,
    p2..p6, the selected d2 mask, cleaned frames, moments, angle, the crops at
    the oracle pose, and per frame the conditioning of its selected mask."""
    key = (depth, B, wseed)
    if key in _ORACLE:
        return _ORACLE[key]
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import model_ref as R
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = ModelConfig(depth=depth, score_thresh_test=0.0)
    sd = synthetic_state_dict(cfg, wseed)
    s = synth.SyntheticSession(B, seed=SEED)
    raw = s.frames(0, B)
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    scaled = O.scale_raw_frames(prepped, 0, 100)
    want, feats = [], []
    for a in range(0, B, ORACLE_CHUNK):
        w, inter = R.forward(sd, cfg, scaled[a:a + ORACLE_CHUNK, ..., None])
        want.extend(w)
        for j in range(len(w)):
            feats.append({k: inter[k][j].clone() for k in ("p2", "p3", "p4", "p5", "p6")})
        del inter
    d2 = np.zeros(prepped.shape, np.uint8)
    keeps = []
    for i, w in enumerate(want):
        keep = FR.nms_mask_instances(w["pred_masks"].numpy(), w["scores"].numpy())
        keeps.append(keep)
        if keep:
            d2[i] = w["pred_masks"][keep[0]].numpy()
    cl = O.clean_frames(prepped, iters_tail=3)
    fw = O.get_frame_features(cl, 3, mask=d2)
    ang = np.mod(-np.rad2deg(fw["orientation"]), 360)
    cond = [_conditioning(O, want[i], keeps[i], d2[i], cl[i], fw["centroid"][i], ang[i]) for i in range(B)]
    res = dict(cfg=cfg, sd=sd, wseed=wseed, raw=raw, roi=(s.bground_im, s.roi), prepped=prepped, want=want,
               feats=feats, keeps=keeps, d2=d2, cleaned=cl, centroid=fw["centroid"], angle=ang, cond=cond,
               crop=O.crop_and_rotate_frames(prepped, fw["centroid"], ang),
               crop_mask=O.crop_and_rotate_frames(d2, fw["centroid"], ang))
    _ORACLE[key] = res
    return res


def _conditioning(O, w, keep, d2, cleaned, cen, ang, max_single=32):
    """Conditioning of one frame's selected mask: the pixels of the oracle's
    pasted probability within NEAR_EPS of 0.5 (also counted at other eps, for
    the record), and how far flipping them moves the oracle's own pose --
    each near pixel alone (up to max_single of them) and all of them on and
    off at once -- as (max centroid shift px, max angle shift deg mod 180)."""
    out = {"near_px": 0, "near_px_by_eps": {}, "pose_shift": [0.0, 0.0]}
    if not keep:
        return out
    p = w["pred_mask_probs"][keep[0]].numpy()
    dist = np.abs(p.astype(np.float64) - 0.5)
    for e in (1e-6, 1e-5, 1e-4, 1e-3):
        out["near_px_by_eps"][str(e)] = int((dist < e).sum())
    near = np.argwhere(dist < NEAR_EPS)
    out["near_px"] = int(len(near))
    if not len(near) or np.isnan(cen).any():
        return out
    variants = []
    for yx in near[:max_single]:
        m = d2.copy()
        m[yx[0], yx[1]] ^= 1
        variants.append(m)
    for v in (0, 1):
        m = d2.copy()
        m[near[:, 0], near[:, 1]] = v
        variants.append(m)
    g = O.get_frame_features(np.repeat(cleaned[None], len(variants), 0), 3, mask=np.stack(variants))
    ga = np.mod(-np.rad2deg(g["orientation"]), 360)
    dc = np.abs(g["centroid"] - cen[None]).max(1)
    da = _ang_diff(ga, ang)
    nan = np.isnan(dc) | np.isnan(da)
    out["pose_shift"] = [float(np.inf) if nan.any() else float(dc.max()),
                         float(np.inf) if nan.any() else float(da.max())]
    return out


FP32_VARIANTS = [("fp32", 4, 0), ("fp32", 6, 0), ("fp32", 2, 0), ("fp32", 0, 0), ("fp32", 4, 6), ("fp32", 6, 6)]


@pytest.mark.parametrize("depth,B,dtype,wino,split,wseed",
                         [(50, 32, d, w, x, ws) for ws in R50_SEEDS for d, w, x in FP32_VARIANTS] +
                         [(101, 64, "fp16", 0, 0, R101_SEED), (101, 64, "mixed", 6, 0, R101_SEED),
                          (101, 64, "fp32", 6, 0, R101_SEED)])
def test_forward_full_frame(mdx, depth, B, dtype, wino, split, wseed):
    """wino: the fp32 3x3 algorithm (mdx_policy.winograd: 4 = F(4x4,3x3),
    6 = F(6x6,3x3) on the large maps and F(4x4,3x3) elsewhere, 2 = F(2x2,3x3),
    0 = direct); split: the fp32 layers as exact bf16 plane
    products (mdx_policy.fp32_split, 0 = the f32 MFMA kernels); wseed: the
    synthetic weights; the same fp32 tolerances hold for all."""
    with _policy(wino, split):
        st = _forward_full_frame(depth, B, dtype, wino, split, wseed)["summary"]
    if dtype == "fp16":
        assert st["detections_ok"] >= FP16_FRAMES * B and st["pose_ok"] >= FP16_FRAMES * B, st
        assert st["crop_bit_exact_vs_oracle_non_nan"][0] >= FP16_CROP_EXACT * st["crop_bit_exact_vs_oracle_non_nan"][1], st


def test_forward_full_frame_fp16_seeds(mdx):
    """R50 B=32 all-fp16 against the fp32 oracle on every seed of R50_SEEDS:
    per seed and over all seeds, the fraction of frames passing the detection
    and pose checks (FP16_FRAMES_MIN / FP16_FRAMES) and the crop exactness
    (FP16_CROP_EXACT); the failing detection checks are recorded."""
    tot = {"frames": 0, "detections_ok": 0, "pose_ok": 0, "crop_exact": 0, "non_nan": 0}
    per = {}
    for ws in R50_SEEDS:
        with _policy(0, 0):
            st = _forward_full_frame(50, 32, "fp16", 0, 0, ws)["summary"]
        per[ws] = st
        tot["frames"] += st["frames"]
        tot["detections_ok"] += st["detections_ok"]
        tot["pose_ok"] += st["pose_ok"]
        tot["crop_exact"] += st["crop_bit_exact_vs_oracle_non_nan"][0]
        tot["non_nan"] += st["crop_bit_exact_vs_oracle_non_nan"][1]
    _record("parity_full_R50_B32_fp16_seeds", {"per_seed": per, "total": tot})
    for ws, st in per.items():
        assert st["detections_ok"] >= FP16_FRAMES_MIN * st["frames"], (ws, st)
        assert st["pose_ok"] >= FP16_FRAMES_MIN * st["frames"], (ws, st)
    assert tot["detections_ok"] >= FP16_FRAMES * tot["frames"], tot
    assert tot["pose_ok"] >= FP16_FRAMES * tot["frames"], tot
    assert tot["crop_exact"] >= FP16_CROP_EXACT * tot["non_nan"], tot


def _policy(wino, split):
    """The thread's policy for the case: the Predictor's handle, created
    inside, captures it."""
    from moseq2_detectron_extract_amd._lib import policy_scope
    return policy_scope(winograd=wino, fp32_split=split)


def _record(name, obj):
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, name + ".json"), "w") as fh:
            json.dump(obj, fh, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))


def _forward_full_frame(depth, B, dtype, wino, split=0, wseed=None):
    from moseq2_detectron_extract_amd.model import Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
    wseed = (R50_SEEDS[0] if depth == 50 else R101_SEED) if wseed is None else wseed
    orc = _oracle(depth, B, wseed)
    tol = TOL[dtype]
    pred = Predictor.from_config(orc["cfg"], weights=orc["sd"], dtype=dtype)
    ex = GPUExtractor(*orc["roi"], pred, ExtractConfig(batch_size=B))
    prepped_d, cleaned_d = ex.front(torch.from_numpy(orc["raw"]).cuda())
    inf = ex.infer(prepped_d)
    gfeat = {k: pred.model.tensor(k).cpu().permute(0, 3, 1, 2).double() for k in ("p2", "p3", "p4", "p5", "p6")}
    tail = ex.tail(prepped_d, cleaned_d, inf)
    # the crops and windows at the ORACLE's pose, through the same kernel
    from moseq2_detectron_extract_amd import proc
    oc, ocm, owin = proc.crop_and_rotate_frames(prepped_d, torch.from_numpy(orc["centroid"]).cuda(),
                                                torch.from_numpy(orc["angle"]).cuda(), frames2=inf["d2_mask"],
                                                return_window=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(prepped_d.cpu().numpy(), orc["prepped"])  # bit-exact frame ops feed both sides
    masks_all = torch.cat([m for m in inf["masks"]]).cpu().numpy()
    stats = {"case": f"R{depth} B={B} {dtype}" + (f" winograd F({wino}x{wino},3x3)" if wino else "") +
             (f" bf16x{split} plane products" if split else "") + f" weights seed {wseed}", "near_eps": NEAR_EPS,
             "frames": []}
    try:
        _compare(orc, tol, dtype, B, inf, gfeat, masks_all, cleaned_d, tail,
                 (oc.cpu().numpy(), ocm.cpu().numpy(), owin.cpu().numpy()), stats)
    finally:
        _record(f"parity_full_R{depth}_B{B}_{dtype}" + (f"_wino{wino}" if wino else "") +
                (f"_x{split}" if split else "") + f"_s{wseed}", stats)
    return stats


def _compare(orc, tol, dtype, B, inf, gfeat, masks_all, cleaned_d, tail, at_oracle_pose, stats):
    oc, ocm, owin = at_oracle_pose
    from oracle import frameops as O
    cleaned = cleaned_d.cpu().numpy()
    g_cen = tail["centroid"].cpu().numpy()
    g_ang = tail["angle"].cpu().numpy()
    g_depth = tail["depth_frames"].cpu().numpy()
    g_d2 = inf["d2_mask"].cpu().numpy()
    # the GPU crops re-made by the oracle at the GPU's own pose
    oc_gpose = O.crop_and_rotate_frames(orc["prepped"], g_cen, g_ang)
    for i in range(B):
        w = orc["want"][i]
        fe = {}
        for k in ("p2", "p3", "p4", "p5", "p6"):
            g, ww = gfeat[k][i], orc["feats"][i][k].double()
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
        wp = w["pred_mask_probs"].numpy()
        rec["mask_px_raw"] = [_mask_px(gm[match[j]], w["pred_masks"][j].numpy()) for j in range(m)]
        rec["mask_px"] = [_mask_px(gm[match[j]], w["pred_masks"][j].numpy(), wp[j], tol["margin"]) for j in range(m)]
        gk = inf["keypoints"][i, :n].cpu().numpy()
        wk = w["pred_keypoints"].numpy()[:m]
        d = np.abs(gk[match][..., :2] - wk[..., :2]).max(-1)
        rec["kp_within_1px"] = float((d < 1.0).mean()) if m else 1.0
        # downstream: the oracle chain on the oracle's own masks
        keep = orc["keeps"][i]
        d2w, d2g = orc["d2"][i].astype(bool), g_d2[i].astype(bool)
        rec["sel_mask_identical"] = bool(np.array_equal(d2g, d2w))
        rec["sel_mask_px_raw"] = _mask_px(d2g, d2w)
        rec["sel_mask_px"] = _mask_px(d2g, d2w, wp[keep[0]] if keep else None, tol["margin"])
        rec["cleaned_bit_exact"] = bool(np.array_equal(cleaned[i], orc["cleaned"][i]))
        cw, aw = orc["centroid"][i], float(orc["angle"][i])
        cg, ag = g_cen[i], float(g_ang[i])
        rec["centroid"] = [cg.tolist(), cw.tolist()]
        rec["angle"] = [ag, aw]
        rec["pose_non_nan"] = bool(not np.isnan(cw).any() and not np.isnan(cg).any())
        rec["pose_bit_exact"] = bool(np.array_equal(cg, cw, equal_nan=True) and
                                     np.array_equal(ag, aw, equal_nan=True))
        rec["centroid_bit_exact"] = bool(np.array_equal(cg, cw, equal_nan=True))
        rec["angle_ulps"] = 0.0 if (np.isnan(ag) and np.isnan(aw)) else float(abs(ag - aw) / np.spacing(aw))
        # crops: the GPU crop equals the oracle crop at the same centre / angle
        rec["crop_bit_exact_same_pose"] = bool(np.array_equal(g_depth[i], oc_gpose[i]))
        # ... and at the oracle's pose: the GPU crop kernel there vs the oracle
        # chain's crops and window, and the pipeline's own crop vs the oracle's
        rec["window_oracle_pose"] = [owin[i].tolist(), _window(cw, aw)]
        rec["crop_oracle_pose_bit_exact"] = bool(np.array_equal(oc[i], orc["crop"][i]))
        rec["crop_mask_oracle_pose_bit_exact"] = bool(np.array_equal(ocm[i], orc["crop_mask"][i]))
        rec["crop_bit_exact_vs_oracle"] = bool(np.array_equal(g_depth[i], orc["crop"][i]))
        # conditioning of the oracle's selected mask (computed on the oracle side)
        cnd = orc["cond"][i]
        rec["near_px"], rec["near_px_by_eps"], rec["pose_shift"] = cnd["near_px"], cnd["near_px_by_eps"], cnd["pose_shift"]
        rec["conditioned"] = cnd["near_px"] == 0
        rec["pose_excusable"] = bool(cnd["pose_shift"][0] > tol["cen"] or cnd["pose_shift"][1] > tol["ang"])
        # how close to the threshold the pixels the two sides disagree on are
        diff = np.logical_xor(d2g, d2w)
        rec["sel_diff_min_dist"] = float(np.abs(wp[keep[0]][diff] - 0.5).min()) if keep and diff.any() else None
    frames = stats["frames"]
    n_pose = sum(r["pose_non_nan"] for r in frames)
    n_sel = sum(r["sel_mask_identical"] for r in frames)
    exact_vs = [r["crop_bit_exact_vs_oracle"] for r in frames if r["pose_non_nan"]]
    stats["summary"] = {"frames": B, "non_nan_poses": n_pose, "sel_mask_identical": n_sel,
                        "pose_bit_exact": sum(r["pose_bit_exact"] for r in frames),
                        "crop_bit_exact_vs_oracle_non_nan": [sum(exact_vs), len(exact_vs)]}
    det_ok = pose_ok = 0
    excluded = []
    fails = {"box": 0, "score": 0, "mask": 0, "kp": 0}
    for rec in frames:
        assert max(rec["feat_rel_err"].values()) <= tol["feat"], rec
        assert rec["ndet"][0] == rec["ndet"][1], rec
        assert rec["cleaned_bit_exact"], rec
        assert rec["crop_bit_exact_same_pose"], rec
        # the crop kernel at the oracle's pose reproduces the oracle's window and
        # depth crop (same prepped frames); the mask crop of the GPU's selected
        # mask equals the oracle's wherever the selected masks agree
        assert rec["window_oracle_pose"][0] == rec["window_oracle_pose"][1], rec
        assert rec["crop_oracle_pose_bit_exact"], rec
        if rec["sel_mask_identical"]:
            assert rec["crop_mask_oracle_pose_bit_exact"], rec
        checks = {"box": rec["box_iou_min"] >= tol["box_iou"], "score": rec["score_diff_max"] <= tol["score"],
                  "mask": all(_mask_ok(x, tol["mask_px"]) for x in rec["mask_px"]),
                  "kp": rec["kp_within_1px"] >= tol["kp"]}
        rec["failed_checks"] = [k for k, v in checks.items() if not v]
        for k in rec["failed_checks"]:
            fails[k] += 1
        det = all(checks.values())
        a, b = rec["angle"]
        pose = (_mask_ok(rec["sel_mask_px"], tol["mask_px"]) and
                _close_nan(rec["centroid"][0], rec["centroid"][1], tol["cen"]) and
                ((np.isnan(a) and np.isnan(b)) or (not np.isnan(a) and not np.isnan(b) and
                                                   _ang_diff(a, b) <= tol["ang"])))
        rec["detections_ok"], rec["pose_ok"] = bool(det), bool(pose)
        det_ok += int(det)
        pose_ok += int(pose)
        if not rec["conditioned"]:
            excluded.append({"frame": rec["frame"], "near_px": rec["near_px"], "pose_shift": rec["pose_shift"],
                             "reason": f"{rec['near_px']} px of the oracle's selected mask within {NEAR_EPS} of the "
                                       "0.5 paste threshold: excluded from MIN_SEL_EXACT" +
                                       ("; flipping them moves the oracle pose past the bounds: pose bound excused"
                                        if rec["pose_excusable"] else ""),
                             "sel_mask_identical": rec["sel_mask_identical"], "pose_ok": bool(pose)})
        if dtype == "fp32":
            assert det, rec
            assert pose or (not rec["conditioned"] and rec["pose_excusable"]), rec
            if rec["sel_mask_identical"]:
                # identical selected mask => the chain is integer-exact
                assert rec["centroid_bit_exact"] and rec["angle_ulps"] <= ANGLE_ULPS, rec
                assert rec["crop_bit_exact_vs_oracle"], rec
    n_cond = sum(r["conditioned"] for r in frames)
    n_sel_cond = sum(r["sel_mask_identical"] for r in frames if r["conditioned"])
    stats["excluded"] = excluded
    stats["summary"].update(detections_ok=det_ok, pose_ok=pose_ok, failed_checks=fails, conditioned=n_cond,
                            sel_mask_identical_conditioned=n_sel_cond,
                            pose_outside_bounds=sum(1 for r in frames if not r["pose_ok"]))
    assert n_pose >= MIN_POSES[orc["cfg"].depth], stats["summary"]
    if dtype == "fp32":
        assert n_sel_cond >= MIN_SEL_EXACT * n_cond, stats["summary"]
    elif dtype == "mixed":
        assert det_ok == B and pose_ok == B, stats["summary"]
        assert sum(exact_vs) >= MIXED_CROP_EXACT * len(exact_vs), stats["summary"]
    else:  # fp16: the per-case floor (the fractions over several cases: test_forward_full_frame_fp16_seeds)
        assert det_ok >= FP16_FRAMES_MIN * B and pose_ok >= FP16_FRAMES_MIN * B, stats["summary"]
