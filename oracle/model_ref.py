"""PyTorch-CPU fp32 restatement of the reference's model forward.

TEST INFRASTRUCTURE ONLY (checker + cpu_baseline).  Detectron2 and torchvision
are not in this image and their versions are unpinned in the reference
(README.md:16, setup.py:25-48), so their inference semantics are restated here
from their published code, with plain torch ops only:

* Predictor.__call__              M/model/predict.py:53-102 (1->3 channel
                                  replication, per-image CHW tensors)
* GeneralizedRCNN.preprocess      (x - PIXEL_MEAN) / PIXEL_STD, zero pad to /32
* ResNet (FrozenBN, STRIDE_IN_1X1) + FPN (GN, avg fuse, LastLevelMaxPool)
                                  config: M/model/config.py:21-94
* RPN: StandardRPNHead, DefaultAnchorGenerator, find_top_rpn_proposals
  (per-level topk, decode, clip, nonempty, per-level NMS 0.7, top 1000)
* ROIPooler(ROIAlignV2) = torchvision roi_align(aligned=True, sampling 0)
  (roi_align / nms below restate torchvision's CPU kernels in torch; the
  forward runs their C twins in model_ops.c, bit-identical and ~100x faster)
* FastRCNNConvFCHead + fast_rcnn_inference_single_image
* MaskRCNNConvUpsampleHead + mask_rcnn_inference + paste_masks_in_image
* KRCNNConvDeconvUpsampleHead + heatmaps_to_keypoints
* detector_postprocess            (M/model/util.py:45-62)

``forward(sd, cfg, images_u8)`` returns per-image dicts with the Instances
fields the reference's downstream code reads plus a dict of
intermediates for stage-wise parity tests.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_CLIB = None


def _clib():
    """model_ops.c (torchvision's CPU roi_align / nms kernels restated in C;
    bit-identical to the torch restatements below, which stay as their
    cross-check)."""
    global _CLIB
    if _CLIB is None:
        so = os.path.join(_HERE, "liboracle_model.so")
        src = os.path.join(_HERE, "model_ops.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(so)
        P, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        lib.orc_roi_align.argtypes = [P, i32, i32, i32, i32, P, i32, i32, f32, i32, i32, P]
        lib.orc_nms.argtypes = [P, P, i32, f32, P]
        lib.orc_nms.restype = i32
        _CLIB = lib
    return _CLIB


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def roi_align_c(feat, rois, out_size, scale, sampling_ratio, aligned):
    """roi_align through model_ops.c (same values as roi_align below)."""
    feat = feat.detach().to(torch.float32).contiguous()
    rois = rois.detach().to(torch.float32).contiguous()
    N, C, H, W = feat.shape
    out = torch.empty((rois.shape[0], C, out_size, out_size), dtype=torch.float32)
    if rois.shape[0]:
        _clib().orc_roi_align(_ptr(feat), N, C, H, W, _ptr(rois), rois.shape[0], out_size, float(scale),
                              int(sampling_ratio), int(bool(aligned)), _ptr(out))
    return out


def nms_c(boxes, scores, thresh):
    """nms through model_ops.c (same result as nms below)."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64)
    order = torch.sort(scores, descending=True, stable=True)[1].contiguous()
    b = boxes.detach().to(torch.float32).contiguous()
    keep = torch.empty(len(order), dtype=torch.int64)
    n = _clib().orc_nms(_ptr(b), _ptr(order), len(order), float(thresh), _ptr(keep))
    return keep[:n].clone()


# ---------------------------------------------------------------- backbone
def _frozen_bn(x, sd, p):
    # FrozenBatchNorm2d: scale = w * rsqrt(var + eps); bias = b - mean * scale
    scale = sd[p + ".weight"] * (sd[p + ".running_var"] + 1e-5).rsqrt()
    bias = sd[p + ".bias"] - sd[p + ".running_mean"] * scale
    return x * scale.view(1, -1, 1, 1) + bias.view(1, -1, 1, 1)


def _conv_bn(x, sd, p, stride=1, padding=0, relu=True):
    y = F.conv2d(x, sd[p + ".weight"], None, stride, padding)
    y = _frozen_bn(y, sd, p + ".norm")
    return F.relu(y) if relu else y


def resnet(x, sd, cfg):
    specs = _stage_specs(cfg)
    bu = "backbone.bottom_up"
    x = _conv_bn(x, sd, f"{bu}.stem.conv1", 2, 3)
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    outs = {}
    for name, nb, _cin, _bott, _cout, stride in specs:
        for b in range(nb):
            p = f"{bu}.{name}.{b}"
            s = stride if b == 0 else 1
            s1, s3 = (s, 1) if cfg.stride_in_1x1 else (1, s)
            sc = _conv_bn(x, sd, f"{p}.shortcut", s, 0, relu=False) if f"{p}.shortcut.weight" in sd else x
            y = _conv_bn(x, sd, f"{p}.conv1", s1, 0)
            y = _conv_bn(y, sd, f"{p}.conv2", s3, 1)
            y = _conv_bn(y, sd, f"{p}.conv3", 1, 0, relu=False)
            x = F.relu(y + sc)
        outs[name] = x
    return outs


def _stage_specs(cfg):
    specs = []
    in_ch, out_ch = cfg.stem_out_channels, cfg.res2_out_channels
    bott = cfg.num_groups * cfg.width_per_group
    for i, n in enumerate(cfg.res_blocks):
        specs.append((f"res{i + 2}", n, in_ch, bott, out_ch, 1 if i == 0 else 2))
        in_ch, out_ch, bott = out_ch, out_ch * 2, bott * 2
    return specs


def _fpn_conv(x, sd, p, cfg, padding):
    y = F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), 1, padding)
    if cfg.fpn_norm == "GN":
        y = F.group_norm(y, cfg.gn_groups, sd[p + ".norm.weight"], sd[p + ".norm.bias"], cfg.gn_eps)
    return y


def fpn(res, sd, cfg):
    names = ["res2", "res3", "res4", "res5"]
    lv = cfg.fpn_levels
    prev = _fpn_conv(res[names[-1]], sd, f"backbone.fpn_lateral{lv[-1]}", cfg, 0)
    results = [_fpn_conv(prev, sd, f"backbone.fpn_output{lv[-1]}", cfg, 1)]
    for idx in range(len(names) - 2, -1, -1):
        top_down = F.interpolate(prev, scale_factor=2.0, mode="nearest")
        lat = _fpn_conv(res[names[idx]], sd, f"backbone.fpn_lateral{lv[idx]}", cfg, 0)
        prev = lat + top_down
        if cfg.fpn_fuse_type == "avg":
            prev = prev / 2
        results.insert(0, _fpn_conv(prev, sd, f"backbone.fpn_output{lv[idx]}", cfg, 1))
    results.append(F.max_pool2d(results[-1], kernel_size=1, stride=2, padding=0))  # p6
    return {f"p{l}": r for l, r in zip(lv + [lv[-1] + 1], results)}


# ---------------------------------------------------------------- boxes
def apply_deltas(deltas, boxes, weights, clamp):
    deltas = deltas.float()
    boxes = boxes.to(deltas.dtype)
    widths = boxes[:, 2] - boxes[:, 0]
    heights = boxes[:, 3] - boxes[:, 1]
    ctr_x = boxes[:, 0] + 0.5 * widths
    ctr_y = boxes[:, 1] + 0.5 * heights
    wx, wy, ww, wh = weights
    dx = deltas[:, 0::4] / wx
    dy = deltas[:, 1::4] / wy
    dw = deltas[:, 2::4] / ww
    dh = deltas[:, 3::4] / wh
    dw = torch.clamp(dw, max=clamp)
    dh = torch.clamp(dh, max=clamp)
    pred_ctr_x = dx * widths[:, None] + ctr_x[:, None]
    pred_ctr_y = dy * heights[:, None] + ctr_y[:, None]
    pred_w = torch.exp(dw) * widths[:, None]
    pred_h = torch.exp(dh) * heights[:, None]
    x1 = pred_ctr_x - 0.5 * pred_w
    y1 = pred_ctr_y - 0.5 * pred_h
    x2 = pred_ctr_x + 0.5 * pred_w
    y2 = pred_ctr_y + 0.5 * pred_h
    return torch.stack((x1, y1, x2, y2), dim=-1).reshape(deltas.shape)


def clip_boxes(b, h, w):
    x1 = b[:, 0].clamp(min=0, max=w)
    y1 = b[:, 1].clamp(min=0, max=h)
    x2 = b[:, 2].clamp(min=0, max=w)
    y2 = b[:, 3].clamp(min=0, max=h)
    return torch.stack((x1, y1, x2, y2), dim=-1)


def nms(boxes, scores, thresh):
    """torchvision.ops.nms (CPU kernel): stable descending sort, suppress IoU > thresh."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64)
    order = torch.sort(scores, descending=True, stable=True)[1]
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    b = boxes.numpy(); a = areas.numpy(); o = order.numpy()
    sup = np.zeros(len(o), bool)
    keep = []
    for _i in range(len(o)):
        i = o[_i]
        if sup[i]:
            continue
        keep.append(i)
        ix1, iy1, ix2, iy2 = b[i]
        rest = o[_i + 1:]
        xx1 = np.maximum(np.float32(ix1), b[rest, 0]); yy1 = np.maximum(np.float32(iy1), b[rest, 1])
        xx2 = np.minimum(np.float32(ix2), b[rest, 2]); yy2 = np.minimum(np.float32(iy2), b[rest, 3])
        w = np.maximum(np.float32(0), xx2 - xx1); h = np.maximum(np.float32(0), yy2 - yy1)
        inter = w * h
        ovr = inter / (a[i] + a[rest] - inter)
        sup[rest[ovr > thresh]] = True
    return torch.as_tensor(np.array(keep, np.int64))


def batched_nms(boxes, scores, idxs, thresh):
    """torchvision batched_nms, per-class form (_batched_nms_vanilla)."""
    keep_mask = torch.zeros_like(scores, dtype=torch.bool)
    for c in torch.unique(idxs):
        ci = torch.where(idxs == c)[0]
        keep_mask[ci[nms_c(boxes[ci], scores[ci], thresh)]] = True
    keep = torch.where(keep_mask)[0]
    return keep[scores[keep].sort(descending=True, stable=True)[1]]


def anchors_for(cfg, level_idx, H, W):
    size = cfg.anchor_sizes[level_idx]
    stride = 2 ** (level_idx + 2)
    cell = []
    for ar in cfg.aspect_ratios:
        area = float(size) ** 2.0
        w = math.sqrt(area / ar)
        h = ar * w
        cell.append([-w / 2.0, -h / 2.0, w / 2.0, h / 2.0])
    cell = torch.tensor(cell)
    off = cfg.anchor_offset * stride
    sx = torch.arange(off, W * stride, step=stride, dtype=torch.float32)
    sy = torch.arange(off, H * stride, step=stride, dtype=torch.float32)
    yy, xx = torch.meshgrid(sy, sx, indexing="ij")
    xx, yy = xx.reshape(-1), yy.reshape(-1)
    shifts = torch.stack((xx, yy, xx, yy), dim=1)
    return (shifts.view(-1, 1, 4) + cell.view(1, -1, 4)).reshape(-1, 4)


def rpn_heads(feats, sd, cfg):
    A = len(cfg.aspect_ratios)
    p = "proposal_generator.rpn_head"
    logits, deltas, anchors = [], [], []
    for i, l in enumerate(range(2, 7)):
        x = feats[f"p{l}"]
        t = F.relu(F.conv2d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], padding=1))
        o = F.conv2d(t, sd[p + ".objectness_logits.weight"], sd[p + ".objectness_logits.bias"])
        d = F.conv2d(t, sd[p + ".anchor_deltas.weight"], sd[p + ".anchor_deltas.bias"])
        N, _, Hh, Ww = o.shape
        logits.append(o.permute(0, 2, 3, 1).flatten(1))
        deltas.append(d.view(N, A, 4, Hh, Ww).permute(0, 3, 4, 1, 2).flatten(1, -2))
        anchors.append(anchors_for(cfg, i, Hh, Ww))
    return logits, deltas, anchors


def find_top_rpn_proposals(logits, deltas, anchors, cfg, image_size):
    N = logits[0].shape[0]
    h, w = image_size
    out = []
    for n in range(N):
        boxes_l, scores_l, lvl_l = [], [], []
        for li in range(len(logits)):
            k = min(cfg.rpn_pre_nms_topk_test, logits[li].shape[1])
            sc, idx = logits[li][n].topk(k, sorted=True)
            props = apply_deltas(deltas[li][n][idx], anchors[li][idx], cfg.rpn_bbox_reg_weights, cfg.bbox_reg_clamp)
            boxes_l.append(props); scores_l.append(sc); lvl_l.append(torch.full((k,), li, dtype=torch.int64))
        boxes = torch.cat(boxes_l); scores = torch.cat(scores_l); lvl = torch.cat(lvl_l)
        valid = torch.isfinite(boxes).all(dim=1) & torch.isfinite(scores)
        boxes, scores, lvl = boxes[valid], scores[valid], lvl[valid]
        boxes = clip_boxes(boxes, h, w)
        ws, hs = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
        keep = (ws > cfg.rpn_min_box_size) & (hs > cfg.rpn_min_box_size)
        boxes, scores, lvl = boxes[keep], scores[keep], lvl[keep]
        keep = batched_nms(boxes, scores, lvl, cfg.rpn_nms_thresh)[:cfg.rpn_post_nms_topk_test]
        out.append((boxes[keep], scores[keep]))
    return out


def rpn(feats, sd, cfg, image_size):
    logits, deltas, anchors = rpn_heads(feats, sd, cfg)
    return find_top_rpn_proposals(logits, deltas, anchors, cfg, image_size)


# ---------------------------------------------------------------- pooler
def roi_align(feat, rois, out_size, scale, sampling_ratio, aligned, chunk=256):
    """torchvision.ops.roi_align CPU semantics (roi_align_kernel.cpp), vectorised
    over ROIs/bins/samples with the kernel's float32 operation order.
    feat (N,C,H,W) float32; rois (R,5) = (batch, x1, y1, x2, y2)."""
    R = rois.shape[0]
    N, C, H, W = feat.shape
    P = out_size
    out = torch.zeros((R, C, P, P), dtype=torch.float32)
    f32 = torch.float32
    sc = torch.tensor(scale, dtype=f32)
    off = torch.tensor(0.5 if aligned else 0.0, dtype=f32)
    for r0 in range(0, R, chunk):
        rr = rois[r0:r0 + chunk].to(f32)
        n = rr.shape[0]
        b = rr[:, 0].to(torch.int64)
        sw = rr[:, 1] * sc - off
        sh = rr[:, 2] * sc - off
        ew = rr[:, 3] * sc - off
        eh = rr[:, 4] * sc - off
        rw, rh = ew - sw, eh - sh
        if not aligned:
            rw, rh = rw.clamp(min=1.0), rh.clamp(min=1.0)
        bh = rh / torch.tensor(float(P), dtype=f32)
        bw = rw / torch.tensor(float(P), dtype=f32)
        if sampling_ratio > 0:
            gh = torch.full((n,), sampling_ratio, dtype=torch.int64)
            gw = gh.clone()
        else:
            gh = torch.ceil(rh / torch.tensor(float(P), dtype=f32)).to(torch.int64)
            gw = torch.ceil(rw / torch.tensor(float(P), dtype=f32)).to(torch.int64)
        count = (gh * gw).clamp(min=1).to(f32)
        G = int(max(int(gh.max()), int(gw.max()), 1))
        it = torch.arange(G, dtype=f32) + 0.5                         # (iy + .5f)
        ph = torch.arange(P, dtype=f32)
        # yy[r, ph, iy] = sh + ph*bh + (iy+.5)*bh/gh
        yy = (sh[:, None, None] + ph[None, :, None] * bh[:, None, None]) + \
            (it[None, None, :] * bh[:, None, None]) / gh.to(f32)[:, None, None]
        xx = (sw[:, None, None] + ph[None, :, None] * bw[:, None, None]) + \
            (it[None, None, :] * bw[:, None, None]) / gw.to(f32)[:, None, None]
        vy = torch.arange(G)[None, None, :] < gh[:, None, None]
        vx = torch.arange(G)[None, None, :] < gw[:, None, None]

        def prep(v, size):
            # a zero-size ROI has grid 0 (no samples; masked by vy / vx below)
            # and NaN positions: keep its gather indices in range
            v = torch.where(torch.isfinite(v), v, torch.zeros_like(v))
            empty = (v < -1.0) | (v > size)
            v = torch.where(v <= 0, torch.zeros_like(v), v)
            lo = v.to(torch.int64)
            top = lo >= size - 1
            lo = torch.where(top, torch.full_like(lo, size - 1), lo)
            hi = torch.where(top, lo, lo + 1)
            v = torch.where(top, lo.to(f32), v)
            l = v - lo.to(f32)
            h = 1.0 - l
            return empty, lo, hi, l, h

        ey, yl, yh, ly, hy = prep(yy, H)   # (n, P, G)
        ex, xl, xh, lx, hx = prep(xx, W)
        # combine to (n, P(ph), P(pw), G(iy), G(ix))
        def E(t, ax):  # expand y-terms along pw/ix, x-terms along ph/iy
            return t[:, :, None, :, None] if ax == "y" else t[:, None, :, None, :]
        w1 = E(hy, "y") * E(hx, "x"); w2 = E(hy, "y") * E(lx, "x")
        w3 = E(ly, "y") * E(hx, "x"); w4 = E(ly, "y") * E(lx, "x")
        valid = (E(vy, "y") & E(vx, "x")) & ~(E(ey, "y") | E(ex, "x"))
        fb = feat[b]                                                   # (n, C, H, W)
        flat = fb.reshape(n, C, H * W)

        def g(yi, xi):
            idx = (E(yi, "y") * W + E(xi, "x")).reshape(n, 1, -1).expand(n, C, -1)
            return torch.gather(flat, 2, idx).reshape(n, C, P, P, G, G)
        v = (w1[:, None] * g(yl, xl) + w2[:, None] * g(yl, xh)) + w3[:, None] * g(yh, xl)
        v = v + w4[:, None] * g(yh, xh)
        v = torch.where(valid[:, None], v, torch.zeros_like(v))
        acc = torch.zeros((n, C, P, P), dtype=f32)
        for iy in range(G):
            for ix in range(G):
                acc = acc + v[..., iy, ix]
        out[r0:r0 + n] = acc / count[:, None, None, None]
    return out


def pooler(feats, boxes_per_image, out_size, cfg):
    """ROIPooler: FPN level assignment + ROIAlignV2 over p2..p5."""
    lv = cfg.fpn_levels
    boxes = torch.cat([b for b in boxes_per_image]) if boxes_per_image else torch.zeros((0, 4))
    bidx = torch.cat([torch.full((len(b),), i, dtype=torch.float32) for i, b in enumerate(boxes_per_image)])
    rois = torch.cat([bidx[:, None], boxes], dim=1)
    C = feats[f"p{lv[0]}"].shape[1]
    out = torch.zeros((len(boxes), C, out_size, out_size))
    if len(boxes) == 0:
        return out
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    lvl = torch.floor(cfg.canonical_level + torch.log2(torch.sqrt(area) / cfg.canonical_box_size + 1e-8))
    lvl = torch.clamp(lvl, min=lv[0], max=lv[-1]).to(torch.int64) - lv[0]
    for li, l in enumerate(lv):
        sel = torch.where(lvl == li)[0]
        if len(sel):
            out[sel] = roi_align_c(feats[f"p{l}"], rois[sel], out_size, 1.0 / 2 ** l, cfg.pooler_sampling_ratio,
                                   cfg.pooler_aligned)
    return out


# ---------------------------------------------------------------- heads
def box_head(x, sd, cfg):
    x = x.flatten(1)
    for i in range(cfg.box_num_fc):
        x = F.relu(F.linear(x, sd[f"roi_heads.box_head.fc{i + 1}.weight"], sd[f"roi_heads.box_head.fc{i + 1}.bias"]))
    cls = F.linear(x, sd["roi_heads.box_predictor.cls_score.weight"], sd["roi_heads.box_predictor.cls_score.bias"])
    reg = F.linear(x, sd["roi_heads.box_predictor.bbox_pred.weight"], sd["roi_heads.box_predictor.bbox_pred.bias"])
    return cls, reg


def fast_rcnn_inference_single(boxes, scores, image_shape, score_thresh, nms_thresh, topk):
    valid = torch.isfinite(boxes).all(dim=1) & torch.isfinite(scores).all(dim=1)
    if not valid.all():
        boxes, scores = boxes[valid], scores[valid]
    scores = scores[:, :-1]
    num_bbox_reg_classes = boxes.shape[1] // 4
    boxes = clip_boxes(boxes.reshape(-1, 4), *image_shape).view(-1, num_bbox_reg_classes, 4)
    filter_mask = scores > score_thresh
    filter_inds = filter_mask.nonzero()
    if num_bbox_reg_classes == 1:
        boxes = boxes[filter_inds[:, 0], 0]
    else:
        boxes = boxes[filter_mask]
    scores = scores[filter_mask]
    keep = batched_nms(boxes, scores, filter_inds[:, 1], nms_thresh)
    if topk >= 0:
        keep = keep[:topk]
    return boxes[keep], scores[keep], filter_inds[keep, 1]


def mask_head(x, sd, cfg):
    for i in range(cfg.mask_num_conv):
        x = F.relu(F.conv2d(x, sd[f"roi_heads.mask_head.mask_fcn{i + 1}.weight"],
                            sd[f"roi_heads.mask_head.mask_fcn{i + 1}.bias"], padding=1))
    x = F.relu(F.conv_transpose2d(x, sd["roi_heads.mask_head.deconv.weight"], sd["roi_heads.mask_head.deconv.bias"],
                                  stride=2))
    return F.conv2d(x, sd["roi_heads.mask_head.predictor.weight"], sd["roi_heads.mask_head.predictor.bias"])


def keypoint_head(x, sd, cfg):
    for i in range(len(cfg.keypoint_conv_dims)):
        x = F.relu(F.conv2d(x, sd[f"roi_heads.keypoint_head.conv_fcn{i + 1}.weight"],
                            sd[f"roi_heads.keypoint_head.conv_fcn{i + 1}.bias"], padding=1))
    x = F.conv_transpose2d(x, sd["roi_heads.keypoint_head.score_lowres.weight"],
                           sd["roi_heads.keypoint_head.score_lowres.bias"], stride=2, padding=4 // 2 - 1)
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def heatmaps_to_keypoints(maps, rois):
    offset_x = rois[:, 0]
    offset_y = rois[:, 1]
    widths = (rois[:, 2] - rois[:, 0]).clamp(min=1)
    heights = (rois[:, 3] - rois[:, 1]).clamp(min=1)
    widths_ceil = widths.ceil()
    heights_ceil = heights.ceil()
    num_rois, num_keypoints = maps.shape[:2]
    xy_preds = maps.new_zeros(rois.shape[0], num_keypoints, 4)
    width_corrections = widths / widths_ceil
    height_corrections = heights / heights_ceil
    kidx = torch.arange(num_keypoints)
    for i in range(num_rois):
        outsize = (int(heights_ceil[i]), int(widths_ceil[i]))
        roi_map = F.interpolate(maps[[i]], size=outsize, mode="bicubic", align_corners=False)
        roi_map = roi_map.reshape(roi_map.shape[1:])
        max_score, _ = roi_map.view(num_keypoints, -1).max(1)
        max_score = max_score.view(num_keypoints, 1, 1)
        tmp_full = (roi_map - max_score).exp_()
        tmp_pool = (maps[i] - max_score).exp_()
        roi_map_scores = tmp_full / tmp_pool.sum((1, 2), keepdim=True)
        w = roi_map.shape[2]
        pos = roi_map.view(num_keypoints, -1).argmax(1)
        x_int = pos % w
        y_int = (pos - x_int) // w
        x = (x_int.float() + 0.5) * width_corrections[i]
        y = (y_int.float() + 0.5) * height_corrections[i]
        xy_preds[i, :, 0] = x + offset_x[i]
        xy_preds[i, :, 1] = y + offset_y[i]
        xy_preds[i, :, 2] = roi_map[kidx, y_int, x_int]
        xy_preds[i, :, 3] = roi_map_scores[kidx, y_int, x_int]
    return xy_preds


def paste_masks(masks, boxes, img_h, img_w, threshold=0.5):
    """paste_masks_in_image (skip_empty=False form; identical values).
    threshold=None returns the pasted probabilities (test margins)."""
    N = masks.shape[0]
    if N == 0:
        return torch.zeros((N, img_h, img_w), dtype=torch.bool if threshold is not None else torch.float32)
    x0, y0, x1, y1 = torch.split(boxes, 1, dim=1)
    img_y = torch.arange(0, img_h, dtype=torch.float32) + 0.5
    img_x = torch.arange(0, img_w, dtype=torch.float32) + 0.5
    img_y = (img_y - y0) / (y1 - y0) * 2 - 1
    img_x = (img_x - x0) / (x1 - x0) * 2 - 1
    gx = img_x[:, None, :].expand(N, img_y.size(1), img_x.size(1))
    gy = img_y[:, :, None].expand(N, img_y.size(1), img_x.size(1))
    grid = torch.stack([gx, gy], dim=3)
    img_masks = F.grid_sample(masks[:, None].float(), grid, align_corners=False)[:, 0]
    return img_masks if threshold is None else img_masks >= threshold


# ---------------------------------------------------------------- forward
def preprocess(images_u8, sd, cfg):
    """images_u8: uint8 (N, H, W, 1|3) already scaled (scale_raw_frames)."""
    x = torch.as_tensor(np.ascontiguousarray(images_u8))
    if cfg.input_format == "RGB" and x.shape[3] == 1:
        x = torch.cat([x] * 3, dim=3)
    x = x.permute(0, 3, 1, 2).float()
    x = (x - sd["pixel_mean"].view(1, -1, 1, 1)) / sd["pixel_std"].view(1, -1, 1, 1)
    N, C, H, W = x.shape
    d = cfg.size_divisibility
    Hp, Wp = (H + d - 1) // d * d, (W + d - 1) // d * d
    out = torch.zeros((N, C, Hp, Wp))
    out[:, :, :H, :W] = x
    return out, (H, W)


@torch.no_grad()
def forward(sd: Dict[str, torch.Tensor], cfg, images_u8: np.ndarray, keep_intermediates: bool = True):
    x, (h, w) = preprocess(images_u8, sd, cfg)
    inter = {"input": x}
    res = resnet(x, sd, cfg)
    feats = fpn(res, sd, cfg)
    inter.update(res)
    inter.update(feats)
    props = rpn(feats, sd, cfg, (h, w))
    inter["proposals"] = props
    pbox = [p[0] for p in props]
    bx = pooler(feats, pbox, cfg.box_pooler_resolution, cfg)
    inter["box_pooled"] = bx
    cls, reg = box_head(bx, sd, cfg)
    inter["box_cls"], inter["box_reg"] = cls, reg
    scores_all = F.softmax(cls, dim=-1)
    boxes_all = apply_deltas(reg, torch.cat(pbox), cfg.box_reg_weights, cfg.bbox_reg_clamp)
    results = []
    start = 0
    for b, pb in enumerate(pbox):
        n = len(pb)
        bb, ss, cc = fast_rcnn_inference_single(boxes_all[start:start + n], scores_all[start:start + n], (h, w),
                                                cfg.score_thresh_test, cfg.nms_thresh_test, cfg.detections_per_image)
        start += n
        # detector_postprocess: scale 1, clip, nonempty
        bb = clip_boxes(bb, h, w)
        ne = ((bb[:, 2] - bb[:, 0]) > 0) & ((bb[:, 3] - bb[:, 1]) > 0)
        results.append({"pred_boxes": bb[ne], "scores": ss[ne], "pred_classes": cc[ne]})
    dboxes = [r["pred_boxes"] for r in results]
    if cfg.mask_on:
        mx = pooler(feats, dboxes, cfg.mask_pooler_resolution, cfg)
        ml = mask_head(mx, sd, cfg)
        inter["mask_logits"] = ml
        probs = ml.sigmoid()
        s = 0
        for r in results:
            n = len(r["pred_boxes"])
            cls_idx = r["pred_classes"]
            pm = probs[s:s + n][torch.arange(n), cls_idx] if n else probs[:0, 0]
            r["pred_mask_probs"] = paste_masks(pm, r["pred_boxes"], h, w, None)
            r["pred_masks"] = r["pred_mask_probs"] >= cfg.mask_threshold
            s += n
    if cfg.keypoint_on:
        kx = pooler(feats, dboxes, cfg.keypoint_pooler_resolution, cfg)
        kl = keypoint_head(kx, sd, cfg)
        inter["keypoint_logits"] = kl
        s = 0
        for r in results:
            n = len(r["pred_boxes"])
            hm = kl[s:s + n]
            kp = heatmaps_to_keypoints(hm, r["pred_boxes"]) if n else torch.zeros((0, cfg.num_keypoints, 4))
            r["pred_keypoints"] = kp[:, :, [0, 1, 3]]
            r["pred_keypoint_heatmaps"] = hm
            s += n
    return results, (inter if keep_intermediates else None)
