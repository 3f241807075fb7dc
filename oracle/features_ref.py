"""numpy restatement of the host-side feature/selection logic (TEST
INFRASTRUCTURE ONLY).

* nms_mask_instances  M/pipeline/process_features_step.py:63-113 (mask-IoU
  NMS with the reference's deletion quirk), on (n, H, W) bool masks + scores.
* flips_ref           flips_from_keypoints (M/proc/proc.py:851-889), checker
                      of libmdx's mdx_flips_from_keypoints
* iterative_filter_angles_ref  filter_angles / iterative_filter_angles
                      (M/proc/proc.py:600-654), checker of
                      mdx_iterative_filter_angles
* frame_scalars_ref   the per-frame reductions of compute_scalars
  (M/proc/scalars.py:79-103) and the keypoint z lookup of keypoints_to_dict
  (M/proc/keypoints.py:122-130) -- checker of mdx_frame_scalars.
"""
from __future__ import annotations

import numpy as np


def nms_mask_instances(masks: np.ndarray, scores: np.ndarray, iou_threshold: float = 0.5):
    """Returns the picked instance indices (into the ORIGINAL instance list) in
    pick order, literally following the reference's loop."""
    n = len(scores)
    if n <= 1:
        return list(range(n))
    has_pos = masks.reshape(n, -1).any(axis=1)
    orig = np.where(has_pos)[0]
    masks = masks[has_pos]
    scores = scores[has_pos]
    idxs = np.argsort(scores, kind="stable")
    pick = []
    flat = masks.reshape(len(masks), -1).astype(np.int64)
    while len(idxs) > 0:
        last = len(idxs) - 1
        i = idxs[last]
        pick.append(i)
        m = flat[idxs]
        inter = m @ m.T
        areas = np.broadcast_to(m.sum(axis=1), (len(idxs), len(idxs)))
        union = areas + areas.T - inter
        ious = np.triu((inter.astype(np.float32) / union.astype(np.float32)), k=1)
        over = np.where(ious > iou_threshold)[0]
        idxs = np.delete(idxs, np.unique(np.concatenate(([last], over))))
    return [int(orig[p]) for p in pick]


def frame_scalars_ref(frames, masks, min_height, max_height, keypoints=None, z_frames=None):
    """(area_px int64 (n,), height_ave float64 (n,), z_data float64 (n,K) | None),
    literally as the reference computes them."""
    fm = frames if masks is None else frames * masks          # uint8 product
    masked = np.logical_and(fm > min_height, fm < max_height)
    area = np.sum(masked, axis=(1, 2)).astype(np.int64)
    hmean = np.zeros(fm.shape[0])
    for i in range(fm.shape[0]):
        if area[i] > 0:
            hmean[i] = np.mean(fm[i, masked[i]])
    z = None
    if keypoints is not None:
        zf = frames if z_frames is None else z_frames
        with np.errstate(invalid="ignore"):
            x = np.clip(np.floor(keypoints[:, :, 0]).astype(int), 0, zf.shape[2] - 1)
            y = np.clip(np.floor(keypoints[:, :, 1]).astype(int), 0, zf.shape[1] - 1)
        z = np.zeros((zf.shape[0], keypoints.shape[1]))
        for k in range(keypoints.shape[1]):
            z[:, k] = zf[np.arange(zf.shape[0]), y[:, k], x[:, k]]
    return area, hmean, z


def flips_ref(keypoints, centroids, angles, length=80):
    """(flips, confidence) of the keypoint head/tail vote, numpy."""
    kp = np.asarray(keypoints, np.float64)[:, :7]
    th = np.deg2rad(-np.asarray(angles, np.float64))[:, None]
    ox = centroids[:, 0:1]
    xr = np.cos(th) * (kp[..., 0] - ox) + (-np.sin(th)) * (kp[..., 1] - centroids[:, 1:2]) + ox
    half = np.asarray(length, np.float64) / 2
    near_min = np.abs((centroids[:, 0] - half)[:, None] - xr) < np.abs((centroids[:, 0] + half)[:, None] - xr)
    side = np.where(near_min, -1, 1)
    flips = side[:, :4].mean(axis=1) < side[:, 4:7].mean(axis=1)
    want_front = np.where(flips, -1, 1)[:, None]
    agree = (side[:, :4] == want_front).sum(axis=1) + (side[:, 4:7] == -want_front).sum(axis=1)
    return flips, agree / 7


def _trailing_nanmedian(x, window):
    out = np.empty(len(x))
    for i in range(len(x)):
        w = x[max(0, i - window + 1):i + 1]
        w = w[~np.isnan(w)]
        out[i] = np.median(w) if len(w) else np.nan
    return out


def iterative_filter_angles_ref(angles, window=3, tolerance=60, max_iters=1000):
    """The 180-degree jump filter repeated to a fixed point, with the
    reference's stop rule (np.allclose) and iteration cap, in plain numpy."""
    angles = np.asarray(angles, np.float64)
    cur = angles.copy()
    for _ in range(max_iters + 1):  # at most max_iters + 1 passes; the last pass's output is kept
        dev = cur - _trailing_nanmedian(cur, min(window, len(cur)))
        jump = (np.abs(dev) > 180 - tolerance) & (np.abs(dev) < 180 + tolerance)
        nxt = cur.copy()
        nxt[jump] = nxt[jump] - 180 * np.sign(dev[jump])
        done = np.allclose(nxt, cur)
        cur = nxt
        if done:
            break
    return cur, np.isclose(np.abs(cur - angles), 180)
