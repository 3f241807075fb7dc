"""numpy restatement of the host-side feature/selection logic (TEST
INFRASTRUCTURE ONLY).

* nms_mask_instances  M/pipeline/process_features_step.py:63-113 (mask-IoU
  NMS with the reference's deletion quirk), on (n, H, W) bool masks + scores.
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
