"""The C twins of the oracle's torchvision kernels (oracle/model_ops.c) equal
the torch restatements (oracle/model_ref.roi_align / nms) bit for bit, on the
cases torchvision's kernels branch on: samples outside the map, boxes on and
past the border, degenerate and huge boxes, adaptive and fixed sampling,
aligned and not, ties in the score order."""
import numpy as np
import pytest
import torch

from oracle import model_ref as R


def _rois(rng, n, H, W, scale):
    b = rng.integers(0, 2, n).astype(np.float32)
    x1 = rng.uniform(-40, W / scale + 20, n)
    y1 = rng.uniform(-40, H / scale + 20, n)
    w = np.exp(rng.uniform(-1, np.log(W / scale * 1.5), n))
    h = np.exp(rng.uniform(-1, np.log(H / scale * 1.5), n))
    r = np.stack([b, x1, y1, x1 + w, y1 + h], 1).astype(np.float32)
    r[:4, 3] = r[:4, 1]  # zero-width boxes
    r[4:8, 1:3] = -500  # fully outside
    return torch.from_numpy(r)


@pytest.mark.parametrize("aligned", [True, False])
@pytest.mark.parametrize("sampling", [0, 2])
@pytest.mark.parametrize("P", [7, 14])
def test_roi_align_c_equals_torch(aligned, sampling, P):
    rng = np.random.default_rng(P * 10 + sampling + aligned)
    H, W, scale = 13, 17, 0.25
    feat = torch.from_numpy(rng.standard_normal((2, 5, H, W)).astype(np.float32))
    rois = _rois(rng, 64, H, W, scale)
    a = R.roi_align(feat, rois, P, scale, sampling, aligned)
    b = R.roi_align_c(feat, rois, P, scale, sampling, aligned)
    assert torch.equal(a, b)


def test_roi_align_c_empty():
    feat = torch.zeros((1, 3, 4, 4))
    out = R.roi_align_c(feat, torch.zeros((0, 5)), 7, 1.0, 0, True)
    assert out.shape == (0, 3, 7, 7)


@pytest.mark.parametrize("seed", range(4))
def test_nms_c_equals_torch(seed):
    rng = np.random.default_rng(seed)
    n = 300
    xy = rng.uniform(0, 100, (n, 2))
    wh = rng.uniform(1, 40, (n, 2))
    boxes = torch.from_numpy(np.concatenate([xy, xy + wh], 1).astype(np.float32))
    scores = torch.from_numpy(rng.integers(0, 20, n).astype(np.float32))  # many ties
    for thr in (0.3, 0.5, 0.7):
        assert torch.equal(R.nms(boxes, scores, thr), R.nms_c(boxes, scores, thr))
    assert R.nms_c(boxes[:0], scores[:0], 0.5).numel() == 0
