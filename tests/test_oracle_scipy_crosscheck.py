"""The C frame-op oracle's median and morphology (oracle/frameops.c) against
an independent implementation of the same OpenCV semantics, SciPy's
ndimage, on random and extreme uint8 frames.  CPU only.

cv2 is not importable here, so these ops stay unpinned to OpenCV itself
(DESIGN.md section 4); this checks the restatement of the documented
semantics the reference calls (M/proc/proc.py:480-515 clean_frames):
  * cv2.medianBlur(ksize=3): borders replicated -- scipy median_filter,
    mode 'nearest';
  * cv2.erode / cv2.dilate with the default border (BORDER_CONSTANT at
    morphologyDefaultBorderValue: the border never wins the min / max) --
    grey_erosion with cval 255, grey_dilation with cval 0, the structuring
    element anchored at its centre;
  * cv2.morphologyEx(op, kernel, iterations=k): OPEN = k erosions then k
    dilations, CLOSE = k dilations then k erosions."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import frameops as F


def _frames(seed, n=3, h=37, w=53):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, h, w), dtype=np.uint8)
    f[0, :5] = 0          # flat runs and extremes at the borders
    f[0, -3:, :] = 255
    f[1, :, :4] = 255
    f[2] = (rng.random((h, w)) < 0.1).astype(np.uint8) * 255  # sparse speckle (the mask case)
    return f


def _scipy_morph(f, op, strel, iters):
    fp = strel.astype(bool)
    ero = lambda a: ndimage.grey_erosion(a, footprint=fp, mode="constant", cval=255)  # noqa: E731
    dil = lambda a: ndimage.grey_dilation(a, footprint=fp, mode="constant", cval=0)  # noqa: E731
    seq = {"erode": [ero] * iters, "dilate": [dil] * iters,
           "open": [ero] * iters + [dil] * iters, "close": [dil] * iters + [ero] * iters}[op]
    out = []
    for img in f:
        a = img
        for g in seq:
            a = g(a)
        out.append(a)
    return np.stack(out)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_median3_equals_scipy_nearest(seed):
    f = _frames(seed)
    want = np.stack([ndimage.median_filter(img, size=3, mode="nearest") for img in f])
    np.testing.assert_array_equal(F.median3(f), want)


@pytest.mark.parametrize("op", ["erode", "dilate", "open", "close"])
@pytest.mark.parametrize("strel", ["ellipse9", "ellipse5", "rect3x5", "cross3"])
@pytest.mark.parametrize("iters", [1, 3])
def test_morph_equals_scipy(op, strel, iters):
    k = {"ellipse9": F.ellipse_strel((9, 9)), "ellipse5": F.ellipse_strel((5, 5)),
         "rect3x5": np.ones((3, 5), np.uint8),
         "cross3": np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], np.uint8)}[strel]
    f = _frames(7)
    np.testing.assert_array_equal(F.morph(f, op, k, iters), _scipy_morph(f, op, k, iters))


def test_clean_frames_chain_equals_scipy():
    """The extract chain: medianBlur(3), then MORPH_OPEN with the 9x9
    ellipse, 3 iterations (ExtractConfig.iters_tail)."""
    f = _frames(11, n=3, h=64, w=80)
    med = np.stack([ndimage.median_filter(img, size=3, mode="nearest") for img in f])
    want = _scipy_morph(med, "open", F.ellipse_strel(), 3)
    np.testing.assert_array_equal(F.clean_frames(f, iters_tail=3), want)
