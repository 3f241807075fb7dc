"""Golden fixtures for session setup, produced by the
REFERENCE's own functions under /opt/conda/bin/python3.9 (real numpy 1.26,
scipy 1.7.1, scikit-image 0.18.3):

  plane_fit3 / plane_ransac   M/proc/roi.py:97-212   (seeded np.random)
  get_roi                     M/proc/roi.py:14-94    (skimage label/regionprops,
                                                      rankdata, binary_fill_holes)
  get_bground_im              M/proc/roi.py:293-307  (np.median part)

OpenCV is absent: the cv2 functions these call (getStructuringElement,
dilate, medianBlur) are provided by the small restatements below, so the
fixture pins everything around them but NOT OpenCV itself (its formulas are
restated from OpenCV's published imgproc source).

Run in the build container only (reads /root/reference):
    /opt/conda/bin/python3.9 tests/golden/make_golden_roi.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ref_roi.npz")


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    mod.__path__ = []
    mod.__getattr__ = lambda attr: type(attr, (), {}) if not attr.startswith("__") else None
    sys.modules[name] = mod
    return mod


def cv_strel(shape, ksize):
    """getStructuringElement: MORPH_RECT=0, MORPH_ELLIPSE=2 (OpenCV formula)."""
    w, h = ksize
    if shape == 0:
        return np.ones((h, w), np.uint8)
    r, c = h // 2, w // 2
    inv_r2 = 1.0 / (r * r) if r else 0.0
    k = np.zeros((h, w), np.uint8)
    for i in range(h):
        dy = i - r
        if abs(dy) <= r:
            dx = int(np.rint(c * np.sqrt((r * r - dy * dy) * inv_r2)))
            k[i, max(c - dx, 0):min(c + dx + 1, w)] = 1
    return k


def cv_dilate(img, kernel, iterations=1):
    out = np.asarray(img).copy()
    kh, kw = kernel.shape
    ay, ax = kh // 2, kw // 2
    H, W = out.shape
    for _ in range(iterations):
        src = out.copy()
        res = np.full_like(src, -np.inf, dtype=np.float64)
        for i in range(kh):
            for j in range(kw):
                if not kernel[i, j]:
                    continue
                dy, dx = i - ay, j - ax
                ys, ye = max(0, -dy), min(H, H - dy)
                xs, xe = max(0, -dx), min(W, W - dx)
                res[ys:ye, xs:xe] = np.maximum(res[ys:ye, xs:xe], src[ys + dy:ye + dy, xs + dx:xe + dx])
        out = res.astype(src.dtype)
    return out


def cv_median_blur(img, k):
    from scipy.ndimage import median_filter
    return median_filter(img, size=k, mode="nearest")


def install():
    import matplotlib.pyplot  # noqa: F401
    import pandas  # noqa: F401
    import scipy.signal  # noqa: F401
    import skimage.measure  # noqa: F401  (real)
    _stub("cv2", MORPH_ELLIPSE=2, MORPH_RECT=0, MORPH_OPEN=2, getStructuringElement=cv_strel, dilate=cv_dilate,
          medianBlur=cv_median_blur, INPAINT_NS=0, INPAINT_TELEA=1)
    _stub("h5py", File=object, Group=object, Dataset=object)
    _stub("ruamel")
    _stub("ruamel.yaml")
    _stub("pykalman", KalmanFilter=object)
    _stub("tifffile")
    _stub("imageio", imwrite=lambda *a, **k: None)
    _stub("detectron2")
    _stub("detectron2.data", MetadataCatalog=object, DatasetCatalog=object)
    _stub("detectron2.structures", Instances=object, Boxes=object)
    _stub("pycocotools")
    sys.path.insert(0, REF)


def arena(H=96, W=120, seed=0):
    """Floor plane at ~700 mm inside a circular arena, a wall ring out of
    range, a raised box (in range, off the floor plane) and a small floor
    patch disconnected from the arena; background median granularity .5."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    floor = 700 + 0.05 * xx - 0.03 * yy
    img = np.full((H, W), 560.0)                       # walls / rim: out of range
    r = np.hypot(yy - H / 2, xx - W / 2)
    img[r < 0.4 * H] = floor[r < 0.4 * H]
    img[5:15, 5:25] = floor[5:15, 5:25]                # disconnected floor patch
    img[70:85, 95:112] = 655.0                         # raised box, in range
    img += rng.normal(0, 0.8, img.shape)
    return np.round(img * 2) / 2


def main():
    install()
    from moseq2_detectron_extract.proc import roi as R
    from moseq2_detectron_extract.proc.util import select_strel
    fx = {}
    for k, seed in enumerate([3, 11]):
        img = arena(seed=k)
        np.random.seed(seed)
        plane, dist = R.plane_ransac(img, iters=200, progress_bar=False)
        fx[f"ransac_img_{k}"] = img
        fx[f"ransac_seed_{k}"] = np.array(seed)
        fx[f"ransac_plane_{k}"] = plane
        fx[f"ransac_dist_{k}"] = dist
        np.random.seed(seed)
        rois, plane2, bboxes, label_im, ranks, shape_index = R.get_roi(
            img, strel_dilate=select_strel("ellipse", (10, 10)), weights=(1, .1, 1), depth_range=(650, 750),
            gradient_filter=False, fill_holes=True, progress_bar=False, iters=200)
        fx[f"roi_plane_{k}"] = plane2
        fx[f"roi_label_{k}"] = label_im.astype(np.int32)
        fx[f"roi_ranks_{k}"] = ranks
        fx[f"roi_shape_index_{k}"] = shape_index
        fx[f"roi_rois_{k}"] = np.stack([np.asarray(r, bool) for r in rois])
        fx[f"roi_bboxes_{k}"] = np.stack(bboxes)
        fx[f"roi_true_depth_{k}"] = np.array(float(np.median(img[rois[0] > 0])))
    # get_bground_im on small int16 frames (np.median over blurred frames)
    rng = np.random.default_rng(5)
    for k, n in enumerate([7, 8]):
        fr = (700 + rng.normal(0, 20, (n, 24, 32))).round().astype(np.int16)
        fr[rng.random(fr.shape) < 0.05] = 0
        fx[f"bg_frames_{k}"] = fr.copy()
        fx[f"bg_out_{k}"] = R.get_bground_im(fr.copy())
    fx["strel_ellipse_10"] = select_strel("ellipse", (10, 10))
    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, len(fx), "arrays")


if __name__ == "__main__":
    main()
