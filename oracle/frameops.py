"""ctypes front-end of the C frame-op oracle (TEST INFRASTRUCTURE ONLY).

Mirrors the reference's Python signatures so parity tests read like the
reference: ``prep_raw_frames`` (M/proc/proc.py:129-172), ``scale_raw_frames``
(:214-234), ``clean_frames`` (:480-515), ``get_frame_features`` (:237-302),
``crop_and_rotate_frame`` (:305-340).  See frameops.c for the restated
OpenCV semantics.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "liboracle_frameops.so")
        src = os.path.join(_HERE, "frameops.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(so)
        P = ctypes.c_void_p
        i64, i32, f64 = ctypes.c_int64, ctypes.c_int, ctypes.c_double
        lib.orc_prep.argtypes = [P, i64, i32, i32, P, P, i32, i32, i32, i32, i32, f64, i32, f64, P, P]
        lib.orc_scale_lut.argtypes = [f64, f64, i32, P]
        lib.orc_median3.argtypes = [P, i64, i32, i32, P]
        lib.orc_morph.argtypes = [P, i64, i32, i32, i32, P, i32, i32, i32, P]
        lib.orc_frame_features.argtypes = [P, P, i64, i32, i32, f64, P, P, P, P]
        lib.orc_crop_rotate.argtypes = [P, i64, i32, i32, P, P, i32, i32, P]
        lib.orc_inpaint_ns.argtypes = [P, P, i64, i32, i32, i32, P]
        _LIB = lib
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def ellipse_strel(ksize=(9, 9)) -> np.ndarray:
    """cv2.getStructuringElement(cv2.MORPH_ELLIPSE, ksize), OpenCV formula."""
    w, h = ksize
    r, c = h // 2, w // 2
    inv_r2 = 1.0 / (r * r) if r else 0.0
    k = np.zeros((h, w), np.uint8)
    for i in range(h):
        dy = i - r
        if abs(dy) <= r:
            dx = int(np.rint(c * np.sqrt((r * r - dy * dy) * inv_r2)))
            j1, j2 = max(c - dx, 0), min(c + dx + 1, w)
            k[i, j1:j2] = 1
    return k


def get_bbox(roi: np.ndarray):
    """M/proc/roi.py:239-254 get_bbox -> ((ymin, xmin), (ymax, xmax)) or None."""
    y, x = np.where(roi > 0)
    if len(y) == 0:
        return None
    return np.array([[y.min(), x.min()], [y.max(), x.max()]])


def prep_raw_frames(frames, bground_im=None, roi=None, vmin=None, vmax=None,
                    fix_invalid_pixels=True):
    """Restatement of prep_raw_frames (uint8 output)."""
    frames = np.ascontiguousarray(frames, dtype=np.int16)
    n, H, W = frames.shape
    bg = None if bground_im is None else np.ascontiguousarray(bground_im, np.float64)
    r = None if roi is None else np.ascontiguousarray(roi > 0, np.uint8)
    bbox = None if r is None else get_bbox(r)
    if bbox is None:
        y0, y1, x0, x1 = 0, H, 0, W
    else:
        y0, x0, y1, x1 = int(bbox[0, 0]), int(bbox[0, 1]), int(bbox[1, 0]), int(bbox[1, 1])
    out = np.empty((n, y1 - y0, x1 - x0), np.uint8)
    inv = np.empty_like(out)
    _lib().orc_prep(_p(frames), n, H, W, None if bg is None else _p(bg), None if r is None else _p(r),
                    y0, y1, x0, x1, int(vmin is not None), float(vmin or 0), int(vmax is not None),
                    float(vmax or 0), _p(out), _p(inv))
    if fix_invalid_pixels:
        out = inpaint_ns(out, inv)
    return out, inv


def inpaint_ns(frames, invalid, radius=3):
    frames = np.ascontiguousarray(frames, np.uint8)
    invalid = np.ascontiguousarray(invalid, np.uint8)
    out = np.empty_like(frames)
    n, H, W = frames.shape
    _lib().orc_inpaint_ns(_p(frames), _p(invalid), n, H, W, radius, _p(out))
    return out


def scale_lut(vmin, vmax) -> np.ndarray:
    lut = np.empty(256, np.uint8)
    int_vmin = isinstance(vmin, (int, np.integer)) and not isinstance(vmin, bool)
    _lib().orc_scale_lut(float(vmin), float(vmax), int(int_vmin), _p(lut))
    return lut


def scale_raw_frames(frames, vmin, vmax):
    return scale_lut(vmin, vmax)[np.asarray(frames, np.uint8)]


def median3(frames):
    frames = np.ascontiguousarray(frames, np.uint8)
    out = np.empty_like(frames)
    n, H, W = frames.shape
    _lib().orc_median3(_p(frames), n, H, W, _p(out))
    return out


def morph(frames, op: str, strel: np.ndarray, iters: int):
    frames = np.ascontiguousarray(frames, np.uint8)
    strel = np.ascontiguousarray(strel, np.uint8)
    out = np.empty_like(frames)
    n, H, W = frames.shape
    code = {"erode": 0, "dilate": 1, "open": 2, "close": 3}[op]
    _lib().orc_morph(_p(frames), n, H, W, code, _p(strel), strel.shape[0], strel.shape[1], iters, _p(out))
    return out


def clean_frames(frames, prefilter_space=(3,), iters_tail=None, strel_tail=None):
    """clean_frames(frames, prefilter_space=(3,), iters_tail=it) for uint8."""
    out = np.ascontiguousarray(frames, np.uint8).copy()
    if prefilter_space is not None and all(p > 0 for p in prefilter_space):
        for pfs in prefilter_space:
            assert pfs == 3, "oracle restates medianBlur(3) only"
            out = median3(out)
    if iters_tail is not None and iters_tail > 0:
        out = morph(out, "open", ellipse_strel() if strel_tail is None else strel_tail, iters_tail)
    return out


def get_frame_features(frames, frame_threshold=10, mask=None):
    frames = np.ascontiguousarray(frames, np.uint8)
    n, H, W = frames.shape
    m = None if mask is None or np.asarray(mask).size == 0 else np.ascontiguousarray(mask, np.uint8)
    cen = np.empty((n, 2)); ori = np.empty(n); ax = np.empty((n, 2)); area = np.empty(n)
    _lib().orc_frame_features(_p(frames), None if m is None else _p(m), n, H, W, float(frame_threshold),
                              _p(cen), _p(ori), _p(ax), _p(area))
    return {"centroid": cen, "orientation": ori, "axis_length": ax, "area": area}


def crop_and_rotate_frames(frames, centers, angles, crop_size=(80, 80)):
    frames = np.ascontiguousarray(frames, np.uint8)
    n, H, W = frames.shape
    c = np.ascontiguousarray(centers, np.float64).reshape(n, 2)
    a = np.ascontiguousarray(angles, np.float64).reshape(n)
    out = np.empty((n, crop_size[1], crop_size[0]), np.uint8)
    _lib().orc_crop_rotate(_p(frames), n, H, W, _p(c), _p(a), crop_size[0], crop_size[1], _p(out))
    return out


def bground_ref(frames, med_scale=5):
    """get_bground_im (M/proc/roi.py:293-307): per-frame medianBlur(med_scale)
    (BORDER_REPLICATE == scipy 'nearest'), then np.median over frames."""
    from scipy.ndimage import median_filter
    f = np.asarray(frames).copy()
    for i in range(f.shape[0]):
        f[i] = median_filter(f[i], size=med_scale, mode="nearest")
    return np.median(f, axis=0)
