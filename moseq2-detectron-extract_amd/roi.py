"""Session setup: the background image, the arena ROI and
the true floor depth that the hot path's frame prep consumes.

=========================  =================================================
this module                reference (M/ = moseq2_detectron_extract/)
=========================  =================================================
get_bground_im             M/proc/roi.py:293-307   (device: mdx_bground_median)
plane_fit3                 M/proc/roi.py:97-123
plane_ransac               M/proc/roi.py:126-212
get_roi                    M/proc/roi.py:14-94
select_strel               M/proc/util.py:9-26
find_roi                   Session.find_roi M/io/session.py:181-268
                           (no tiff cache: the frames, the plane fit and the
                           ROI are recomputed, as with cache_dir=None)
=========================  =================================================

The background is the one bulk step (a median over every 500th frame of the
session, each median-blurred first): it runs on the GPU.  RANSAC draws its
samples from numpy's global RNG exactly as the reference does
(``np.random.choice(n, 3, replace=True)`` per iteration), so a seeded run
picks the same planes; connected components, region ranking, dilation and hole
filling are host numpy/scipy on one image, as in the reference.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import scipy.ndimage as ndi
import scipy.stats

from ._lib import MdxError, call
from .proc import _ptr, _stream, _torch, ellipse_strel, get_bbox, rect_strel


def select_strel(shape: str = "e", size: Tuple[int, int] = (10, 10)) -> np.ndarray:
    """cv2 structuring element by name: 'e'llipse (default) or 'r'ect."""
    if shape[0].lower() == "r":
        return rect_strel(size)
    return ellipse_strel(size)


def get_bground_im(frames, med_scale: int = 5) -> np.ndarray:
    """Median over frames of the per-frame medianBlur(med_scale) images,
    float64 (H, W).  `frames` int16 (n, H, W), numpy or a device tensor."""
    torch = _torch()
    if not torch.cuda.is_available():
        raise MdxError("get_bground_im needs an AMD GPU; there is no CPU fallback")
    f = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames, dtype=np.int16))
    f = f.to(device="cuda", dtype=torch.int16).contiguous()
    if f.ndim != 3:
        raise ValueError("frames must be (n, H, W)")
    n, H, W = f.shape
    work = torch.empty_like(f)
    out = torch.empty((H, W), dtype=torch.float64, device=f.device)
    call("mdx_bground_median", _ptr(f), n, H, W, int(med_scale), _ptr(work), _ptr(out), _stream())
    return out.cpu().numpy()


def plane_fit3(points: np.ndarray) -> np.ndarray:
    """Plane (a, b, c, d), unit normal, through 3 points (x, y, z); NaN when
    they are collinear."""
    a = points[1, :] - points[0, :]
    b = points[2, :] - points[0, :]
    normal = np.array([[a[1] * b[2] - a[2] * b[1]],
                       [a[2] * b[0] - a[0] * b[2]],
                       [a[0] * b[1] - a[1] * b[0]]])
    denom = np.sum(np.square(normal))
    if denom < np.spacing(1):
        return np.full((4,), np.nan)
    normal /= np.sqrt(denom)
    d = np.dot(-points[0, :], normal)
    return np.hstack((normal.flatten(), d))


def plane_ransac(depth_image: np.ndarray, depth_range=(650, 750), iters: int = 1000, noise_tolerance: float = 30,
                 in_ratio: float = 0.1, progress_bar: bool = False, mask: Optional[np.ndarray] = None):
    """RANSAC plane fit of the in-range pixels.  Returns (best_plane, |distance|
    of every pixel to it).  Consumes np.random's global state like the
    reference."""
    use = np.logical_and(depth_image > depth_range[0], depth_image < depth_range[1])
    if mask is not None:
        use = np.logical_and(use, mask)
    xx, yy = np.meshgrid(np.arange(depth_image.shape[1]), np.arange(depth_image.shape[0]))
    coords = np.vstack((xx[use].ravel(), yy[use].ravel(), depth_image[use].ravel())).T
    npoints = np.sum(use)
    best_dist, best_num, best_plane = np.inf, 0, None
    for _ in range(iters):
        sel = coords[np.random.choice(coords.shape[0], 3, replace=True), :]
        plane = plane_fit3(sel)
        if np.all(np.isnan(plane)):
            continue
        dist = np.abs(np.dot(coords, plane[:3]) + plane[3])
        ninl = np.sum(dist < noise_tolerance)
        if (ninl / npoints) > in_ratio and ninl > best_num:
            md = np.mean(dist)
            if md < best_dist:
                best_dist, best_num, best_plane = md, ninl, plane
    if best_plane is None:
        raise ValueError("plane_ransac: no plane reached the inlier ratio")
    allc = np.vstack((xx.ravel(), yy.ravel(), depth_image.ravel())).T
    return best_plane, np.abs(np.dot(allc, best_plane[:3]) + best_plane[3])


def _sobel_abs(img: np.ndarray, axis: int, ksize: int) -> np.ndarray:
    """|cv2.Sobel(img, CV_64F, dx, dy, ksize)| (BORDER_REFLECT_101): the
    derivative kernel along `axis` (1 = x), the binomial smoother across."""
    smooth = np.array([1.0])
    for _ in range(ksize - 1):
        smooth = np.convolve(smooth, [1.0, 1.0])
    deriv = np.array([-1.0, 0.0, 1.0])
    for _ in range(ksize - 3):
        deriv = np.convolve(deriv, [1.0, 1.0])
    out = ndi.correlate1d(img.astype(np.float64), deriv, axis=axis, mode="mirror")
    out = ndi.correlate1d(out, smooth, axis=1 - axis, mode="mirror")
    return np.abs(out)


def _morph(img: np.ndarray, strel: np.ndarray, op) -> np.ndarray:
    """cv2.dilate / cv2.erode, one iteration, anchor at the kernel centre
    (OpenCV's default border leaves values unchanged)."""
    kh, kw = strel.shape
    ay, ax = kh // 2, kw // 2
    H, W = img.shape
    fill = -np.inf if op is np.maximum else np.inf
    pad = np.full((H + kh, W + kw), fill)
    pad[ay:ay + H, ax:ax + W] = img
    out = None
    for i, j in zip(*np.nonzero(strel)):
        win = pad[i:i + H, j:j + W]
        out = win.copy() if out is None else op(out, win)
    return out.astype(img.dtype)


def get_roi(depth_image: np.ndarray, strel_dilate: Optional[np.ndarray] = rect_strel((15, 15)),
            strel_erode: Optional[np.ndarray] = None, noise_tolerance: float = 30, weights=(1, .1, 1),
            overlap_roi: Optional[np.ndarray] = None, gradient_filter: bool = False, gradient_kernel: int = 7,
            gradient_threshold: float = 3000, fill_holes: bool = True, **kwargs):
    """Candidate arena ROIs ranked by area, extent and distance from the image
    centre.  Returns (rois, plane, bboxes, label_im, ranks, shape_index) like
    the reference."""
    mask = None
    if gradient_filter:
        gx = _sobel_abs(depth_image, 1, gradient_kernel)
        gy = _sobel_abs(depth_image, 0, gradient_kernel)
        mask = np.logical_and(gx < gradient_threshold, gy < gradient_threshold)
    plane, dists = plane_ransac(depth_image, noise_tolerance=noise_tolerance, mask=mask, **kwargs)
    dist_ims = dists.reshape(depth_image.shape)
    if gradient_filter:
        dist_ims[~mask] = np.inf
    bin_im = dist_ims < noise_tolerance
    # skimage.measure.label: 8-connectivity, labels in raster order
    label_im, nlab = ndi.label(bin_im, structure=np.ones((3, 3), int))
    center = np.array(depth_image.shape) / 2
    areas = np.zeros((nlab,))
    extents = np.zeros_like(areas)
    far = np.zeros_like(areas)
    coords_of = []
    for i, sl in enumerate(ndi.find_objects(label_im)):
        rr, cc = np.nonzero(label_im[sl] == i + 1)
        rr = rr + sl[0].start
        cc = cc + sl[1].start
        coords = np.stack([rr, cc], 1)
        coords_of.append(coords)
        areas[i] = len(rr)
        extents[i] = len(rr) / ((sl[0].stop - sl[0].start) * (sl[1].stop - sl[1].start))
        far[i] = np.sqrt(np.sum(np.square(coords - center), 1)).max()
    ranks = np.vstack((scipy.stats.rankdata(-areas, method="max"),
                       scipy.stats.rankdata(-extents, method="max"),
                       scipy.stats.rankdata(far, method="max")))
    w = np.array(weights, "float32")
    # ties keep region order (numpy 1.x argsort of a short array is insertion sort)
    shape_index = np.mean(np.multiply(ranks.astype("float32"), w[:, np.newaxis]), 0).argsort(kind="stable")
    rois, bboxes = [], []
    for shape in shape_index:
        roi = np.zeros_like(depth_image)
        c = coords_of[shape]
        roi[c[:, 0], c[:, 1]] = 1
        if strel_dilate is not None:
            roi = _morph(roi, strel_dilate, np.maximum)
        if strel_erode is not None:
            roi = _morph(roi, strel_erode, np.minimum)
        if fill_holes:
            roi = ndi.binary_fill_holes(roi)
        rois.append(roi)
        bboxes.append(get_bbox(roi))
    if overlap_roi is not None:
        overlaps = np.zeros_like(areas)
        for i, roi in enumerate(rois):
            overlaps[i] = np.sum(np.logical_and(overlap_roi, roi))
        k = int(np.argmax(overlaps))
        del rois[k]
        del bboxes[k]
    return rois, plane, bboxes, label_im, ranks, shape_index


def find_roi(source, bg_roi_dilate=(10, 10), bg_roi_shape: str = "ellipse", bg_roi_index: int = 0,
             bg_roi_weights=(1, .1, 1), bg_roi_depth_range=(650, 750), bg_roi_gradient_filter: bool = False,
             bg_roi_gradient_threshold: float = 3000, bg_roi_gradient_kernel: int = 7,
             bg_roi_fill_holes: bool = True, use_plane_bground: bool = False, bg_step: int = 500):
    """Session.find_roi without the tiff cache: (first_frame, bground_im, roi,
    true_depth) for a RawDepthSource (or anything with .read(idxs) and
    .nframes)."""
    first_frame = source.read([0])
    idx = np.arange(0, source.nframes, bg_step)
    bground_im = get_bground_im(source.read(list(idx)))
    rois, plane, *_ = get_roi(bground_im, strel_dilate=select_strel(bg_roi_shape, tuple(bg_roi_dilate)),
                              weights=bg_roi_weights, depth_range=bg_roi_depth_range,
                              gradient_filter=bg_roi_gradient_filter, gradient_threshold=bg_roi_gradient_threshold,
                              gradient_kernel=bg_roi_gradient_kernel, fill_holes=bg_roi_fill_holes)
    if use_plane_bground:
        xx, yy = np.meshgrid(np.arange(bground_im.shape[1]), np.arange(bground_im.shape[0]))
        coords = np.vstack((xx.ravel(), yy.ravel()))
        bground_im = ((np.dot(coords.T, plane[:2]) + plane[3]) / -plane[2]).reshape(bground_im.shape)
    roi = rois[bg_roi_index]
    true_depth = float(np.median(bground_im[roi > 0]))
    return first_frame, bground_im, roi, true_depth
