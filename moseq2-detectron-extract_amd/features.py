"""Host-side feature post-processing of the extraction path.

What ProcessFeaturesStep does after the frame ops, with the same names,
argument meaning and return dtypes as the reference (M/ =
moseq2_detectron_extract/):

=================================  ==========================================
this module                        reference
=================================  ==========================================
convert_pxs_to_mm                  M/proc/util.py:29-60
clamp_angles_deg / _rad            M/proc/proc.py:688-697
angle_difference                   M/proc/kalman.py:93-98
rotate_points / _batch             M/proc/keypoints.py:11-64
flips_from_keypoints               M/proc/proc.py:851-889 (libmdx host code)
estimate_keypoint_rotation         M/proc/proc.py:892-907
compute_keypoint_alignment_scores  M/proc/proc.py:936-985
move_median                        bottleneck.move_median (min_count semantics)
filter_angles / iterative_...      M/proc/proc.py:600-654
finalize_angles (no tracking)      M/proc/proc.py:720-724, 827-839 (libmdx host code)
compute_scalars                    M/proc/scalars.py:36-120
keypoints_to_dict                  M/proc/keypoints.py:93-165
scalar_attributes / keypoint_...   M/proc/scalars.py:6-33, keypoints.py:67-90
=================================  ==========================================

The per-frame reductions over whole frames (area and mean height of the
masked animal, keypoint z lookup) run on the GPU (``frame_scalars`` ->
``mdx_frame_scalars``); everything here is O(frames x keypoints) sequential
host arithmetic, as in the reference.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from ._lib import MdxError, call

# M/io/annot.py:51-60 (order matters: indices are used by the flip logic)
default_keypoint_names = ['Nose', 'Left Ear', 'Right Ear', 'Neck', 'Left Hip', 'Right Hip', 'TailBase', 'TailTip']


# ---------------------------------------------------------------------------
# units / angles
# ---------------------------------------------------------------------------
def convert_pxs_to_mm(coords: np.ndarray, resolution=(512, 424), field_of_view=(70.6, 60),
                      true_depth: float = 673.1) -> np.ndarray:
    """Pixel -> mm on the floor plane at `true_depth`: a pinhole camera whose
    focal lengths follow from the Kinect field of view (M/proc/util.py:29-60).
    Element-wise: mm = true_depth * (px - centre) / focal."""
    centre = (resolution[0] // 2, resolution[1] // 2)
    focal = [resolution[a] / (2 * np.deg2rad(field_of_view[a] / 2)) for a in (0, 1)]
    out = np.zeros_like(coords)
    for a in (0, 1):
        out[:, a] = true_depth * (coords[:, a] - centre[a]) / focal[a]
    return out


def clamp_angles_deg(angles: np.ndarray) -> np.ndarray:
    return np.where(angles < 0, 360 + angles, angles) % 360


def clamp_angles_rad(angles: np.ndarray) -> np.ndarray:
    return np.where(angles < 0, (2 * np.pi) + angles, angles) % (2 * np.pi)


def _wrap180(d: np.ndarray) -> np.ndarray:
    """Degrees in [0, 360) -> (-180, 180]."""
    return np.where(d > 180, d - 360, d)


def angle_difference(angles1: np.ndarray, angles2: np.ndarray) -> np.ndarray:
    """Signed smaller difference angles2 - angles1 in degrees (M/proc/kalman.py:93-98)."""
    return _wrap180((angles2 - angles1) % 360)


# ---------------------------------------------------------------------------
# keypoint geometry
# ---------------------------------------------------------------------------
def rotate_points_batch(points: np.ndarray, centers: np.ndarray, angles: Union[np.ndarray, float]) -> np.ndarray:
    """Rotate every frame's points by -angle degrees about its centre, in
    place on columns 0-1 of `points` (M/proc/keypoints.py:42-64):
    x' = c (x - ox) - s (y - oy) + ox, y' = s (x - ox) + c (y - oy) + oy,
    (c, s) = (cos, sin) of deg2rad(-angle)."""
    if isinstance(angles, (int, float)):
        angles = np.full(points.shape[0], float(angles))
    elif not isinstance(angles, np.ndarray):
        raise TypeError(f'Expected angles to be of type numpy.ndarray or float, got {type(angles).__name__} instead!')
    if points.shape[-1] not in (2, 3):
        raise ValueError(f'Expected axis 2 of `points` to have length 2 or 3, but got {points.shape[-1]}')
    theta = np.deg2rad(-np.asarray(angles, np.float64))
    c, s = np.cos(theta)[:, None], np.sin(theta)[:, None]
    ox, oy = centers[:, 0:1], centers[:, 1:2]
    dx, dy = points[..., 0] - ox, points[..., 1] - oy
    points[..., 0], points[..., 1] = c * dx + (-s) * dy + ox, s * dx + c * dy + oy
    return points


def rotate_points(points: np.ndarray, center=(0, 0), angle: float = 0) -> np.ndarray:
    """One frame of rotate_points_batch on (K, 2|3) points (column 2 carried
    through) (M/proc/keypoints.py:11-39)."""
    if points.shape[1] not in (2, 3):
        raise ValueError(f'Expected axis 1 of `points` to have length 2 or 3, but got {points.shape[1]}')
    out = rotate_points_batch(np.array(points, np.float64)[None], np.asarray(center, np.float64).reshape(1, 2),
                              np.array([float(angle)]))[0]
    return np.squeeze(out)


def flips_from_keypoints(keypoints: np.ndarray, centroids: np.ndarray, angles: np.ndarray,
                         length: Union[float, np.ndarray] = 80) -> Tuple[np.ndarray, np.ndarray]:
    """Head/tail vote of the keypoints along the body axis (M/proc/proc.py:
    851-889): (flips bool (n,), confidence (n,)).  Runs in libmdx
    (mdx_flips_from_keypoints, host code)."""
    kp = np.ascontiguousarray(keypoints, np.float64)
    n, K = kp.shape[0], kp.shape[1]
    cen = np.ascontiguousarray(centroids, np.float64)
    ang = np.ascontiguousarray(np.broadcast_to(np.asarray(angles, np.float64), (n,)))
    ln = np.ascontiguousarray(np.broadcast_to(np.asarray(length, np.float64), (n,)))
    flips = np.empty(n, np.uint8)
    conf = np.empty(n, np.float64)
    call("mdx_flips_from_keypoints", _np(kp), n, K, _np(cen), _np(ang), _np(ln), _np(flips), _np(conf))
    return flips.astype(bool), conf


def estimate_keypoint_rotation(keypoints: np.ndarray) -> np.ndarray:
    """Per-frame median of the keypoints' polar-angle change since the
    previous frame, wrapped to (-180, 180] (M/proc/proc.py:892-907)."""
    theta = clamp_angles_deg(np.rad2deg(np.arctan2(keypoints[..., 1], keypoints[..., 0])))
    step = np.diff(theta, axis=0, prepend=theta[:1])
    return np.median(_wrap180(step % 360), axis=1)


def get_expected_keypoint_alignment() -> np.ndarray:
    """Expected east/west sign of keypoint i relative to keypoint j (M/proc/proc.py:960-985)."""
    return np.array([
        [0, 1, 1, 1, 1, 1, 1],
        [-1, 0, 0, 1, 1, 1, 1],
        [-1, 0, 0, 1, 1, 1, 1],
        [-1, -1, -1, 0, 1, 1, 1],
        [-1, -1, -1, -1, 0, 0, 1],
        [-1, -1, -1, -1, 0, 0, 1],
        [-1, -1, -1, -1, -1, -1, 0],
    ])


def compute_keypoint_alignment_scores(keypoints: np.ndarray, expected_alignment: Optional[np.ndarray] = None):
    """Fraction of the constrained keypoint pairs (non-zero entries of the
    expectation) whose x order -- sign of x_i - x_j -- matches it
    (M/proc/proc.py:910-957)."""
    exp = get_expected_keypoint_alignment() if expected_alignment is None else expected_alignment
    sign = np.sign(keypoints[..., :, None, 0] - keypoints[..., None, :, 0])
    met = (sign == exp) & (exp != 0)
    count = met.sum(axis=(-2, -1)) if keypoints.ndim == 3 else met.sum()
    return count / np.count_nonzero(exp)


# ---------------------------------------------------------------------------
# angle filtering
# ---------------------------------------------------------------------------
def _nan_median_small(v: np.ndarray, min_count: int) -> float:
    v = v[~np.isnan(v)]
    if len(v) < max(min_count, 1):
        return np.nan
    v = np.sort(v)
    c = len(v)
    return v[(c - 1) // 2] if c % 2 else (v[c // 2 - 1] + v[c // 2]) / 2


def _move_median3(x: np.ndarray, min_count: int) -> np.ndarray:
    """Window-3 moving median (the angle filter's case): median of three by
    min/max for full windows (exact); the two leading partial windows and the
    windows holding a NaN (min/max propagate it) are recomputed one by one."""
    n = x.shape[0]
    out = np.empty(n)
    if n >= 3:
        p, q, r = x[:-2], x[1:-1], x[2:]
        out[2:] = np.maximum(np.minimum(p, q), np.minimum(np.maximum(p, q), r))
        if min_count > 3:
            out[2:] = np.nan
    for i in range(min(n, 2)):
        out[i] = _nan_median_small(x[:i + 1], min_count)
    if n >= 3:
        for i in (np.flatnonzero(np.isnan(out[2:])) + 2).tolist():
            out[i] = _nan_median_small(x[i - 2:i + 1], min_count)
    return out


def move_median(a: np.ndarray, window: int, min_count: Optional[int] = None, axis: int = -1) -> np.ndarray:
    """bottleneck.move_median: median of the trailing `window` values (the
    first window-1 outputs use the values available), NaNs ignored, NaN where
    fewer than `min_count` (default `window`) non-NaN values are present.
    Output float64 (float32 for float32 input), like bottleneck."""
    a = np.asarray(a)
    if min_count is None:
        min_count = window
    if not 1 <= window:
        raise ValueError("window must be >= 1")
    out_dtype = np.float32 if a.dtype == np.float32 else np.float64
    x = np.moveaxis(a.astype(np.float64), axis, -1)
    n = x.shape[-1]
    if window == 3 and x.ndim == 1:
        return _move_median3(x, min_count).astype(out_dtype)
    pad = np.full(x.shape[:-1] + (window - 1,), np.nan)
    xp = np.concatenate([pad, x], axis=-1)
    win = np.lib.stride_tricks.sliding_window_view(xp, window, axis=-1)[..., :n, :]
    cnt = np.sum(~np.isnan(win), axis=-1)
    # exact median of the non-NaN values of each window: sort (NaNs go last)
    # and pick the middle one, or the mean of the middle two for even counts
    srt = np.sort(win, axis=-1)
    c = np.maximum(cnt, 1)
    lo = np.take_along_axis(srt, ((c - 1) // 2)[..., None], axis=-1)[..., 0]
    hi = np.take_along_axis(srt, (c // 2)[..., None], axis=-1)[..., 0]
    med = np.where(c % 2 == 1, lo, (lo + hi) / 2)
    med = np.where((cnt >= min_count) & (cnt > 0), med, np.nan)
    return np.moveaxis(med, -1, axis).astype(out_dtype)


def filter_angles(angles: np.ndarray, window: int = 3, tolerance: float = 60) -> np.ndarray:
    """One pass of the 180-degree jump filter (M/proc/proc.py:600-624): an
    angle within `tolerance` of 180 degrees away from its trailing moving
    median is moved back by 180 towards it."""
    out = np.array(angles, copy=True)
    dev = out - move_median(angles, window=min(window, out.shape[0]), min_count=1)
    jump = (np.abs(dev) > 180 - tolerance) & (np.abs(dev) < 180 + tolerance)
    out[jump] -= 180 * np.sign(dev[jump])
    return out


def iterative_filter_angles(angles: np.ndarray, window: int = 3, tolerance: float = 60,
                            max_iters: int = 1000) -> Tuple[np.ndarray, np.ndarray]:
    """filter_angles repeated until it stops changing (M/proc/proc.py:627-654);
    returns (angles, flips).  1-D angles with window <= 8 (the extract path:
    window 3) run in libmdx (mdx_iterative_filter_angles, host code) without
    holding the GIL: the reference loops up to 1000 times whenever an angle is
    NaN.  Other shapes / windows take the numpy statement of the same loop."""
    a = np.ascontiguousarray(angles, dtype=np.float64)
    if a.ndim != 1 or not 1 <= window <= 8:
        last, it = a, 0
        while it <= max_iters:
            it += 1
            curr = filter_angles(last, window=window, tolerance=tolerance)
            if np.allclose(curr, last):
                break
            last = curr
        return curr, np.isclose(np.abs(curr - a), 180)
    out = np.empty_like(a)
    flips = np.empty(a.shape, dtype=np.uint8)
    call("mdx_iterative_filter_angles", _np(a), a.shape[0], int(window), float(tolerance), int(max_iters), _np(out),
         _np(flips))
    return out, flips.astype(bool)


def finalize_angles(orientation: np.ndarray, axis_length: np.ndarray, centroid: np.ndarray,
                    keypoints: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """The no-tracking branch of instances_to_features (M/proc/proc.py:720-724,
    827-839) in one libmdx host call (mdx_finalize_angles): orientation (rad)
    -> degrees in [0, 360), keypoint flips (+180), iterative 180-degree
    filtering.  keypoints (n, K, 3) of instance 0.  Returns (angles deg,
    flips bool)."""
    o = np.ascontiguousarray(orientation, np.float64)
    n = o.shape[0]
    ax = np.ascontiguousarray(axis_length, np.float64)
    cen = np.ascontiguousarray(centroid, np.float64)
    kp = np.ascontiguousarray(keypoints, np.float64)
    ang = np.empty(n, np.float64)
    flips = np.empty(n, np.uint8)
    call("mdx_finalize_angles", _np(o), _np(ax), _np(cen), _np(kp), n, kp.shape[1] if kp.ndim == 3 else 8,
         _np(ang), _np(flips))
    return ang, flips.astype(bool)


def _np(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------------------
# scalars and keypoint tables
# ---------------------------------------------------------------------------
def scalar_attributes() -> Dict[str, str]:
    """Scalar names -> descriptions, as written to the h5 (M/proc/scalars.py:6-33)."""
    return {
        'centroid_x_px': 'X centroid (pixels)',
        'centroid_y_px': 'Y centroid (pixels)',
        'velocity_2d_px': '2D velocity (pixels / frame), note that missing frames are not accounted for',
        'velocity_3d_px': '3D velocity (pixels / frame), note that missing frames are not accounted for, also '
                          'height is in mm, not pixels for calculation',
        'width_px': 'Mouse width (pixels)',
        'length_px': 'Mouse length (pixels)',
        'area_px': 'Mouse area (pixels)',
        'centroid_x_mm': 'X centroid (mm)',
        'centroid_y_mm': 'Y centroid (mm)',
        'velocity_2d_mm': '2D velocity (mm / frame), note that missing frames are not accounted for',
        'velocity_3d_mm': '3D velocity (mm / frame), note that missing frames are not accounted for',
        'width_mm': 'Mouse width (mm)',
        'length_mm': 'Mouse length (mm)',
        'area_mm': 'Mouse area (mm)',
        'height_ave_mm': 'Mouse average height (mm)',
        'angle': 'Angle (radians, unwrapped)',
        'velocity_theta': 'Angular component of velocity (arctan(vel_x, vel_y))'
    }


def keypoint_attributes(keypoint_names: Optional[List[str]] = None) -> Dict[str, str]:
    """Keypoint table names -> descriptions (M/proc/keypoints.py:67-90)."""
    if keypoint_names is None:
        keypoint_names = default_keypoint_names
    attributes = {}
    for kpn in keypoint_names:
        for cs in ['reference', 'rotated']:
            attributes[f'{cs}/{kpn}_x_px'] = f'X position of {kpn} (pixels) in {cs} coordinate system.'
            attributes[f'{cs}/{kpn}_y_px'] = f'Y position of {kpn} (pixels) in {cs} coordinate system.'
            attributes[f'{cs}/{kpn}_x_mm'] = f'X position of {kpn} (mm) in {cs} coordinate system.'
            attributes[f'{cs}/{kpn}_y_mm'] = f'Y position of {kpn} (mm) in {cs} coordinate system.'
            attributes[f'{cs}/{kpn}_z_mm'] = f'Z position of {kpn} (mm) in {cs} coordinate system.'
            attributes[f'{cs}/{kpn}_score'] = f'Inference score of {kpn}.'
    return attributes


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def frame_scalars(frames, masks=None, min_height: float = 10, max_height: float = 100, keypoints=None,
                  z_frames=None):
    """GPU reductions behind compute_scalars / keypoints_to_dict for frames
    already in HBM: returns (area_px int64 (n,), height_ave float64 (n,),
    z_data float64 (n, K) or None) as device tensors."""
    import torch
    if not torch.cuda.is_available():
        raise MdxError("frame_scalars needs an AMD GPU; there is no CPU fallback")
    from .proc import _to_dev
    f = _to_dev(frames, torch.uint8)
    n, H, W = f.shape
    m = None if masks is None else _to_dev(masks, torch.uint8)
    if m is not None and tuple(m.shape) != (n, H, W):
        raise ValueError("masks must match frames")
    area = torch.empty((n,), dtype=torch.int64, device=f.device)
    hmean = torch.empty((n,), dtype=torch.float64, device=f.device)
    K = 0
    kp = zf = z = None
    if keypoints is not None:
        kp = _to_dev(keypoints, torch.float64)
        K = kp.shape[1]
        zf = _to_dev(z_frames if z_frames is not None else frames, torch.uint8)
        z = torch.empty((n, K), dtype=torch.float64, device=f.device)
    call("mdx_frame_scalars", _ptr(f), _ptr(m), n, H, W, float(min_height), float(max_height), _ptr(kp), K,
         _ptr(zf), _ptr(area), _ptr(hmean), _ptr(z), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    return area, hmean, z


def compute_scalars(frames, track_features: dict, min_height: float = 10, max_height: float = 100,
                    true_depth: float = 673.1, reductions=None) -> Dict[str, np.ndarray]:
    """Per-frame scalars of the h5 schema (M/proc/scalars.py:36-120).
    The frame reductions (pixels with min_height < v < max_height in
    frames * masks, and their mean height) come from the device
    (reductions=(area_px, height_ave) of frame_scalars; `frames` may then be
    None); everything else is derived from the tracked centroid / axes /
    orientation.  Dtypes are the reference's: float64 except height_ave_mm
    (float32) and area_px (int64)."""
    cen = np.asarray(track_features['centroid'])
    axes = np.asarray(track_features['axis_length'])
    if reductions is None:
        area, hmean, _ = frame_scalars(frames, None, min_height, max_height)
        reductions = (area.cpu().numpy(), hmean.cpu().numpy())
    area_px, hmean = (np.asarray(r) for r in reductions)
    cen_mm = convert_pxs_to_mm(cen, true_depth=true_depth)
    mm_per_px = np.abs(convert_pxs_to_mm(cen + 1, true_depth=true_depth) - cen_mm)  # at the centroid
    width, length = np.min(axes, axis=1), np.max(axes, axis=1)
    area = area_px.astype(np.int64)
    height = np.where(area > 0, hmean, 0).astype(np.float32)

    def step(x):  # frame-to-frame change, 0 at the first frame
        return np.diff(x, prepend=x[:1])

    dz2 = np.square(step(height))  # float32, as the reference squares it
    vx, vy = step(cen[:, 0]), step(cen[:, 1])
    vx_mm, vy_mm = step(cen_mm[:, 0]), step(cen_mm[:, 1])
    vals = {
        'centroid_x_px': cen[:, 0], 'centroid_y_px': cen[:, 1],
        'velocity_2d_px': np.hypot(vx, vy), 'velocity_3d_px': np.sqrt(np.square(vx) + np.square(vy) + dz2),
        'width_px': width, 'length_px': length, 'area_px': area,
        'centroid_x_mm': cen_mm[:, 0], 'centroid_y_mm': cen_mm[:, 1],
        'velocity_2d_mm': np.hypot(vx_mm, vy_mm),
        'velocity_3d_mm': np.sqrt(np.square(vx_mm) + np.square(vy_mm) + dz2),
        'width_mm': width * mm_per_px[:, 1], 'length_mm': length * mm_per_px[:, 0],
        'area_mm': area * mm_per_px.mean(axis=1), 'height_ave_mm': height,
        'angle': np.deg2rad(track_features['orientation']), 'velocity_theta': np.arctan2(vy_mm, vx_mm),
    }
    return {k: vals[k] for k in scalar_attributes()}


def keypoints_to_dict(keypoints: np.ndarray, frames, centers: np.ndarray, angles: np.ndarray,
                      true_depth: float = 673.1, keypoint_names: Optional[List[str]] = None,
                      z_data: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """The keypoint tables of the h5 schema (M/proc/keypoints.py:93-165):
    every keypoint in the camera ('reference') frame and in the animal's
    ('rotated': about the centroid by -angle, centroid at the origin) frame,
    in px and mm, with its score and the depth under it (z, read from
    `frames` on the device, or given as z_data)."""
    n, K = keypoints.shape[0], keypoints.shape[1]
    with np.errstate(invalid="ignore"):
        if z_data is None:  # device lookup (mdx_frame_scalars)
            _, _, z = frame_scalars(frames, None, 0, 0, keypoints=keypoints, z_frames=frames)
            z_data = z.cpu().numpy()
        ref_px = np.copy(keypoints)
        ref_mm = np.zeros_like(keypoints)
        ref_mm[..., 2] = keypoints[..., 2]
        ref_mm[..., :2] = convert_pxs_to_mm(keypoints[..., :2].reshape(n * K, 2),
                                            true_depth=true_depth).reshape(n, K, 2)
        cen_mm = convert_pxs_to_mm(centers, true_depth=true_depth)
        rot_px = rotate_points_batch(np.copy(keypoints), centers=centers, angles=angles)
        rot_px[..., :2] -= centers[:, None, :]
        rot_mm = rotate_points_batch(np.copy(ref_mm), centers=cen_mm, angles=angles)
        rot_mm[..., :2] -= cen_mm[:, None, :]
    frames_by_system = (("reference", ref_px, ref_mm), ("rotated", rot_px, rot_mm))
    out = {}
    # the reference names the columns by default_keypoint_names whatever names it is given
    for k, name in enumerate(default_keypoint_names):
        for system, px, mm in frames_by_system:
            out.update({f'{system}/{name}_x_px': px[:, k, 0], f'{system}/{name}_y_px': px[:, k, 1],
                        f'{system}/{name}_score': px[:, k, 2], f'{system}/{name}_x_mm': mm[:, k, 0],
                        f'{system}/{name}_y_mm': mm[:, k, 1], f'{system}/{name}_z_mm': z_data[:, k]})
    return out
