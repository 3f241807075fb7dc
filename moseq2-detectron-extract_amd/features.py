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
flips_from_keypoints               M/proc/proc.py:851-889
estimate_keypoint_rotation         M/proc/proc.py:892-907
compute_keypoint_alignment_scores  M/proc/proc.py:936-985
move_median                        bottleneck.move_median (min_count semantics)
filter_angles / iterative_...      M/proc/proc.py:600-654
finalize_angles (no tracking)      M/proc/proc.py:720-724, 827-839
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
    """Pixel -> mm (Kinect intrinsics from the field of view), M/proc/util.py:29-60."""
    cx = resolution[0] // 2
    cy = resolution[1] // 2
    xhat = coords[:, 0] - cx
    yhat = coords[:, 1] - cy
    f_w = resolution[0] / (2 * np.deg2rad(field_of_view[0] / 2))
    f_h = resolution[1] / (2 * np.deg2rad(field_of_view[1] / 2))
    new_coords = np.zeros_like(coords)
    new_coords[:, 0] = true_depth * xhat / f_w
    new_coords[:, 1] = true_depth * yhat / f_h
    return new_coords


def clamp_angles_deg(angles: np.ndarray) -> np.ndarray:
    return np.where(angles < 0, 360 + angles, angles) % 360


def clamp_angles_rad(angles: np.ndarray) -> np.ndarray:
    return np.where(angles < 0, (2 * np.pi) + angles, angles) % (2 * np.pi)


def angle_difference(angles1: np.ndarray, angles2: np.ndarray) -> np.ndarray:
    """Signed smaller difference angles2 - angles1 in degrees (M/proc/kalman.py:93-98)."""
    diff = (angles2 - angles1) % 360
    to_min = diff > 180
    diff[to_min] = -(360 - diff[to_min])
    return diff


# ---------------------------------------------------------------------------
# keypoint geometry
# ---------------------------------------------------------------------------
def rotate_points(points: np.ndarray, center=(0, 0), angle: float = 0) -> np.ndarray:
    """Rotate (K, 2|3) points about `center` by -angle degrees; column 2 (if
    present) is carried as a weight (M/proc/keypoints.py:11-39)."""
    if points.shape[1] == 3:
        weights = points[:, 2]
        points = points[:, :2]
    elif points.shape[1] == 2:
        weights = None
    else:
        raise ValueError(f'Expected axis 1 of `points` to have length 2 or 3, but got {points.shape[1]}')
    a = np.deg2rad(-angle)
    R = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
    o = np.atleast_2d(center)
    p = np.atleast_2d(points)
    rotated = np.squeeze((R @ (p.T - o.T) + o.T).T)
    if weights is not None:
        rotated = np.append(rotated, weights[..., None], 1)
    return rotated


def rotate_points_batch(points: np.ndarray, centers: np.ndarray, angles: Union[np.ndarray, float]) -> np.ndarray:
    """Per-frame rotate_points, in place on `points` (M/proc/keypoints.py:42-64).
    Vectorised over frames: x' = c (x - ox) - s (y - oy) + ox,
    y' = s (x - ox) + c (y - oy) + oy with c, s of deg2rad(-angle)."""
    if isinstance(angles, (int, float)):
        angles_array = np.array([angles] * points.shape[0])
    elif isinstance(angles, np.ndarray):
        angles_array = np.array(angles)
    else:
        raise TypeError(f'Expected angles to be of type numpy.ndarray or float, got {type(angles).__name__} instead!')
    if points.shape[-1] not in (2, 3):
        raise ValueError(f'Expected axis 2 of `points` to have length 2 or 3, but got {points.shape[-1]}')
    a = np.deg2rad(-angles_array.astype(np.float64))
    c, s = np.cos(a)[:, None], np.sin(a)[:, None]
    ox, oy = centers[:, 0:1], centers[:, 1:2]
    dx, dy = points[..., 0] - ox, points[..., 1] - oy
    x = c * dx + (-s) * dy + ox
    y = s * dx + c * dy + oy
    points[..., 0] = x
    points[..., 1] = y
    return points


def flips_from_keypoints(keypoints: np.ndarray, centroids: np.ndarray, angles: np.ndarray,
                         length: Union[float, np.ndarray] = 80) -> Tuple[np.ndarray, np.ndarray]:
    """Front (0-3) vs rear (4-6) keypoints vote on which end of the rotated
    body they sit; returns (flips bool, confidence) (M/proc/proc.py:851-889)."""
    front_keypoints = [0, 1, 2, 3]
    rear_keypoints = [4, 5, 6]
    rotated_keypoints = rotate_points_batch(np.copy(keypoints), centroids, angles)
    extent_x_min = centroids[:, 0] - (length / 2)
    extent_x_max = centroids[:, 0] + (length / 2)
    left_dist = np.abs(extent_x_min[:, np.newaxis] - rotated_keypoints[:, :, 0])
    right_dist = np.abs(extent_x_max[:, np.newaxis] - rotated_keypoints[:, :, 0])
    rot_keypoint_scores = np.where(left_dist < right_dist, -1, 1)
    front_votes = np.mean(rot_keypoint_scores[:, front_keypoints], axis=1)
    rear_votes = np.mean(rot_keypoint_scores[:, rear_keypoints], axis=1)
    flips = np.where(front_votes < rear_votes, True, False)
    expected = np.where(flips[:, None], np.array([-1, 1]), np.array([1, -1]))
    agree = np.count_nonzero(rot_keypoint_scores[:, front_keypoints] == expected[:, 0, None], axis=1) \
        + np.count_nonzero(rot_keypoint_scores[:, rear_keypoints] == expected[:, 1, None], axis=1)
    conf_scores = agree / (len(front_keypoints) + len(rear_keypoints))
    return flips, conf_scores


def estimate_keypoint_rotation(keypoints: np.ndarray) -> np.ndarray:
    """Median per-frame rotation of the keypoints between frames (M/proc/proc.py:892-907)."""
    angles = np.arctan2(keypoints[..., 1], keypoints[..., 0])
    angles = clamp_angles_deg(np.rad2deg(angles))
    angles = np.diff(angles, axis=0, prepend=angles[0, None, ...])
    angles = angles % 360
    to_min = angles > 180
    angles[to_min] = -(360 - angles[to_min])
    return np.median(angles, axis=1)


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
    """Share of keypoint pairs whose x-order matches the expectation (M/proc/proc.py:936-957)."""
    if expected_alignment is None:
        expected_alignment = get_expected_keypoint_alignment()
    # pairwise x differences (calc_keypoint_keypoint_distance, metric 'x', :910-933)
    distances = keypoints[..., :, None, 0] - keypoints[..., None, :, 0]
    distance_signs = np.sign(distances)
    masked_distance_signs = np.where(expected_alignment == 0, 0, distance_signs)
    axis = (1, 2) if len(keypoints.shape) == 3 else None
    num_expectations_met = np.count_nonzero(masked_distance_signs == expected_alignment, axis=axis) \
        - np.count_nonzero(expected_alignment == 0)
    return num_expectations_met / np.count_nonzero(expected_alignment)


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
    """Undo ~180 degree jumps against a moving median (M/proc/proc.py:600-624)."""
    out = np.copy(angles)
    window = min(window, out.shape[0])
    windows = move_median(angles, window=window, min_count=1)
    diff = out - windows
    absdiff = np.abs(diff)
    flips = ((absdiff > (180 - tolerance)) & (absdiff < (180 + tolerance)))
    signs = np.sign(diff[flips])
    out[flips] = out[flips] + (-180 * signs)
    return out


def iterative_filter_angles(angles: np.ndarray, window: int = 3, tolerance: float = 60,
                            max_iters: int = 1000) -> Tuple[np.ndarray, np.ndarray]:
    """filter_angles until it stops changing (M/proc/proc.py:627-654).  Runs
    in libmdx (mdx_iterative_filter_angles, host code, bit-identical to
    iterative_filter_angles_numpy) without holding the GIL: the reference
    loops up to 1000 times whenever an angle is NaN."""
    a = np.ascontiguousarray(angles, dtype=np.float64)
    if a.ndim != 1 or window > 8:
        return iterative_filter_angles_numpy(angles, window, tolerance, max_iters)
    out = np.empty_like(a)
    flips = np.empty(a.shape, dtype=np.uint8)
    call("mdx_iterative_filter_angles", a.ctypes.data_as(ctypes.c_void_p), a.shape[0], int(window), float(tolerance),
         int(max_iters), out.ctypes.data_as(ctypes.c_void_p), flips.ctypes.data_as(ctypes.c_void_p))
    return out, flips.astype(bool)


def iterative_filter_angles_numpy(angles: np.ndarray, window: int = 3, tolerance: float = 60,
                                  max_iters: int = 1000) -> Tuple[np.ndarray, np.ndarray]:
    """The same loop in numpy (the reference's formulation)."""
    last = np.copy(angles)
    iterations = 0
    while True:
        if iterations > max_iters:
            break
        iterations += 1
        curr = filter_angles(last, window=window, tolerance=tolerance)
        if np.allclose(curr, last):
            break
        last = curr
    flips = np.isclose(np.abs(curr - angles), 180)
    return curr, flips


def finalize_angles(orientation: np.ndarray, axis_length: np.ndarray, centroid: np.ndarray,
                    keypoints: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """The no-tracking branch of instances_to_features (M/proc/proc.py:720-724,
    827-839): orientation (rad) -> degrees in [0, 360), keypoint flips,
    iterative 180-degree filtering.  keypoints (n, K, 3) of instance 0.
    Returns (angles deg, flips bool)."""
    lengths = np.max(axis_length, axis=1)
    angles = -np.rad2deg(orientation)
    angles = clamp_angles_deg(angles)
    flips, _ = flips_from_keypoints(keypoints, centroid, angles, lengths)
    angles[flips] += 180
    angles, filter_flips = iterative_filter_angles(angles)
    flips = np.logical_xor(flips, filter_flips)
    return angles, flips


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
    """Per-frame scalars (M/proc/scalars.py:36-120).  `frames` is the uint8
    chunk already multiplied by the masks (or pass reductions=(area_px,
    height_ave) from frame_scalars, computed on the device, and frames=None /
    any object with shape[0] == nframes).  Dtypes follow the reference."""
    centroid = np.asarray(track_features['centroid'])
    nframes = centroid.shape[0]
    if reductions is None:
        area, hmean, _ = frame_scalars(frames, None, min_height, max_height)
        reductions = (area.cpu().numpy(), hmean.cpu().numpy())
    area_px, height_mean = (np.asarray(r) for r in reductions)
    features = {
        'centroid_x_px': np.zeros((nframes,), 'float32'),
        'centroid_y_px': np.zeros((nframes,), 'float32'),
        'velocity_2d_px': np.zeros((nframes,), 'float32'),
        'velocity_3d_px': np.zeros((nframes,), 'float32'),
        'width_px': np.zeros((nframes,), 'float32'),
        'length_px': np.zeros((nframes,), 'float32'),
        'area_px': np.zeros((nframes,)),
        'centroid_x_mm': np.zeros((nframes,), 'float32'),
        'centroid_y_mm': np.zeros((nframes,), 'float32'),
        'velocity_2d_mm': np.zeros((nframes,), 'float32'),
        'velocity_3d_mm': np.zeros((nframes,), 'float32'),
        'width_mm': np.zeros((nframes,), 'float32'),
        'length_mm': np.zeros((nframes,), 'float32'),
        'area_mm': np.zeros((nframes,)),
        'height_ave_mm': np.zeros((nframes,), 'float32'),
        'angle': np.zeros((nframes,), 'float32'),
        'velocity_theta': np.zeros((nframes,)),
    }
    centroid_mm = convert_pxs_to_mm(centroid, true_depth=true_depth)
    centroid_mm_shift = convert_pxs_to_mm(centroid + 1, true_depth=true_depth)
    px_to_mm = np.abs(centroid_mm_shift - centroid_mm)
    features['centroid_x_px'] = centroid[:, 0]
    features['centroid_y_px'] = centroid[:, 1]
    features['centroid_x_mm'] = centroid_mm[:, 0]
    features['centroid_y_mm'] = centroid_mm[:, 1]
    features['width_px'] = np.min(track_features['axis_length'], axis=1)
    features['length_px'] = np.max(track_features['axis_length'], axis=1)
    features['area_px'] = area_px.astype(np.int64)
    features['width_mm'] = features['width_px'] * px_to_mm[:, 1]
    features['length_mm'] = features['length_px'] * px_to_mm[:, 0]
    features['area_mm'] = features['area_px'] * px_to_mm.mean(axis=1)
    features['angle'] = np.deg2rad(track_features['orientation'])
    nz = area_px > 0
    features['height_ave_mm'][nz] = height_mean[nz]
    vel_x = np.diff(np.concatenate((features['centroid_x_px'][:1], features['centroid_x_px'])))
    vel_y = np.diff(np.concatenate((features['centroid_y_px'][:1], features['centroid_y_px'])))
    vel_z = np.diff(np.concatenate((features['height_ave_mm'][:1], features['height_ave_mm'])))
    features['velocity_2d_px'] = np.hypot(vel_x, vel_y)
    features['velocity_3d_px'] = np.sqrt(np.square(vel_x) + np.square(vel_y) + np.square(vel_z))
    vel_x = np.diff(np.concatenate((features['centroid_x_mm'][:1], features['centroid_x_mm'])))
    vel_y = np.diff(np.concatenate((features['centroid_y_mm'][:1], features['centroid_y_mm'])))
    features['velocity_2d_mm'] = np.hypot(vel_x, vel_y)
    features['velocity_3d_mm'] = np.sqrt(np.square(vel_x) + np.square(vel_y) + np.square(vel_z))
    features['velocity_theta'] = np.arctan2(vel_y, vel_x)
    return features


def keypoints_to_dict(keypoints: np.ndarray, frames, centers: np.ndarray, angles: np.ndarray,
                      true_depth: float = 673.1, keypoint_names: Optional[List[str]] = None,
                      z_data: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """Keypoints in reference/rotated coordinates, px and mm, plus the z of
    each keypoint read from `frames` (M/proc/keypoints.py:93-165).  Pass
    z_data from frame_scalars (device lookup) to skip the frame gather."""
    if keypoint_names is None:
        keypoint_names = default_keypoint_names
    old_error_settings = np.seterr(invalid='ignore')
    try:
        if z_data is None:  # device lookup (mdx_frame_scalars)
            _, _, z = frame_scalars(frames, None, 0, 0, keypoints=keypoints, z_frames=frames)
            z_data = z.cpu().numpy()
        ref_kpts_px = np.copy(keypoints)
        ref_kpts_mm = np.zeros_like(keypoints)
        ref_kpts_mm[:, :, 2] = keypoints[:, :, 2]
        for kpi in range(keypoints.shape[1]):
            ref_kpts_mm[:, kpi, :2] = convert_pxs_to_mm(keypoints[:, kpi, :2], true_depth=true_depth)
        rot_kpts_px = rotate_points_batch(np.copy(keypoints[:, :, :]), centers=centers, angles=angles)
        rot_kpts_px[:, :, :2] -= np.expand_dims(centers, axis=1)
        centroid_mm = convert_pxs_to_mm(centers, true_depth=true_depth)
        rot_kpts_mm = rotate_points_batch(np.copy(ref_kpts_mm), centers=centroid_mm, angles=angles)
        rot_kpts_mm[:, :, :2] -= np.expand_dims(centroid_mm, axis=1)
        out = {}
        # the reference iterates default_keypoint_names here whatever names it was given
        for kpi, kpn in enumerate(default_keypoint_names):
            out[f'reference/{kpn}_x_px'] = ref_kpts_px[:, kpi, 0]
            out[f'reference/{kpn}_y_px'] = ref_kpts_px[:, kpi, 1]
            out[f'reference/{kpn}_score'] = ref_kpts_px[:, kpi, 2]
            out[f'reference/{kpn}_x_mm'] = ref_kpts_mm[:, kpi, 0]
            out[f'reference/{kpn}_y_mm'] = ref_kpts_mm[:, kpi, 1]
            out[f'reference/{kpn}_z_mm'] = z_data[:, kpi]
            out[f'rotated/{kpn}_x_px'] = rot_kpts_px[:, kpi, 0]
            out[f'rotated/{kpn}_y_px'] = rot_kpts_px[:, kpi, 1]
            out[f'rotated/{kpn}_score'] = rot_kpts_px[:, kpi, 2]
            out[f'rotated/{kpn}_x_mm'] = rot_kpts_mm[:, kpi, 0]
            out[f'rotated/{kpn}_y_mm'] = rot_kpts_mm[:, kpi, 1]
            out[f'rotated/{kpn}_z_mm'] = z_data[:, kpi]
    finally:
        np.seterr(**old_error_settings)
    return out
