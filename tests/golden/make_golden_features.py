"""Golden fixtures for the host feature post-processing,
produced by the REFERENCE's own functions.

Run in the build container only (reads /root/reference):
    /opt/conda/bin/python3.9 tests/golden/make_golden_features.py
That interpreter carries the real bottleneck 1.3.2 (move_median, used by
filter_angles) and h5py; modules absent there (OpenCV, pykalman, Detectron2,
ruamel.yaml, pycocotools) are replaced by inert stubs that are never called.

Pinned reference functions (M/ = moseq2_detectron_extract/):
  convert_pxs_to_mm            M/proc/util.py:29-60
  rotate_points_batch          M/proc/keypoints.py:42-64
  flips_from_keypoints         M/proc/proc.py:851-889
  compute_keypoint_alignment_scores, estimate_keypoint_rotation  :892-985
  filter_angles / iterative_filter_angles (real bottleneck.move_median)  :600-654
  bottleneck.move_median itself (min_count=1 and default, 1-D and axis 0)
  the no-tracking angle branch of instances_to_features  :720-724, 827-839
  compute_scalars              M/proc/scalars.py:36-120
  keypoints_to_dict            M/proc/keypoints.py:93-165
  angle_difference             M/proc/kalman.py:93-98
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_features.npz")


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    mod.__path__ = []
    mod.__getattr__ = lambda attr: type(attr, (), {}) if not attr.startswith("__") else None
    sys.modules[name] = mod
    return mod


def install_stubs():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot  # noqa: F401
    import pandas  # noqa: F401
    import scipy.signal  # noqa: F401

    def _strel(shape, ksize):
        w, h = ksize
        return np.ones((h, w), np.uint8)

    def need(name):
        try:
            importlib.import_module(name)
            return False
        except Exception:
            return True

    _stub("cv2", MORPH_ELLIPSE=2, MORPH_RECT=0, MORPH_OPEN=2, getStructuringElement=_strel, INPAINT_NS=0,
          INPAINT_TELEA=1)
    for name, attrs in [("ruamel", {}), ("ruamel.yaml", {}), ("pykalman", {"KalmanFilter": object}),
                        ("detectron2", {}), ("detectron2.data", {"MetadataCatalog": object, "DatasetCatalog": object}),
                        ("detectron2.structures", {"Instances": object, "Boxes": object}), ("pycocotools", {}),
                        ("skimage", {}), ("skimage.measure", {}), ("skimage.draw", {}), ("tifffile", {}),
                        ("imageio", {"imwrite": lambda *a, **k: None}),
                        ("tqdm.contrib.logging", {"_TqdmLoggingHandler": object})]:
        if need(name):
            _stub(name, **attrs)
    sys.path.insert(0, REF)


def main():
    install_stubs()
    import bottleneck
    from moseq2_detectron_extract.proc import proc as P
    from moseq2_detectron_extract.proc import keypoints as KP
    from moseq2_detectron_extract.proc import scalars as SC
    from moseq2_detectron_extract.proc import util as U
    from moseq2_detectron_extract.proc import kalman as KA
    assert not isinstance(bottleneck.move_median, type), "real bottleneck required"

    rng = np.random.default_rng(2024)
    fx = {}

    # ---- units
    c = rng.uniform(-50, 560, size=(64, 2))
    fx["px2mm_in"] = c
    fx["px2mm_out"] = U.convert_pxs_to_mm(c)
    fx["px2mm_out_td"] = U.convert_pxs_to_mm(c, true_depth=655.5)

    # ---- a synthetic keypoint track: body along the heading, some frames flipped / NaN
    n, K = 240, 8
    cen = np.cumsum(rng.normal(0, 2.0, size=(n, 2)), 0) + [256, 212]
    head = np.cumsum(rng.normal(0, 6.0, size=n)) % 360          # degrees
    along = np.array([30, 22, 22, 14, -8, -8, -26, -50], float)  # nose .. tail tip
    across = np.array([0, 6, -6, 0, 7, -7, 0, 0], float)
    th = np.deg2rad(head)[:, None]
    kx = cen[:, :1] + along * np.cos(th) - across * np.sin(th) + rng.normal(0, 2, (n, K))
    ky = cen[:, 1:] + along * np.sin(th) + across * np.cos(th) + rng.normal(0, 2, (n, K))
    kp = np.stack([kx, ky, rng.uniform(0, 1, (n, K))], -1)
    kp[rng.random(n) < 0.03] = np.nan                           # frames without an instance
    orient = -np.deg2rad(head + np.where(rng.random(n) < 0.25, 180, 0))  # moments angle, flipped sometimes
    axl = np.column_stack([rng.uniform(60, 90, n), rng.uniform(20, 35, n)])
    fx["kp"] = kp
    fx["cen"] = cen
    fx["orient"] = orient
    fx["axl"] = axl

    ang = P.clamp_angles_deg(-np.rad2deg(orient))
    lengths = np.max(axl, axis=1)
    fx["rot_batch"] = KP.rotate_points_batch(np.copy(kp), cen, ang)
    flips, conf = P.flips_from_keypoints(kp, cen, ang, lengths)
    fx["flips"] = flips
    fx["flip_conf"] = conf
    rot7 = KP.rotate_points_batch(np.copy(kp[:, :7, :2]), cen, ang)
    fx["align_scores"] = P.compute_keypoint_alignment_scores(rot7)
    fx["kp_rotation"] = P.estimate_keypoint_rotation(rot7)

    # the no-tracking angle branch (M/proc/proc.py:720-724, 827-839) composed from the reference's functions
    angles = P.clamp_angles_deg(-np.rad2deg(orient))
    fl, _ = P.flips_from_keypoints(kp[:, :, :], cen, angles, lengths)
    angles[fl] += 180
    angles, filter_flips = P.iterative_filter_angles(angles)
    fx["final_angles"] = angles
    fx["final_flips"] = np.logical_xor(fl, filter_flips)

    # ---- filter_angles / move_median on their own
    a = (np.cumsum(rng.normal(0, 5, 300)) % 360) + np.where(rng.random(300) < 0.2, 180, 0)
    fx["filt_in"] = a
    fx["filt_out"] = P.filter_angles(a)
    ia, iflip = P.iterative_filter_angles(a)
    fx["ifilt_out"] = ia
    fx["ifilt_flips"] = iflip
    mm = rng.normal(0, 1, (40, 3))
    mm[rng.random(mm.shape) < 0.15] = np.nan
    fx["mm_in"] = mm
    for w in (1, 2, 3, 4, 7):
        fx[f"mm_w{w}_mc1"] = bottleneck.move_median(mm, window=w, min_count=1, axis=0)
        fx[f"mm_w{w}_mcdef"] = bottleneck.move_median(mm, window=w, axis=0)
        fx[f"mm_w{w}_1d"] = bottleneck.move_median(mm[:, 0], window=w, min_count=1)

    # ---- angle_difference (kalman.py)
    a1 = rng.uniform(-400, 400, 50)
    a2 = rng.uniform(-400, 400, 50)
    fx["adiff_a1"], fx["adiff_a2"] = a1, a2
    fx["adiff_out"] = KA.angle_difference(a1, a2)

    # ---- compute_scalars on a masked uint8 chunk
    nf, H, W = 12, 40, 56
    fr = rng.integers(0, 140, size=(nf, H, W), dtype=np.uint8)
    mk = (rng.random((nf, H, W)) < 0.6).astype(np.uint8)
    mk[3] = 0                                                    # empty mask -> height 0
    masked = fr * mk
    tf = {"centroid": rng.uniform(0, 500, (nf, 2)), "axis_length": rng.uniform(5, 90, (nf, 2)),
          "orientation": rng.uniform(0, 360, nf)}
    tf["centroid"][5] = np.nan
    fx["sc_frames"], fx["sc_masks"] = fr, mk
    for k, v in tf.items():
        fx[f"sc_tf_{k}"] = v
    for mh, xh, td in [(10, 100, 673.1), (0, 100, 650.0)]:
        out = SC.compute_scalars(masked, tf, min_height=mh, max_height=xh, true_depth=td)
        for k, v in out.items():
            fx[f"sc_{mh}_{xh}_{k}"] = np.asarray(v)

    # ---- keypoints_to_dict (z from a uint8 frame, NaN / out-of-range keypoints)
    kk = np.copy(kp[:nf])
    kk[0, 0, :2] = [-5.5, 1000.0]
    kk[1, 2, :2] = [np.inf, -np.inf]
    kk[2, 1, :] = np.nan
    yy, xx = np.mgrid[0:424, 0:512]
    fr2 = np.stack([((xx * 3 + yy * 7 + 11 * i) % 251) for i in range(nf)]).astype(np.uint8)  # distinct, compressible
    fx["kd_kp"], fx["kd_frames"], fx["kd_cen"], fx["kd_ang"] = kk, fr2, cen[:nf], ang[:nf]
    kd = KP.keypoints_to_dict(kk, fr2, cen[:nf], ang[:nf], true_depth=660.0)
    fx["kd_keys"] = np.array(list(kd.keys()))
    for i, (k, v) in enumerate(kd.items()):
        fx[f"kd_{i}"] = np.asarray(v)

    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, len(fx), "arrays")


if __name__ == "__main__":
    main()
