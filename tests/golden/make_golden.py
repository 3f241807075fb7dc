"""Generate golden fixtures by importing the REFERENCE's own numpy code.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):  python tests/golden/make_golden.py

The reference's frame-op module (M/proc/proc.py) imports OpenCV, bottleneck,
h5py, pykalman ... which are absent here.  Those modules are replaced by inert
stubs; only functions whose arithmetic is pure numpy are executed, so the
fixtures contain the reference's own results:

* scale_raw_frames          M/proc/proc.py:214-234
* prep_raw_frames(fix_invalid_pixels=False)   M/proc/proc.py:129-172
  (background subtract, apply_roi/get_bbox M/proc/roi.py:215-254, clamp, cast)
* find_invalid_pixels       M/proc/proc.py:175-186
* getStructuringElement(MORPH_ELLIPSE,(9,9)) as restated by the oracle is NOT
  pinned here (OpenCV formula); it is checked against the literal rows quoted
  in SURVEY.md A17.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_frameops.npz")


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    mod.__path__ = []  # allow submodules
    # any other attribute is an inert placeholder class (PEP 562)
    mod.__getattr__ = lambda attr: type(attr, (), {}) if not attr.startswith("__") else None
    sys.modules[name] = mod
    return mod


def install_stubs():
    # real modules first so the stubs below never shadow them
    import matplotlib.pyplot  # noqa: F401
    import pandas  # noqa: F401
    import scipy.signal  # noqa: F401

    def _strel(shape, ksize):
        w, h = ksize
        return np.ones((h, w), np.uint8)

    _stub("cv2", MORPH_ELLIPSE=2, MORPH_RECT=0, MORPH_OPEN=2, getStructuringElement=_strel,
          INPAINT_NS=0, INPAINT_TELEA=1)
    _stub("bottleneck", move_median=lambda *a, **k: (_ for _ in ()).throw(RuntimeError("stub")))
    _stub("h5py", File=object, Group=object, Dataset=object)
    _stub("ruamel")
    _stub("ruamel.yaml")
    _stub("pykalman", KalmanFilter=object)
    _stub("skimage")
    _stub("skimage.measure")
    _stub("skimage.draw")
    _stub("tifffile")
    _stub("imageio", imwrite=lambda *a, **k: None)
    _stub("detectron2")
    _stub("detectron2.data", MetadataCatalog=object, DatasetCatalog=object)
    _stub("detectron2.structures", Instances=object, Boxes=object)
    _stub("pycocotools")
    tq = _stub("tqdm.contrib.logging", _TqdmLoggingHandler=object)
    del tq
    sys.path.insert(0, REF)


def main():
    install_stubs()
    from moseq2_detectron_extract.proc import proc as P  # reference module
    from moseq2_detectron_extract.proc import roi as R

    rng = np.random.default_rng(1234)
    fx = {}

    # ---- scale_raw_frames: full uint8 domain for three (vmin, vmax) pairs
    x = np.arange(256, dtype=np.uint8).reshape(1, 16, 16, 1)
    # integer vmin/vmax as the CLI passes them, plus float ones (k=3,4)
    for k, (vmin, vmax) in enumerate([(0, 100), (0, 255), (10, 80), (10.0, 80.0), (0.5, 99.5)]):
        fx[f"scale_in_{k}"] = x
        fx[f"scale_vmin_{k}"] = np.array(vmin)
        fx[f"scale_vmax_{k}"] = np.array(vmax)
        fx[f"scale_out_{k}"] = P.scale_raw_frames(x, vmin, vmax)

    # ---- prep_raw_frames (numpy part) on small synthetic depth frames
    for k, (n, H, W) in enumerate([(3, 40, 56), (2, 33, 47)]):
        yy, xx = np.mgrid[0:H, 0:W]
        bg = np.round((670 + 0.02 * xx - 0.01 * yy) * 2) / 2  # .5-granular like a median bg
        raw = (bg[None] - rng.uniform(-10, 130, size=(n, H, W))).round().astype(np.int16)
        raw[rng.random((n, H, W)) < 0.05] = 0  # invalid (Kinect zero) pixels
        roi = ((yy - H / 2) ** 2 / (0.45 * H) ** 2 + (xx - W / 2) ** 2 / (0.45 * W) ** 2) <= 1
        for vm in [(0, 100), (None, None), (-5, 80)]:
            out = P.prep_raw_frames(raw.copy(), bground_im=bg, roi=roi, vmin=vm[0], vmax=vm[1],
                                    fix_invalid_pixels=False)
            tag = f"{k}_{'none' if vm[0] is None else f'{vm[0]}_{vm[1]}'}"
            fx[f"prep_raw_{tag}"] = raw
            fx[f"prep_bg_{tag}"] = bg
            fx[f"prep_roi_{tag}"] = roi
            fx[f"prep_vmin_{tag}"] = np.float64(np.nan if vm[0] is None else vm[0])
            fx[f"prep_vmax_{tag}"] = np.float64(np.nan if vm[1] is None else vm[1])
            fx[f"prep_out_{tag}"] = out
        inv = P.find_invalid_pixels(raw)
        fx[f"invalid_raw_{k}"] = raw
        fx[f"invalid_out_{k}"] = inv
        fx[f"invalid_roi_out_{k}"] = R.apply_roi(inv, roi)
        fx[f"bbox_{k}"] = R.get_bbox(roi)

    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, len(fx), "arrays")


if __name__ == "__main__":
    main()
