"""Golden fixtures for the result writers, produced by the
REFERENCE's own code under /opt/conda/bin/python3.9 with the real h5py 3.3.0:

  write_extracted_chunk_to_h5   M/io/result.py:106-130  (into datasets laid
                                out as create_extract_h5 makes them, :14-63)
  ResultWriterStep.__process_csv M/pipeline/write_results_step.py:54-73
                                (the keypoints TSV, final file bytes)

Two chunks are written (offset 0: with chunk overlap the reference's writer
raises, see main()).  torch / cv2 / ... are inert stubs (only the classes'
import needs them).

Run in the build container only (reads /root/reference):
    /opt/conda/bin/python3.9 tests/golden/make_golden_results.py
"""
from __future__ import annotations

import multiprocessing
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ref_results.npz")


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    mod.__path__ = []
    mod.__getattr__ = lambda attr: type(attr, (), {}) if not attr.startswith("__") else None
    sys.modules[name] = mod
    return mod


def install():
    import matplotlib.pyplot  # noqa: F401
    import pandas  # noqa: F401
    import scipy.signal  # noqa: F401
    _stub("torch")
    _stub("torch.multiprocessing", Event=multiprocessing.Event, Process=multiprocessing.Process,
          Queue=multiprocessing.Queue)
    _stub("cv2", MORPH_ELLIPSE=2, MORPH_RECT=0, MORPH_OPEN=2, getStructuringElement=lambda s, k: np.ones(k[::-1]))
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
    sys.path.insert(0, REF)
    # import pipeline submodules without the package __init__ (which pulls in
    # the Detectron2 model)
    import moseq2_detectron_extract  # noqa: F401
    pkg = _stub("moseq2_detectron_extract.pipeline")
    pkg.__path__ = [os.path.join(REF, "moseq2_detectron_extract", "pipeline")]


def chunk(rng, frame_idxs, offset, skeys, kkeys):
    n = len(frame_idxs)
    return {
        "chunk": np.zeros((n, 4, 4), np.uint8),
        "frame_idxs": np.asarray(frame_idxs),
        "offset": offset,
        "scalars": {k: rng.normal(100, 30, n) for k in skeys},
        "keypoints": {k: rng.normal(50, 20, n) for k in kkeys},
        "depth_frames": rng.integers(0, 255, (n, 80, 80)).astype(np.uint8),
        "mask_frames": (rng.random((n, 80, 80)) < 0.3).astype(np.uint8),
        "features": {"flips": rng.random(n) < 0.5,
                     "features": {"centroid": rng.normal(200, 40, (n, 2)),
                                  "orientation": rng.uniform(0, 360, n)}},
    }


def main():
    install()
    import h5py
    from moseq2_detectron_extract.io.result import write_extracted_chunk_to_h5
    from moseq2_detectron_extract.pipeline.write_results_step import ResultWriterStep
    from moseq2_detectron_extract.proc.keypoints import keypoint_attributes
    from moseq2_detectron_extract.proc.scalars import scalar_attributes
    rng = np.random.default_rng(9)
    skeys, kkeys = list(scalar_attributes()), list(keypoint_attributes())
    nframes = 12
    # offset must be 0: with chunk_overlap > 0 the reference's own writer
    # raises (frame_idxs keeps the whole chunk while the data is sliced)
    chunks = [chunk(rng, range(0, 7), 0, skeys, kkeys), chunk(rng, range(7, 12), 0, skeys, kkeys)]
    fx = {"nframes": np.array(nframes)}
    for i, c in enumerate(chunks):
        fx[f"c{i}_frame_idxs"] = c["frame_idxs"]
        fx[f"c{i}_offset"] = np.array(c["offset"])
        fx[f"c{i}_depth_frames"] = c["depth_frames"]
        fx[f"c{i}_mask_frames"] = c["mask_frames"]
        fx[f"c{i}_flips"] = c["features"]["flips"]
        fx[f"c{i}_centroid"] = c["features"]["features"]["centroid"]
        fx[f"c{i}_orientation"] = c["features"]["features"]["orientation"]
        for k in skeys:
            fx[f"c{i}_scalars/{k}"] = c["scalars"][k]
        for k in kkeys:
            fx[f"c{i}_keypoints/{k}"] = c["keypoints"][k]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "r.h5")
        with h5py.File(path, "w") as h:
            # the datasets write_extracted_chunk_to_h5 fills, shaped/typed as
            # create_extract_h5 makes them (M/io/result.py:35-70)
            for k in skeys:
                h.create_dataset(f"scalars/{k}", (nframes,), "float32")
            for k in kkeys:
                h.create_dataset(f"keypoints/{k}", (nframes,), "float32")
            h.create_dataset("frames", (nframes, 80, 80), "uint8")
            h.create_dataset("frames_mask", (nframes, 80, 80), "bool")
            h.create_dataset("metadata/extraction/flips", (nframes,), "bool")
            for c in chunks:
                write_extracted_chunk_to_h5(h, c)
            def grab(name, obj):
                if isinstance(obj, h5py.Dataset):
                    fx[f"h5/{name}"] = obj[()]
            h.visititems(grab)
        step = object.__new__(ResultWriterStep)
        step.config = {"output_dir": td, "bg_roi_index": 0}
        step._ResultWriterStep__init_csv()
        for c in chunks:
            step._ResultWriterStep__process_csv(c)
        with open(os.path.join(td, "keypoints_00.tsv"), "rb") as fh:
            fx["tsv"] = np.frombuffer(fh.read(), np.uint8)
    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, len(fx), "arrays")


if __name__ == "__main__":
    main()
