"""Golden results FILE made by the REFERENCE's own writer, under
/opt/conda/bin/python3.9 with the real h5py 3.3.0:

  create_extract_h5             M/io/result.py:14-103  (the whole tree:
                                metadata, parameters, acquisition metadata)
  write_extracted_chunk_to_h5   M/io/result.py:106-130 (the two chunks of
                                ref_results.npz)

The file is flattened by tests/_h5tree.py (every dataset's value, dtype,
shape, compression filter and attributes) into ref_results_tree.npz,
together with the inputs (config_data, status_dict), so that
tests/test_results_h5.py can run this package's writer on the same inputs
under the same interpreter and compare the trees.  Two reference call sites
are stubbed: importlib.metadata.version (the package is not installed; the
version string is the only value the test does not compare) and
cli.extract / click_param_annot (the click option help texts that become the
parameters' 'description' attributes: the CLI is out of scope, both sides
write the parameters without them).

Run in the build container only (reads /root/reference):
    /opt/conda/bin/python3.9 tests/golden/make_golden_results_tree.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import _h5tree  # noqa: E402
import make_golden_results as MG  # noqa: E402

OUT = os.path.join(HERE, "ref_results_tree.npz")


def inputs():
    """config_data / status_dict of the golden file (shared with the test
    through the fixture)."""
    n = 12
    rng = np.random.default_rng(21)
    arrays = {"in/timestamps": np.arange(n) * 33.333 + 1000.0,
              "in/roi": rng.random((6, 7)) > 0.3,
              "in/first_frame": rng.integers(0, 900, (6, 7)).astype(np.int16),
              "in/bground_im": np.round(rng.normal(670, 3, (6, 7)) * 2) / 2}
    cfg = {"nframes": n, "crop_size": [80, 80], "frame_dtype": "uint8", "use_tracking_model": False,
           "flip_classifier": "keypoints", "true_depth": 673.5}
    status = {"uuid": "0f2c9d4e-golden", "complete": False, "skip": False,
              "parameters": {"chunk_size": 1000, "chunk_overlap": 0, "bg_roi_depth_range": [650, 750],
                             "crop_size": [80, 80], "min_height": 0.0, "max_height": 100.0, "fps": 30,
                             "use_tracking": True, "model": None, "camera_type": "kinect",
                             "nested": {"a": 1.5, "b": "x"}},
              "metadata": {"SubjectName": "m1", "SessionName": "s1", "Tags": ["a", "bc"],
                           "DepthResolution": [512, 424], "StartTime": "2021-01-01", "NoValue": None}}
    return cfg, status, arrays


def config_data(cfg, arrays):
    d = dict(cfg)
    d["crop_size"] = tuple(d["crop_size"])
    for k in ("timestamps", "roi", "first_frame", "bground_im"):
        d[k] = arrays["in/" + k]
    return d


def status_dict(status):
    s = json.loads(json.dumps(status))
    s["parameters"]["bg_roi_depth_range"] = tuple(s["parameters"]["bg_roi_depth_range"])
    s["parameters"]["crop_size"] = tuple(s["parameters"]["crop_size"])
    return s


def chunks():
    g = dict(np.load(os.path.join(HERE, "ref_results.npz")))
    out = []
    for i in range(2):
        p = f"c{i}_"
        out.append({
            "frame_idxs": g[p + "frame_idxs"], "offset": int(g[p + "offset"]),
            "depth_frames": g[p + "depth_frames"], "mask_frames": g[p + "mask_frames"],
            "scalars": {k[len(p + "scalars/"):]: g[k] for k in g if k.startswith(p + "scalars/")},
            "keypoints": {k[len(p + "keypoints/"):]: g[k] for k in g if k.startswith(p + "keypoints/")},
            "features": {"flips": g[p + "flips"],
                         "features": {"centroid": g[p + "centroid"], "orientation": g[p + "orientation"]}},
        })
    return out


def main():
    MG.install()
    MG._stub("moseq2_detectron_extract.cli", extract=None)
    import h5py
    import moseq2_detectron_extract.io.result as R
    R.version = lambda name: "0.0.0-golden"
    R.click_param_annot = lambda cmd: {}
    cfg, status, arrays = inputs()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "results_00.h5")
        with h5py.File(path, "w") as h:
            R.create_extract_h5(h, config_data(cfg, arrays), status_dict(status))
            for c in chunks():
                R.write_extracted_chunk_to_h5(h, c)
        tree, meta = _h5tree.dump(path)
    meta["__inputs__"] = {"config": cfg, "status": status}
    _h5tree.save(OUT, {**tree, **arrays}, meta)
    print("wrote", OUT, len(tree), "datasets")


if __name__ == "__main__":
    main()
