"""Run this package's results writer with a REAL h5py (the h5py branch of
results.open_results) and flatten what it wrote -- the helper of
tests/test_results_h5.py, run under /opt/conda/bin/python3.9 (the image's
interpreter with h5py 3.3.0; it has no torch, so an inert module stands in
for it: the writer path never calls torch).

    python3.9 tests/_h5_writer_run.py OUT_DIR

Writes OUT_DIR/{one,shard}/results_00.h5 + keypoints_00.tsv through
extract._ChunkWriter with the inputs and chunks of
tests/golden/ref_results_tree.npz / ref_results.npz:
  one    one process, chunks in session order (ResultWriterStep);
  shard  the rank-0 writer of a 2-rank sharded session, the chunks
         arriving in reverse order, each tagged with its source rank (TSV
         part files joined at close), after a failed earlier run left a
         stale part file behind;
and OUT_DIR/{one,shard}.npz: the files flattened by tests/_h5tree.py.
"""
from __future__ import annotations

import ctypes
import os
import sys
import types

# libmdx.so (the TSV row formatter) needs the system libstdc++; conda's older
# copy would otherwise be bound first by its scipy / h5py extensions
for _p in ("/usr/lib/x86_64-linux-gnu/libstdc++.so.6", "/lib/x86_64-linux-gnu/libstdc++.so.6"):
    if os.path.exists(_p):
        ctypes.CDLL(_p, mode=ctypes.RTLD_GLOBAL)
        break

import numpy as np  # noqa: E402

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
sys.path[:0] = [ROOT, TESTS, os.path.join(TESTS, "golden")]

if "torch" not in sys.modules:
    _t = types.ModuleType("torch")
    _t.__path__ = []
    _t.__getattr__ = lambda a: type(a, (), {}) if not a.startswith("__") else None
    sys.modules["torch"] = _t

import _h5tree  # noqa: E402
import make_golden_results_tree as G  # noqa: E402  (inputs / chunks only; reads no reference code)


class _Src:
    """The frame source fields _ChunkWriter reads (path -> depth_ts.txt)."""

    def __init__(self, d, n):
        self.path = os.path.join(d, "depth.dat")
        self.last_frame_idx = n


def run(out_dir: str) -> None:
    import h5py  # noqa: F401  (the branch under test)
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.extract import _ChunkWriter
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig
    tree, meta = _h5tree.load(os.path.join(TESTS, "golden", "ref_results_tree.npz"))
    z = np.load(os.path.join(TESTS, "golden", "ref_results_tree.npz"))
    cfg, status = meta["__inputs__"]["config"], meta["__inputs__"]["status"]
    arrays = {k: z[k] for k in z.files if k.startswith("in/")}
    chunks = G.chunks()
    for name, order, parts in (("one", [0, 1], 1), ("shard", [1, 0], 2)):
        d = os.path.join(out_dir, name)
        os.makedirs(d, exist_ok=True)
        np.savetxt(os.path.join(d, "depth_ts.txt"), arrays["in/timestamps"], fmt="%.17g")
        if parts > 1:  # a failed earlier run's part file of a rank that owns no chunk this time
            with open(os.path.join(d, "keypoints_00.tsv.part3"), "w") as fh:
                fh.write("stale\n")
        w = _ChunkWriter(d, _Src(d, cfg["nframes"]), arrays["in/bground_im"], arrays["in/roi"], cfg["true_depth"],
                         ExtractConfig(crop_size=tuple(cfg["crop_size"])), arrays["in/first_frame"],
                         G.status_dict(status), parts=parts)
        for i in order:
            w.write(chunks[i], part=i if parts > 1 else 0)
        w.close()
        t, m = _h5tree.dump(os.path.join(d, "results_00.h5"))
        _h5tree.save(os.path.join(out_dir, name + ".npz"), t, m)
    print("ok")


if __name__ == "__main__":
    run(sys.argv[1])
