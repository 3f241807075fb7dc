"""Flatten an HDF5 results file into (arrays, meta) for comparison: every
dataset's value plus its dtype, shape, compression filter and attributes.
Shared by tests/golden/make_golden_results_tree.py (the reference's writer)
and tests/_h5_writer_run.py (this package's writer); both run under
/opt/conda/bin/python3.9, the image's interpreter with a real h5py.  No
torch, no package imports."""
from __future__ import annotations

import json

import numpy as np


def dump(path: str):
    import h5py
    arrays, meta = {}, {}
    with h5py.File(path, "r") as h:
        def grab(name, obj):
            if not isinstance(obj, h5py.Dataset):
                return
            empty = obj.shape is None
            if not empty:
                v = np.asarray(obj[()])
                if v.dtype.kind == "O":  # variable-length strings: fixed-width bytes (no pickling)
                    v = np.array([x if isinstance(x, bytes) else str(x).encode() for x in v.reshape(-1)],
                                 dtype="S").reshape(v.shape)
                arrays["d/" + name] = v
            meta[name] = {"dtype": str(obj.dtype), "shape": None if empty else list(obj.shape),
                          "compression": obj.compression, "empty": empty,
                          "attrs": {k: _attr(v) for k, v in obj.attrs.items()}}
        h.visititems(grab)
    return arrays, meta


def _attr(v):
    if isinstance(v, bytes):
        return v.decode()
    if isinstance(v, np.generic):
        return v.item()
    return str(v) if not isinstance(v, (str, int, float, bool)) else v


def save(out: str, arrays: dict, meta: dict) -> None:
    np.savez_compressed(out, meta=np.frombuffer(json.dumps(meta, sort_keys=True).encode(), np.uint8), **arrays)


def load(path: str):
    z = np.load(path)
    meta = json.loads(bytes(z["meta"]).decode())
    return {k: z[k] for k in z.files if k.startswith("d/")}, meta
