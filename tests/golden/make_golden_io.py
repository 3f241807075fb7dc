"""Golden fixtures for the frame source, produced by the
REFERENCE's own readers:

  read_frames_raw  M/io/video.py:67-127 (plain file and tar member)
  gen_batch_sequence  M/io/util.py:24-35 (with Session's frame-trim offsets)

Run in the build container only (reads /root/reference):
    python tests/golden/make_golden_io.py
Absent modules (OpenCV, h5py, ...) are inert stubs (tests/golden/make_golden.py).
Small frames (16 x 12) keep the fixture tiny; the reader takes frame_dims.
"""
from __future__ import annotations

import io
import os
import sys
import tarfile
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ref_io.npz")
sys.path.insert(0, HERE)


def main():
    from make_golden import install_stubs
    install_stubs()
    from moseq2_detectron_extract.io import util as U
    from moseq2_detectron_extract.io import video as V

    rng = np.random.default_rng(77)
    W, H, n = 16, 12, 40
    data = rng.integers(-2000, 2000, size=(n, H, W)).astype("<i2")
    fx = {"raw": data}
    sels = {"all": None, "empty": [], "int": 5, "runs": [3, 4, 5, 9, 10, 2, 30, 31], "tail": [38, 39, 0]}
    with tempfile.TemporaryDirectory() as td:
        dat = os.path.join(td, "depth.dat")
        data.tofile(dat)
        tgz = os.path.join(td, "session.tar.gz")
        with tarfile.open(tgz, "w:gz") as tf:
            tf.add(dat, arcname="session/depth.dat")
        with tarfile.open(tgz, "r:gz") as tf:
            member = tf.getmember("session/depth.dat")
            for k, sel in sels.items():
                fx[f"sel_{k}"] = np.array(-1 if sel is None else sel)
                fx[f"read_{k}"] = V.read_frames_raw(dat, sel, frame_dims=(W, H))
                fx[f"readtar_{k}"] = V.read_frames_raw(member, sel, frame_dims=(W, H), tar_object=tf)
    # chunking as SessionFramesIterator.generate_samples calls it, for several trims
    for k, (nf, trim, chunk, ovl) in enumerate([(40, (0, 0), 7, 0), (40, (3, 2), 7, 0), (1000, (0, 0), 100, 0),
                                                 (1000, (10, 5), 300, 0), (40, (0, 0), 8, 2)]):
        first = trim[0] if 0 < trim[0] < nf else 0
        last = nf - trim[1] if nf - trim[1] > first else nf
        seq = list(U.gen_batch_sequence(last - first, chunk, ovl, first))
        fx[f"chunks_{k}_args"] = np.array([nf, trim[0], trim[1], chunk, ovl])
        fx[f"chunks_{k}_lens"] = np.array([len(s) for s in seq])
        fx[f"chunks_{k}_flat"] = np.concatenate([np.asarray(list(s)) for s in seq]) if seq else np.zeros(0, int)
    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, len(fx), "arrays")


if __name__ == "__main__":
    main()
