"""Golden fixtures for the mask-IoU NMS of the feature step, produced by the
REFERENCE's own method ProcessFeaturesStep.__nms_mask_instances
(M/pipeline/process_features_step.py:63-113).

Run in the build container only (it reads /root/reference, absent on the GPU
box):  python tests/golden/make_golden_nms.py

The step module imports Detectron2 (Instances), norfair, the instance logger
and the model utilities, all absent here; they are replaced by inert stubs
except ``detectron2.structures.Instances``, for which a minimal field
container with Detectron2's indexing semantics (``len``, boolean / index-list
``__getitem__`` applied to every field) is supplied.  The method itself runs
unmodified on torch tensors (pred_masks bool (n, h, w), scores float32 (n,)).
An extra ``orig`` field records which input instance each returned one is.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import _stub, install_stubs  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_mask_nms.npz")


class Instances:
    """Minimal detectron2.structures.Instances: named per-instance fields."""

    def __init__(self, image_size, **fields):
        object.__setattr__(self, "_image_size", image_size)
        object.__setattr__(self, "_fields", dict(fields))

    def __getattr__(self, name):
        f = object.__getattribute__(self, "_fields")
        if name in f:
            return f[name]
        raise AttributeError(name)

    def __len__(self):
        for v in self._fields.values():
            return len(v)
        return 0

    def __getitem__(self, item):
        return Instances(self._image_size, **{k: v[item] for k, v in self._fields.items()})


def main():
    install_stubs()
    import torch
    _stub("detectron2.structures", Instances=Instances, Boxes=object)
    _stub("norfair", Detection=object, Tracker=object)
    import moseq2_detectron_extract  # noqa: F401  (the real top-level package)
    # the model package's __init__ builds Detectron2 models: never executed
    mp = _stub("moseq2_detectron_extract.model")
    mp.__path__ = [os.path.join("/root/reference", "moseq2_detectron_extract", "model")]
    _stub("moseq2_detectron_extract.model.instance_logger", InstanceLogger=object)
    _stub("moseq2_detectron_extract.model.util", create_empty_instances=lambda *a, **k: None)
    # likewise the pipeline package's __init__ (it imports every step)
    pp = _stub("moseq2_detectron_extract.pipeline")
    pp.__path__ = [os.path.join("/root/reference", "moseq2_detectron_extract", "pipeline")]
    import importlib
    S = importlib.import_module("moseq2_detectron_extract.pipeline.process_features_step")
    nms = S.ProcessFeaturesStep._ProcessFeaturesStep__nms_mask_instances

    rng = np.random.default_rng(2024)
    fx = {}
    cases = 0
    for h, w in ((37, 53), (64, 80)):
        for trial in range(60):
            n = int(rng.integers(0, 6))
            masks = np.zeros((n, h, w), bool)
            for d in range(n):
                y0, x0 = rng.integers(0, h - 4), rng.integers(0, w - 4)
                masks[d, y0:y0 + rng.integers(3, h // 2), x0:x0 + rng.integers(3, w // 2)] = True
            if n >= 2 and trial % 5 == 0:
                masks[1] = masks[0]                     # duplicate -> suppressed
            if n >= 3 and trial % 7 == 0:
                masks[2] = False                        # empty mask dropped
            if n >= 2 and trial % 4 == 0:
                masks[:, 5:h - 5, 5:w - 5] |= True     # heavy overlap
            if n >= 4 and trial % 6 == 0:
                masks[3] = masks[0] & (np.arange(w) < w // 2)  # partial overlap
            scores = rng.random(n).astype(np.float32)
            if n >= 3 and trial % 3 == 0:
                scores[1] = scores[2]                   # a tie
            ins = Instances((h, w), pred_masks=torch.from_numpy(masks), scores=torch.from_numpy(scores),
                            orig=torch.arange(n))
            out = nms(None, ins, 0.5)
            fx[f"masks_{cases}"] = masks
            fx[f"scores_{cases}"] = scores
            fx[f"picks_{cases}"] = np.asarray(out.orig.numpy() if len(out) else np.zeros(0, np.int64), np.int64)
            cases += 1
    fx["ncases"] = np.array(cases)
    np.savez_compressed(OUT, **fx)
    print("wrote", OUT, cases, "cases")


if __name__ == "__main__":
    main()
