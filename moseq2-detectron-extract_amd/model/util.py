"""Model-directory helpers of the reference (M/model/util.py:15-42): the
checkpoint a trained model directory names."""
from __future__ import annotations

import glob
import os


def get_last_checkpoint(path: str) -> str:
    """``<path>/<contents of <path>/last_checkpoint>`` (Detectron2's
    checkpointer records the latest file name there)."""
    with open(os.path.join(path, "last_checkpoint"), "r", encoding="utf-8") as fh:
        return os.path.join(path, fh.read().strip())


def get_specific_checkpoint(path: str, iteration, ext: str = "pth") -> str:
    """The checkpoint of `iteration` (``*<iteration>.<ext>``) in `path`."""
    matches = sorted(glob.glob(os.path.join(path, f"*{iteration}.{ext}")))
    if not matches:
        raise FileNotFoundError(f"no checkpoint *{iteration}.{ext} in {path}")
    return matches[0]
