"""moseq2_detectron_extract_amd -- MI355X-native extraction hot path.

Drop-in for the hot path of tischfieldlab/moseq2-detectron-extract: the
proc/ per-frame ops and the Mask/Keypoint R-CNN forward, as hand-written
gfx950 HIP kernels behind a C ABI (include/mdx.h), with the reference's
Python-level signatures on top (``proc``, ``model``, ``pipeline``).

Hardware queues.  The extract loop keeps up to eight model forwards in
flight beside its frame stages (pipeline.OverlappedExtractor), each on its
own HIP stream; HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware
queues (default 4).  Importing this package before the HIP runtime starts
sets the variable to 12 when the caller has not set it; a caller may set its
own value before HIP initialises.  ``HW_QUEUES`` is the count this process
runs with, and pipeline.ExtractConfig derives its default number of model
streams from it (default_model_streams).
"""
import os as _os

__version__ = "0.1.0"


def _setup_hw_queues() -> int:
    q = _os.environ.get("GPU_MAX_HW_QUEUES")
    if q is not None:
        return int(q)
    try:
        import torch
        started = torch.cuda.is_initialized()
    except Exception:  # torch absent: nothing has started HIP through it
        started = False
    if started:  # too late to change it: HIP's default
        return 4
    _os.environ["GPU_MAX_HW_QUEUES"] = "12"
    return 12


HW_QUEUES = _setup_hw_queues()

from ._lib import MdxError, lib  # noqa: E402,F401
