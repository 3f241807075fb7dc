"""moseq2_detectron_extract_amd -- MI355X-native extraction hot path.

Drop-in for the hot path of tischfieldlab/moseq2-detectron-extract: the
proc/ per-frame ops and the Mask/Keypoint R-CNN forward, as hand-written
gfx950 HIP kernels behind a C ABI (include/mdx.h), with the reference's
Python-level signatures on top (``proc``, ``model``, ``pipeline``).
"""
__version__ = "0.1.0"

from ._lib import MdxError, lib  # noqa: F401
