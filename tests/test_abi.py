"""CPU-side checks of the C ABI: the library builds/loads and exports every
entry point include/mdx.h declares (no device work without a GPU)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = []
    for fn in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names += re.findall(r"\b(mdx_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = _declared()
    assert "mdx_prep_frames" in names and "mdx_crop_rotate" in names


def test_library_exports_every_declared_symbol(mdx):
    import ctypes
    from moseq2_detectron_extract_amd import _build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        _build.build()
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    # every declared symbol has a Python signature (so ctypes calls are typed)
    assert not [n for n in _declared() if n not in _lib.SIGNATURES]


def test_host_only_entry_points(mdx):
    import numpy as np
    from moseq2_detectron_extract_amd import proc
    from oracle import frameops as O
    for vmin, vmax in [(0, 100), (10, 80), (0.5, 99.5)]:
        np.testing.assert_array_equal(proc.scale_lut(vmin, vmax), O.scale_lut(vmin, vmax))
    assert mdx.lib().mdx_version().decode().startswith("mdx")


def test_no_gpu_means_loud_failure(mdx):
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from moseq2_detectron_extract_amd import MdxError, proc
    with pytest.raises(MdxError):
        proc.clean_frames(np.zeros((1, 8, 8), np.uint8), iters_tail=1)
