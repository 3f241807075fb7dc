"""CPU-side checks of the model handle's C ABI (include/mdx.h,
csrc/model.hip): the weights blob format, the config struct layout, and that
mdx_model_create rejects malformed blobs before touching a device."""
import ctypes
import os
import re
import struct

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _parse_blob(b: bytes):
    """The blob format as include/mdx.h documents it."""
    assert b[:4] == b"MDXW"
    ver, n = struct.unpack_from("<II", b, 4)
    assert ver == 1
    off, out = 12, {}
    for _ in range(n):
        (nl,) = struct.unpack_from("<I", b, off)
        off += 4
        name = b[off:off + nl].decode()
        off += nl
        (nd,) = struct.unpack_from("<I", b, off)
        off += 4
        shape = struct.unpack_from(f"<{nd}q", b, off)
        off += 8 * nd
        cnt = int(np.prod(shape)) if nd else 1
        out[name] = np.frombuffer(b, "<f4", cnt, off).reshape(shape)
        off += 4 * cnt
    assert off == len(b)
    return out


def test_pack_blob_roundtrip(mdx):
    from moseq2_detectron_extract_amd.model.weights import pack_blob
    sd = {"a.weight": torch.randn(3, 2, 1, 1), "b": torch.arange(5, dtype=torch.float64), "scalar": torch.tensor(2.5)}
    got = _parse_blob(pack_blob(sd))
    assert list(got) == list(sd)
    for k, v in sd.items():
        np.testing.assert_array_equal(got[k], v.float().numpy())


def test_cfg_struct_matches_header(mdx):
    """ctypes mirror of struct mdx_model_cfg: same field names, same order."""
    from moseq2_detectron_extract_amd.model.runtime import ModelCfgC
    src = open(os.path.join(ROOT, "include", "mdx.h")).read()
    body = re.search(r"typedef struct mdx_model_cfg \{(.*?)\} mdx_model_cfg;", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\b(\w+)\s*(?:\[\d+\])?\s*;", body)
    assert names == [f[0] for f in ModelCfgC._fields_]


def test_cfg_from_model_config(mdx):
    from moseq2_detectron_extract_amd.model import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import model_cfg_c
    c = model_cfg_c(ModelConfig(depth=101, score_thresh_test=0.25), "fp16")
    assert c.depth == 101 and c.dtype == 1 and abs(c.score_thresh - 0.25) < 1e-7
    assert c.n_keypoint_convs == 8 and list(c.keypoint_conv_dims[:8]) == [512] * 8
    assert list(c.anchor_sizes) == [32, 64, 128, 256, 512] and c.fpn_fuse_avg == 1
    with pytest.raises(NotImplementedError):
        model_cfg_c(ModelConfig(fpn_norm=""), "fp32")


@pytest.mark.parametrize("blob,msg", [(b"XXXX" + b"\0" * 12, "MDXW"),
                                      (b"MDXW" + struct.pack("<II", 2, 0), "version"),
                                      (b"MDXW" + struct.pack("<III", 1, 1, 50) + b"abc", "truncated")])
def test_create_rejects_bad_blob(mdx, blob, msg):
    from moseq2_detectron_extract_amd import MdxError
    from moseq2_detectron_extract_amd._lib import call
    from moseq2_detectron_extract_amd.model import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import model_cfg_c
    c = model_cfg_c(ModelConfig(), "fp32")
    h = ctypes.c_void_p()
    with pytest.raises(MdxError, match=msg):
        call("mdx_model_create", blob, len(blob), ctypes.byref(c), 0, ctypes.byref(h))
    assert not h.value


def test_create_rejects_bad_cfg(mdx):
    from moseq2_detectron_extract_amd import MdxError
    from moseq2_detectron_extract_amd._lib import call
    from moseq2_detectron_extract_amd.model import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import model_cfg_c
    c = model_cfg_c(ModelConfig(), "fp32")
    c.depth = 34
    blob = b"MDXW" + struct.pack("<II", 1, 0)
    h = ctypes.c_void_p()
    with pytest.raises(MdxError, match="depth"):
        call("mdx_model_create", blob, len(blob), ctypes.byref(c), 0, ctypes.byref(h))
