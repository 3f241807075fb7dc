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


def test_s2d_decode_folded_matches_normalised_input(mdx):
    """The folded stem's 8-channel space-to-depth input (per 2x2 phase: scaled
    pixel, inside flag) decodes to the normalised NHWC input of the reference
    preprocess ((v - mean_c) / std_c inside the image, 0 in the padding),
    bit for bit; the 16-channel form decodes by layout only."""
    from moseq2_detectron_extract_amd.model.config import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import s2d_to_nhwc
    cfg = ModelConfig()
    g = torch.Generator().manual_seed(0)
    B, h, w, Hp, Wp = 2, 5, 7, 8, 10
    v = torch.randint(0, 256, (B, h, w), generator=g).float()
    inside = torch.zeros(B, Hp, Wp)
    inside[:, :h, :w] = 1
    vp = torch.zeros(B, Hp, Wp)
    vp[:, :h, :w] = v
    # pad by one on each side, then space-to-depth into (B, Hp/2+1, Wp/2+1, 2, 2, C) phases
    def s2d(x):  # x (B, Hp, Wp, C)
        C = x.shape[-1]
        xp = torch.zeros(B, Hp + 2, Wp + 2, C)
        xp[:, 1:Hp + 1, 1:Wp + 1] = x
        return xp.view(B, Hp // 2 + 1, 2, Wp // 2 + 1, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(
            B, Hp // 2 + 1, Wp // 2 + 1, 4 * C)
    folded = s2d(torch.stack([vp, inside], -1))
    got = s2d_to_nhwc(folded, Hp, Wp, cfg)
    want = torch.zeros(B, Hp, Wp, 4)
    for c in range(cfg.in_channels):
        want[..., c] = torch.where(inside > 0, (vp - torch.full_like(vp, cfg.pixel_mean[c])) /
                                   torch.full_like(vp, cfg.pixel_std[c]), torch.zeros_like(vp))
    assert torch.equal(got, want)
    plain = s2d(want)
    assert torch.equal(s2d_to_nhwc(plain, Hp, Wp), want)
