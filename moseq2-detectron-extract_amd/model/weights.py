"""Model weights in Detectron2 state-dict layout.

* ``synthetic_state_dict(cfg, seed)``: seeded random weights with exactly the
  key names and shapes of the reference model (GeneralizedRCNN built from
  M/model/config.py:21-94).  No trained checkpoint exists offline, so parity
  and benchmarks run on these.
* ``load_state_dict(path)``: a Detectron2 ``model_final.pth`` (``{'model':
  state_dict}``), read with ``torch.load(weights_only=True)`` (no unpickling of
  arbitrary objects).
* ``pack_blob(sd)``: the state dict as the weights blob of the C ABI
  (``mdx_model_create``).
"""
from __future__ import annotations

import math
import struct
from collections import OrderedDict
from typing import Mapping

import numpy as np
import torch

from .config import ModelConfig


def resnet_stage_specs(cfg: ModelConfig):
    """[(name, n_blocks, in_ch, bottleneck_ch, out_ch, first_stride)] for res2..res5."""
    specs = []
    in_ch = cfg.stem_out_channels
    out_ch = cfg.res2_out_channels
    bott = cfg.num_groups * cfg.width_per_group
    for i, n in enumerate(cfg.res_blocks):
        stride = 1 if i == 0 else 2
        specs.append((f"res{i + 2}", n, in_ch, bott, out_ch, stride))
        in_ch = out_ch
        out_ch *= 2
        bott *= 2
    return specs


def synthetic_state_dict(cfg: ModelConfig = ModelConfig(), seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    g = torch.Generator().manual_seed(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()

    def normal(shape, std):
        return torch.randn(*shape, generator=g) * std

    def unif(shape, lo, hi):
        return torch.rand(*shape, generator=g) * (hi - lo) + lo

    def conv(name, cout, cin, k, bias=False, std=None):
        fan_in = cin * k * k
        sd[f"{name}.weight"] = normal((cout, cin, k, k), std if std is not None else math.sqrt(2.0 / fan_in))
        if bias:
            sd[f"{name}.bias"] = normal((cout,), 0.05)

    def frozen_bn(name, c, wlo=0.8, whi=1.2):
        sd[f"{name}.weight"] = unif((c,), wlo, whi)
        sd[f"{name}.bias"] = normal((c,), 0.1)
        sd[f"{name}.running_mean"] = normal((c,), 0.1)
        sd[f"{name}.running_var"] = unif((c,), 0.5, 1.5)

    bu = "backbone.bottom_up"
    conv(f"{bu}.stem.conv1", cfg.stem_out_channels, 3, 7)
    frozen_bn(f"{bu}.stem.conv1.norm", cfg.stem_out_channels)
    for name, nb, cin, bott, cout, _stride in resnet_stage_specs(cfg):
        for b in range(nb):
            p = f"{bu}.{name}.{b}"
            ci = cin if b == 0 else cout
            if b == 0:
                conv(f"{p}.shortcut", cout, ci, 1)
                frozen_bn(f"{p}.shortcut.norm", cout)
            conv(f"{p}.conv1", bott, ci, 1)
            frozen_bn(f"{p}.conv1.norm", bott)
            conv(f"{p}.conv2", bott, bott, 3)
            frozen_bn(f"{p}.conv2.norm", bott)
            conv(f"{p}.conv3", cout, bott, 1)
            frozen_bn(f"{p}.conv3.norm", cout, 0.1, 0.3)  # keep the residual stream bounded
    C = cfg.fpn_out_channels
    use_bias = cfg.fpn_norm == ""
    for lvl, (_, _, _, _, cout, _) in zip(cfg.fpn_levels, resnet_stage_specs(cfg)):
        conv(f"backbone.fpn_lateral{lvl}", C, cout, 1, bias=use_bias)
        conv(f"backbone.fpn_output{lvl}", C, C, 3, bias=use_bias)
        if cfg.fpn_norm == "GN":
            for k in ("lateral", "output"):
                sd[f"backbone.fpn_{k}{lvl}.norm.weight"] = 1.0 + normal((C,), 0.1)
                sd[f"backbone.fpn_{k}{lvl}.norm.bias"] = normal((C,), 0.1)
    A = len(cfg.aspect_ratios)
    conv("proposal_generator.rpn_head.conv", C, C, 3, bias=True)
    conv("proposal_generator.rpn_head.objectness_logits", A, C, 1, bias=True, std=0.08)
    conv("proposal_generator.rpn_head.anchor_deltas", 4 * A, C, 1, bias=True, std=0.01)
    R = cfg.box_pooler_resolution
    fin = C * R * R
    for i in range(cfg.box_num_fc):
        sd[f"roi_heads.box_head.fc{i + 1}.weight"] = normal((cfg.box_fc_dim, fin), math.sqrt(2.0 / fin))
        sd[f"roi_heads.box_head.fc{i + 1}.bias"] = normal((cfg.box_fc_dim,), 0.02)
        fin = cfg.box_fc_dim
    sd["roi_heads.box_predictor.cls_score.weight"] = normal((cfg.num_classes + 1, fin), 0.3)
    sd["roi_heads.box_predictor.cls_score.bias"] = normal((cfg.num_classes + 1,), 0.1)
    sd["roi_heads.box_predictor.bbox_pred.weight"] = normal((4 * cfg.num_classes, fin), 0.01)
    sd["roi_heads.box_predictor.bbox_pred.bias"] = normal((4 * cfg.num_classes,), 0.01)
    if cfg.mask_on:
        cin = C
        for i in range(cfg.mask_num_conv):
            conv(f"roi_heads.mask_head.mask_fcn{i + 1}", cfg.mask_conv_dim, cin, 3, bias=True)
            cin = cfg.mask_conv_dim
        sd["roi_heads.mask_head.deconv.weight"] = normal((cin, cfg.mask_conv_dim, 2, 2), math.sqrt(2.0 / (cin * 4)))
        sd["roi_heads.mask_head.deconv.bias"] = normal((cfg.mask_conv_dim,), 0.05)
        conv("roi_heads.mask_head.predictor", cfg.num_classes, cfg.mask_conv_dim, 1, bias=True, std=0.1)
    if cfg.keypoint_on:
        cin = C
        for i, d in enumerate(cfg.keypoint_conv_dims):
            conv(f"roi_heads.keypoint_head.conv_fcn{i + 1}", d, cin, 3, bias=True)
            cin = d
        sd["roi_heads.keypoint_head.score_lowres.weight"] = normal((cin, cfg.num_keypoints, 4, 4), 0.05)
        sd["roi_heads.keypoint_head.score_lowres.bias"] = normal((cfg.num_keypoints,), 0.05)
    sd["pixel_mean"] = torch.tensor(cfg.pixel_mean, dtype=torch.float32).view(-1, 1, 1)
    sd["pixel_std"] = torch.tensor(cfg.pixel_std, dtype=torch.float32).view(-1, 1, 1)
    return sd


def load_state_dict(path: str) -> "OrderedDict[str, torch.Tensor]":
    """Load a Detectron2 checkpoint safely (weights_only=True)."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    sd = obj.get("model", obj) if isinstance(obj, dict) else obj
    return OrderedDict((k, v if isinstance(v, torch.Tensor) else torch.as_tensor(v)) for k, v in sd.items())


def pack_blob(sd: Mapping[str, torch.Tensor]) -> bytes:
    """Serialise a state dict into the "MDXW" weights blob mdx_model_create
    reads (include/mdx.h): "MDXW" | u32 version 1 | u32 count | per tensor
    u32 name_len | name | u32 ndim | i64 shape[ndim] | float32 data."""
    parts = [b"MDXW", struct.pack("<II", 1, len(sd))]
    for k, v in sd.items():
        a = np.ascontiguousarray(torch.as_tensor(v).detach().to("cpu", torch.float32).numpy(), dtype="<f4")
        name = k.encode()
        parts.append(struct.pack("<I", len(name)))
        parts.append(name)
        parts.append(struct.pack("<I", a.ndim))
        parts.append(struct.pack(f"<{a.ndim}q", *a.shape))
        parts.append(a.tobytes())
    return b"".join(parts)
