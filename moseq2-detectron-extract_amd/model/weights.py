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
import os
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


def state_dict_spec(cfg: ModelConfig = ModelConfig()):
    """[(name, shape, init)] of the reference model's state dict, in
    GeneralizedRCNN's order; init = ("normal", std) | ("unif", lo, hi) |
    ("gn_weight", std) | ("const", values).  The names and shapes a
    checkpoint for this configuration must carry (check_state_dict) and the
    draw order of the seeded synthetic weights."""
    spec = []

    def conv(name, cout, cin, k, bias=False, std=None):
        fan_in = cin * k * k
        spec.append((f"{name}.weight", (cout, cin, k, k), ("normal", std if std is not None else math.sqrt(2.0 / fan_in))))
        if bias:
            spec.append((f"{name}.bias", (cout,), ("normal", 0.05)))

    def frozen_bn(name, c, wlo=0.8, whi=1.2):
        spec.append((f"{name}.weight", (c,), ("unif", wlo, whi)))
        spec.append((f"{name}.bias", (c,), ("normal", 0.1)))
        spec.append((f"{name}.running_mean", (c,), ("normal", 0.1)))
        spec.append((f"{name}.running_var", (c,), ("unif", 0.5, 1.5)))

    bu = "backbone.bottom_up"
    conv(f"{bu}.stem.conv1", cfg.stem_out_channels, cfg.in_channels, 7)
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
                spec.append((f"backbone.fpn_{k}{lvl}.norm.weight", (C,), ("gn_weight", 0.1)))
                spec.append((f"backbone.fpn_{k}{lvl}.norm.bias", (C,), ("normal", 0.1)))
    A = len(cfg.aspect_ratios)
    conv("proposal_generator.rpn_head.conv", C, C, 3, bias=True)
    conv("proposal_generator.rpn_head.objectness_logits", A, C, 1, bias=True, std=0.08)
    conv("proposal_generator.rpn_head.anchor_deltas", 4 * A, C, 1, bias=True, std=0.01)
    R = cfg.box_pooler_resolution
    fin = C * R * R
    for i in range(cfg.box_num_fc):
        spec.append((f"roi_heads.box_head.fc{i + 1}.weight", (cfg.box_fc_dim, fin), ("normal", math.sqrt(2.0 / fin))))
        spec.append((f"roi_heads.box_head.fc{i + 1}.bias", (cfg.box_fc_dim,), ("normal", 0.02)))
        fin = cfg.box_fc_dim
    spec.append(("roi_heads.box_predictor.cls_score.weight", (cfg.num_classes + 1, fin), ("normal", 0.3)))
    spec.append(("roi_heads.box_predictor.cls_score.bias", (cfg.num_classes + 1,), ("normal", 0.1)))
    spec.append(("roi_heads.box_predictor.bbox_pred.weight", (4 * cfg.num_classes, fin), ("normal", 0.01)))
    spec.append(("roi_heads.box_predictor.bbox_pred.bias", (4 * cfg.num_classes,), ("normal", 0.01)))
    if cfg.mask_on:
        cin = C
        for i in range(cfg.mask_num_conv):
            conv(f"roi_heads.mask_head.mask_fcn{i + 1}", cfg.mask_conv_dim, cin, 3, bias=True)
            cin = cfg.mask_conv_dim
        spec.append(("roi_heads.mask_head.deconv.weight", (cin, cfg.mask_conv_dim, 2, 2),
                     ("normal", math.sqrt(2.0 / (cin * 4)))))
        spec.append(("roi_heads.mask_head.deconv.bias", (cfg.mask_conv_dim,), ("normal", 0.05)))
        conv("roi_heads.mask_head.predictor", cfg.num_classes, cfg.mask_conv_dim, 1, bias=True, std=0.1)
    if cfg.keypoint_on:
        cin = C
        for i, d in enumerate(cfg.keypoint_conv_dims):
            conv(f"roi_heads.keypoint_head.conv_fcn{i + 1}", d, cin, 3, bias=True)
            cin = d
        spec.append(("roi_heads.keypoint_head.score_lowres.weight", (cin, cfg.num_keypoints, 4, 4), ("normal", 0.05)))
        spec.append(("roi_heads.keypoint_head.score_lowres.bias", (cfg.num_keypoints,), ("normal", 0.05)))
    return spec


def synthetic_state_dict(cfg: ModelConfig = ModelConfig(), seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Seeded random weights with the reference model's names and shapes
    (state_dict_spec, drawn in its order)."""
    g = torch.Generator().manual_seed(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for name, shape, init in state_dict_spec(cfg):
        if init[0] == "normal":
            sd[name] = torch.randn(*shape, generator=g) * init[1]
        elif init[0] == "gn_weight":
            sd[name] = 1.0 + torch.randn(*shape, generator=g) * init[1]
        else:
            sd[name] = torch.rand(*shape, generator=g) * (init[2] - init[1]) + init[1]
    sd["pixel_mean"] = torch.tensor(cfg.pixel_mean, dtype=torch.float32).view(-1, 1, 1)
    sd["pixel_std"] = torch.tensor(cfg.pixel_std, dtype=torch.float32).view(-1, 1, 1)
    return sd


def check_state_dict(sd: Mapping[str, torch.Tensor], cfg: ModelConfig, source: str = "checkpoint") -> list:
    """Every tensor the configuration needs is present with its shape
    (DetectionCheckpointer.load would report a missing or mis-shaped
    parameter; here it is an error, as the native handle cannot run without
    it).  Returns the unexpected keys (ignored, as Detectron2 does)."""
    want = {n: tuple(s) for n, s, _ in state_dict_spec(cfg)}
    missing = [n for n in want if n not in sd]
    if missing:
        raise ValueError(f"{source}: {len(missing)} parameter(s) of this configuration missing, e.g. "
                         f"{missing[:4]} -- does <model_dir>/config.yaml match the checkpoint?")
    bad = [(n, tuple(sd[n].shape), s) for n, s in want.items() if tuple(sd[n].shape) != s]
    if bad:
        raise ValueError(f"{source}: shape mismatch for {len(bad)} parameter(s), e.g. "
                         + "; ".join(f"{n}: {a} in the checkpoint, {b} for the config" for n, a, b in bad[:3]))
    return [n for n in sd if n not in want and n not in ("pixel_mean", "pixel_std")]


def load_state_dict(path: str) -> "OrderedDict[str, torch.Tensor]":
    """Load a Detectron2 checkpoint safely (weights_only=True): a
    ``model_final.pth`` / ``model_XXXXXXX.pth`` as DefaultTrainer writes it
    ({'model': state_dict, 'optimizer': ..., 'iteration': ...}) or a bare
    state dict.  Detectron2's ``.pkl`` model-zoo format is a pickle and is
    refused (nothing in a checkpoint is executed here)."""
    if not os.path.isfile(path):
        raise FileNotFoundError(f"MODEL.WEIGHTS: no checkpoint at {path!r}")
    if path.endswith(".pkl"):
        raise ValueError(f"{path}: Detectron2 .pkl checkpoints are pickles and are not loaded; save the model's "
                         "state_dict as a .pth")
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
