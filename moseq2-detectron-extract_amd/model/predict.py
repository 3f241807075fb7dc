"""Predictor -- drop-in for the reference's DefaultPredictor-shaped wrapper
(M/model/predict.py:12-102), backed by the MI355X-native runtime.

Same constructors (``from_config``; ``from_torchscript`` reads an exported
archive weights-only, see model/torchscript.py),
same ``device`` property and the same call contract: uint8 ``(H,W,C)`` or
``(N,H,W,C)`` (numpy or torch) -> ``{'instances': Instances}`` or a list of
them, with Detectron2's field names.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import numpy as np
import torch

from .config import ModelConfig
from .runtime import MaskRCNN
from .structures import Boxes, Instances
from .weights import load_state_dict, synthetic_state_dict


class Predictor:
    def __init__(self, model: MaskRCNN, is_torchscript: bool = False):
        self.model = model
        self.is_torchscript = is_torchscript

    @property
    def device(self):
        return self.model.device

    @classmethod
    def from_config(cls, cfg: Union[ModelConfig, str], weights: Union[None, str, dict] = None,
                    dtype: str = "fp32", device="cuda", seed: int = 0) -> "Predictor":
        """cfg: ModelConfig or path to a Detectron2 config.yaml.  weights: path to
        a Detectron2 checkpoint (.pth, loaded weights_only), a state dict, or
        None for seeded synthetic weights (no trained checkpoint is available
        offline)."""
        if isinstance(cfg, str):
            cfg = ModelConfig.from_yaml(cfg)
        if weights is None:
            sd = synthetic_state_dict(cfg, seed)
        elif isinstance(weights, str):
            sd = load_state_dict(weights)
        else:
            sd = weights
        return cls(MaskRCNN(cfg, sd, device=device, dtype=dtype))

    @classmethod
    def from_torchscript(cls, path: str, cfg: Optional[ModelConfig] = None, dtype: str = "fp32", device="cuda",
                         **overrides) -> "Predictor":
        """An exported ``model.ts`` (M/model/predict.py:46-51, export
        M/model/deploy.py:77-121): its parameters, buffers and thresholds are
        read weights-only from the archive (model/torchscript.py; no
        TorchScript is executed) and run on the native kernels.  The
        architecture is inferred from the state dict unless `cfg` is given;
        `overrides` set ModelConfig fields (e.g. score_thresh_test)."""
        from .torchscript import infer_config, load_torchscript
        sd, scalars = load_torchscript(path)
        if cfg is None:
            cfg = infer_config(sd, scalars, **overrides)
        else:
            for k, v in overrides.items():
                setattr(cfg, k, v)
        return cls(MaskRCNN(cfg, sd, device=device, dtype=dtype), is_torchscript=True)

    def run(self, frames_u8: torch.Tensor, lut: Optional[np.ndarray] = None) -> dict:
        """Batched device-resident call: uint8 (B,h,w) GPU tensor -> dict of
        fixed-shape device tensors (see MaskRCNN.forward)."""
        return self.model.forward(frames_u8, lut)

    def __call__(self, original_image):
        return_as_list = True
        if len(original_image.shape) == 3:
            return_as_list = False
            original_image = original_image[None, ...]
        if original_image.shape[3] != 1:
            c0 = original_image[..., :1]
            same = bool((original_image == c0).all()) if isinstance(original_image, torch.Tensor) else \
                bool(np.all(original_image == c0))
            if not same:
                raise NotImplementedError("only single-channel depth frames (replicated to RGB) are supported")
            original_image = c0
        if isinstance(original_image, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(original_image[..., 0])).to(self.device)
        else:
            x = original_image[..., 0].to(self.device).contiguous()
        if x.dtype != torch.uint8:
            raise TypeError("Predictor expects uint8 images")
        out = self.model.forward(x)
        preds = outputs_to_instances(out, x.shape[1], x.shape[2])
        if not return_as_list:
            return preds[0]
        return preds


def outputs_to_instances(out: dict, h: int, w: int):
    """Fixed-shape device outputs -> per-image Instances (one host sync for
    the detection counts)."""
    ndet = out["ndet"].cpu().tolist()
    res = []
    for b, n in enumerate(ndet):
        fields = {
            "pred_boxes": Boxes(out["boxes"][b, :n]),
            "scores": out["scores"][b, :n],
            "pred_classes": out["classes"][b, :n],
        }
        if "masks" in out:
            fields["pred_masks"] = out["masks"][b, :n].bool()
        if "keypoints" in out:
            fields["pred_keypoints"] = out["keypoints"][b, :n]
            fields["pred_keypoint_heatmaps"] = out["keypoint_heatmaps"][b, :n]
        res.append({"instances": Instances((h, w), **fields)})
    return res
