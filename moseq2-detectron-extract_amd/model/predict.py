"""Predictor -- drop-in for the reference's DefaultPredictor-shaped wrapper
(M/model/predict.py:12-102), backed by the MI355X-native runtime.

Same constructors (``from_config`` loads ``MODEL.WEIGHTS`` of the config;
``from_model_dir`` is InferenceStep's model-directory set-up;
``from_torchscript`` reads an exported archive weights-only, see
model/torchscript.py),
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
from .weights import check_state_dict, load_state_dict, synthetic_state_dict


class Predictor:
    def __init__(self, model: MaskRCNN, is_torchscript: bool = False):
        self.model = model
        self.is_torchscript = is_torchscript

    @property
    def device(self):
        return self.model.device

    @classmethod
    def from_config(cls, cfg: Union[ModelConfig, str, dict], weights: Union[None, str, dict] = None,
                    dtype: str = "fp32", device="cuda", seed: int = 0,
                    policy: Optional[dict] = None) -> "Predictor":
        """The reference constructor (M/model/predict.py:31-44): build the
        model of `cfg`, load ``cfg.MODEL.WEIGHTS`` and check the input format.

        cfg: a ModelConfig, a path to a Detectron2 ``config.yaml`` or its
        loaded mapping (ModelConfig.from_yaml: every inference key read,
        unsupported settings refused).  weights: None loads MODEL.WEIGHTS
        (``cfg.weights``; a ``.pth`` read weights-only) and raises when it is
        empty or missing; a path or a state dict overrides it; the string
        ``"synthetic"`` selects seeded synthetic weights of this architecture
        (benchmarks and tests: no trained checkpoint exists offline).  The
        state dict must carry every parameter of the configuration with its
        shape (weights.check_state_dict).  policy: kernel-selection policy
        fields for this predictor's model handle (MaskRCNN)."""
        cfg, sd = resolve_model(cfg, weights, seed)
        return cls(MaskRCNN(cfg, sd, device=device, dtype=dtype, policy=policy))

    @classmethod
    def from_model_dir(cls, model_dir: str, checkpoint: Union[str, int] = "last", instance_threshold: float = 0.5,
                       allowed_detections: int = 4, dtype: str = "fp32", device="cuda") -> "Predictor":
        """What InferenceStep.initialize does with a trained model directory
        (M/pipeline/inference_step.py:35-52): ``<model_dir>/config.yaml``,
        MODEL.WEIGHTS = the last checkpoint (``last_checkpoint`` file) or the
        one of iteration `checkpoint`, SCORE_THRESH_TEST = --instance-threshold,
        DETECTIONS_PER_IMAGE = --allowed-detections, then from_config."""
        cfg = model_dir_config(model_dir, checkpoint, instance_threshold, allowed_detections)
        return cls.from_config(cfg, dtype=dtype, device=device)

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


def model_dir_config(model_dir: str, checkpoint: Union[str, int] = "last", instance_threshold: float = 0.5,
                     allowed_detections: int = 4) -> ModelConfig:
    """The ModelConfig InferenceStep.initialize builds for a model directory
    (M/pipeline/inference_step.py:35-51), MODEL.WEIGHTS resolved."""
    from .util import get_last_checkpoint, get_specific_checkpoint
    cfg = ModelConfig.from_yaml(os.path.join(model_dir, "config.yaml"))
    cfg.weights = (get_last_checkpoint(model_dir) if checkpoint == "last"
                   else get_specific_checkpoint(model_dir, checkpoint))
    cfg.score_thresh_test = float(instance_threshold)
    cfg.detections_per_image = int(allowed_detections)
    return cfg


def resolve_model(cfg: Union[ModelConfig, str, dict], weights: Union[None, str, dict] = None, seed: int = 0):
    """The host half of from_config (no GPU needed): the ModelConfig and the
    checked state dict it will run."""
    if not isinstance(cfg, ModelConfig):
        cfg = ModelConfig.from_yaml(cfg)
    cfg.validate()
    if isinstance(weights, str) and weights == "synthetic":
        sd, source = synthetic_state_dict(cfg, seed), "synthetic"
    elif weights is None:
        if not cfg.weights:
            raise ValueError("MODEL.WEIGHTS is empty: set it (or pass weights=<checkpoint path | state dict>); "
                             "weights='synthetic' runs seeded synthetic weights")
        sd, source = load_state_dict(cfg.weights), cfg.weights
    elif isinstance(weights, (str, os.PathLike)):
        sd, source = load_state_dict(str(weights)), str(weights)
    else:
        sd, source = weights, "state dict"
    # DetectionCheckpointer.load + `assert model.input_format ==
    # cfg.INPUT.FORMAT`: every parameter of the configuration, the stem
    # taking the configured channels
    check_state_dict(sd, cfg, source)
    return cfg, sd


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
