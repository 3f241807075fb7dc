"""Architecture hyper-parameters of the extraction model.

Mirrors the Detectron2 config the reference builds in ``get_base_config()``
(M/model/config.py:21-94) on top of COCO ``keypoint_rcnn_R_50_FPN_3x``
(Base-RCNN-FPN + Base-Keypoint-RCNN-FPN), with the dataset additions of
``add_dataset_cfg`` (M/model/config.py:113-150) and the CLI overrides of
``InferenceStep.initialize`` (M/pipeline/inference_step.py:48-51).

Only inference-relevant keys are kept.  ``ModelConfig.from_yaml`` reads the
same keys from a Detectron2 ``config.yaml`` (``<model_dir>/config.yaml``) so a
trained model directory's overrides are honoured.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Tuple


@dataclass
class ModelConfig:
    # MODEL.RESNETS
    depth: int = 50                      # 50 or 101
    stem_out_channels: int = 64
    res2_out_channels: int = 256
    num_groups: int = 1
    width_per_group: int = 64
    stride_in_1x1: bool = True
    res5_dilation: int = 1
    # MODEL.FPN (M/model/config.py:82-83)
    fpn_out_channels: int = 256
    fpn_norm: str = "GN"                 # "" or "GN"
    fpn_fuse_type: str = "avg"           # "sum" or "avg"
    gn_groups: int = 32
    gn_eps: float = 1e-5
    # MODEL.ANCHOR_GENERATOR
    anchor_sizes: Tuple[int, ...] = (32, 64, 128, 256, 512)
    aspect_ratios: Tuple[float, ...] = (0.5, 1.0, 2.0)
    anchor_offset: float = 0.0
    # MODEL.RPN
    rpn_pre_nms_topk_test: int = 1000
    rpn_post_nms_topk_test: int = 1000
    rpn_nms_thresh: float = 0.7
    rpn_min_box_size: float = 0.0
    rpn_bbox_reg_weights: Tuple[float, ...] = (1.0, 1.0, 1.0, 1.0)
    # MODEL.ROI_HEADS
    num_classes: int = 1
    score_thresh_test: float = 0.5       # --instance-threshold (M/cli.py:340)
    nms_thresh_test: float = 0.5
    detections_per_image: int = 4        # --allowed-detections (M/cli.py:394-396)
    # MODEL.ROI_BOX_HEAD
    box_pooler_resolution: int = 7
    box_num_fc: int = 2
    box_fc_dim: int = 1024
    box_reg_weights: Tuple[float, ...] = (10.0, 10.0, 5.0, 5.0)
    # MODEL.ROI_MASK_HEAD
    mask_on: bool = True
    mask_pooler_resolution: int = 14
    mask_num_conv: int = 4
    mask_conv_dim: int = 256
    mask_threshold: float = 0.5
    # MODEL.ROI_KEYPOINT_HEAD (M/model/config.py:84)
    keypoint_on: bool = True
    keypoint_pooler_resolution: int = 7
    keypoint_conv_dims: Tuple[int, ...] = (512,) * 8
    num_keypoints: int = 8
    # pooler
    pooler_sampling_ratio: int = 0
    pooler_aligned: bool = True           # ROIAlignV2
    canonical_box_size: int = 224
    canonical_level: int = 4
    # INPUT / preprocessing (M/model/config.py:44, 141-148)
    input_format: str = "RGB"
    pixel_mean: Tuple[float, ...] = (1.12, 1.12, 1.12)
    pixel_std: Tuple[float, ...] = (5.79, 5.79, 5.79)
    size_divisibility: int = 32
    # extraction-side scaling (scale_raw_frames, M/pipeline/inference_step.py:24)
    min_height: float = 0
    max_height: float = 100

    @property
    def bbox_reg_clamp(self) -> float:
        return math.log(1000.0 / 16)

    @property
    def fpn_levels(self) -> List[int]:
        return [2, 3, 4, 5]

    @property
    def res_blocks(self) -> List[int]:
        return {50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}[self.depth]

    @property
    def in_channels(self) -> int:
        return 1 if self.input_format == "L" else 3

    @classmethod
    def from_yaml(cls, path: str, **overrides) -> "ModelConfig":
        """Read the inference keys of a Detectron2 config.yaml (SafeLoader)."""
        import yaml
        with open(path, "r", encoding="utf-8") as fh:
            y = yaml.safe_load(fh) or {}
        M = y.get("MODEL", {})
        c = cls()
        g = lambda d, k, default: (d or {}).get(k, default)  # noqa: E731
        R = M.get("RESNETS", {})
        c.depth = g(R, "DEPTH", c.depth)
        c.stride_in_1x1 = g(R, "STRIDE_IN_1X1", c.stride_in_1x1)
        c.res2_out_channels = g(R, "RES2_OUT_CHANNELS", c.res2_out_channels)
        c.stem_out_channels = g(R, "STEM_OUT_CHANNELS", c.stem_out_channels)
        F = M.get("FPN", {})
        c.fpn_norm = g(F, "NORM", c.fpn_norm)
        c.fpn_fuse_type = g(F, "FUSE_TYPE", c.fpn_fuse_type)
        c.fpn_out_channels = g(F, "OUT_CHANNELS", c.fpn_out_channels)
        H = M.get("ROI_HEADS", {})
        c.num_classes = g(H, "NUM_CLASSES", c.num_classes)
        c.score_thresh_test = g(H, "SCORE_THRESH_TEST", c.score_thresh_test)
        c.nms_thresh_test = g(H, "NMS_THRESH_TEST", c.nms_thresh_test)
        K = M.get("ROI_KEYPOINT_HEAD", {})
        c.num_keypoints = g(K, "NUM_KEYPOINTS", c.num_keypoints)
        c.keypoint_pooler_resolution = g(K, "POOLER_RESOLUTION", c.keypoint_pooler_resolution)
        c.keypoint_conv_dims = tuple(g(K, "CONV_DIMS", c.keypoint_conv_dims))
        c.keypoint_on = M.get("KEYPOINT_ON", c.keypoint_on)
        c.mask_on = M.get("MASK_ON", c.mask_on)
        c.pixel_mean = tuple(M.get("PIXEL_MEAN", c.pixel_mean))
        c.pixel_std = tuple(M.get("PIXEL_STD", c.pixel_std))
        c.input_format = y.get("INPUT", {}).get("FORMAT", c.input_format)
        c.detections_per_image = y.get("TEST", {}).get("DETECTIONS_PER_IMAGE", c.detections_per_image)
        RPN = M.get("RPN", {})
        c.rpn_pre_nms_topk_test = g(RPN, "PRE_NMS_TOPK_TEST", c.rpn_pre_nms_topk_test)
        c.rpn_post_nms_topk_test = g(RPN, "POST_NMS_TOPK_TEST", c.rpn_post_nms_topk_test)
        c.rpn_nms_thresh = g(RPN, "NMS_THRESH", c.rpn_nms_thresh)
        for k, v in overrides.items():
            setattr(c, k, v)
        return c
