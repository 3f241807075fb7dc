"""Architecture hyper-parameters of the extraction model.

Mirrors the Detectron2 config the reference builds in ``get_base_config()``
(M/model/config.py:21-94) on top of COCO ``keypoint_rcnn_R_50_FPN_3x``
(Base-RCNN-FPN + Base-Keypoint-RCNN-FPN), with the dataset additions of
``add_dataset_cfg`` (M/model/config.py:113-150) and the CLI overrides of
``InferenceStep.initialize`` (M/pipeline/inference_step.py:48-51).

Only inference-relevant keys are kept.  ``ModelConfig.from_yaml`` reads every
one of them from a Detectron2 ``config.yaml`` (``<model_dir>/config.yaml``) so
a trained model directory's overrides are honoured, and refuses settings the
native kernels do not implement.  The zero-padding multiple
(``size_divisibility``) is not a config key in Detectron2: it is the
backbone's (FPN: the res5 stride, 32).
"""
from __future__ import annotations

import math
import os
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
    # MODEL.WEIGHTS: the checkpoint Predictor.from_config loads ("" = none)
    weights: str = ""

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
        """Stem input channels: Detectron2 builds the backbone for
        ShapeSpec(channels=len(MODEL.PIXEL_MEAN)); an 'L' model with the base
        config's three means has a 3-channel stem (its 1-channel image is
        broadcast over the three normalisations in preprocess_image)."""
        return len(self.pixel_mean) if self.input_format == "L" else 3

    @classmethod
    def from_yaml(cls, path, **overrides) -> "ModelConfig":
        """Read a Detectron2 ``config.yaml`` as the reference does
        (``CfgNode.load_cfg``, M/model/config.py:7-18,
        M/pipeline/inference_step.py:37-38; here yaml.SafeLoader) -- a path or
        an already-loaded mapping.  Every key ``struct mdx_model_cfg``
        carries is read; keys the file omits keep the reference's base
        configuration (get_base_config).  Values the native kernels do not
        implement raise NotImplementedError naming the key, so a trained
        model directory is never silently run with another architecture.
        ``MODEL.WEIGHTS`` is kept in ``weights`` (Predictor.from_config
        loads it)."""
        if isinstance(path, (str, os.PathLike)):
            import yaml
            with open(path, "r", encoding="utf-8") as fh:
                y = yaml.safe_load(fh) or {}
        else:
            y = dict(path or {})
        c = cls()
        _read_yaml(c, y)
        for k, v in overrides.items():
            if not hasattr(c, k):
                raise AttributeError(f"ModelConfig has no field {k!r}")
            setattr(c, k, v)
        c.validate()
        return c

    def validate(self) -> "ModelConfig":
        """Refuse what the native model handle does not implement (the same
        limits mdx_model_create checks, with the Detectron2 key named)."""
        def need(ok, key, val, what):
            if not ok:
                raise NotImplementedError(f"{key} = {val!r}: {what}")
        need(self.depth in (50, 101), "MODEL.RESNETS.DEPTH", self.depth, "ResNet-50 and -101 are supported")
        need(self.num_groups == 1, "MODEL.RESNETS.NUM_GROUPS", self.num_groups, "must be 1")
        need(self.res5_dilation == 1, "MODEL.RESNETS.RES5_DILATION", self.res5_dilation, "must be 1")
        need(self.fpn_norm == "GN", "MODEL.FPN.NORM", self.fpn_norm, "the FPN convs run with GroupNorm")
        need(self.fpn_fuse_type in ("avg", "sum"), "MODEL.FPN.FUSE_TYPE", self.fpn_fuse_type, "'avg' or 'sum'")
        need(self.fpn_out_channels % 8 == 0, "MODEL.FPN.OUT_CHANNELS", self.fpn_out_channels, "a multiple of 8")
        need(len(self.anchor_sizes) == 5, "MODEL.ANCHOR_GENERATOR.SIZES", self.anchor_sizes,
             "one anchor size per level p2..p6")
        need(1 <= len(self.aspect_ratios) <= 8, "MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS", self.aspect_ratios,
             "1..8 ratios, the same at every level")
        need(self.num_classes == 1, "MODEL.ROI_HEADS.NUM_CLASSES", self.num_classes,
             "the extraction model has one class")
        need(1 <= self.detections_per_image <= 16, "TEST.DETECTIONS_PER_IMAGE", self.detections_per_image, "1..16")
        need(self.box_num_fc >= 1, "MODEL.ROI_BOX_HEAD.NUM_FC", self.box_num_fc, "at least one FC")
        need(len(self.keypoint_conv_dims) <= 16, "MODEL.ROI_KEYPOINT_HEAD.CONV_DIMS", self.keypoint_conv_dims,
             "at most 16 convs")
        need(self.input_format in ("RGB", "BGR", "L"), "INPUT.FORMAT", self.input_format, "'RGB', 'BGR' or 'L'")
        # one value per stem input channel: 3 for 'RGB' / 'BGR', 1 or 3 for
        # 'L' (a 3-value 'L' model has a 3-channel stem, see in_channels)
        need(len(self.pixel_mean) in ((1, 3) if self.input_format == "L" else (3,)), "MODEL.PIXEL_MEAN",
             self.pixel_mean, f"1 or 3 values for INPUT.FORMAT 'L', 3 otherwise")
        need(len(self.pixel_std) == len(self.pixel_mean), "MODEL.PIXEL_STD", self.pixel_std,
             "one value per MODEL.PIXEL_MEAN entry")
        for k in ("rpn_bbox_reg_weights", "box_reg_weights"):
            w = getattr(self, k)
            need(len(w) == 4 and all(v > 0 for v in w), k, w, "four positive weights")
        return self


def _read_yaml(c: ModelConfig, y: dict) -> None:
    """Detectron2 CfgNode keys -> ModelConfig fields (defaults: the
    reference's base configuration); unsupported settings raise."""
    def node(*path):
        d = y
        for p in path:
            d = (d or {}).get(p) if isinstance(d, dict) else None
        return d if isinstance(d, dict) else {}

    def get(d, k, default):
        v = d.get(k, default)
        return default if v is None else v

    def refuse(ok, key, val, what):
        if not ok:
            raise NotImplementedError(f"{key} = {val!r}: {what}")

    M = node("MODEL")
    refuse(get(M, "META_ARCHITECTURE", "GeneralizedRCNN") == "GeneralizedRCNN", "MODEL.META_ARCHITECTURE",
           M.get("META_ARCHITECTURE"), "GeneralizedRCNN only")
    bb = get(node("MODEL", "BACKBONE"), "NAME", "build_resnet_fpn_backbone")
    refuse(bb == "build_resnet_fpn_backbone", "MODEL.BACKBONE.NAME", bb, "ResNet-FPN only")
    c.weights = str(get(M, "WEIGHTS", "") or "")
    c.mask_on = bool(get(M, "MASK_ON", c.mask_on))
    c.keypoint_on = bool(get(M, "KEYPOINT_ON", c.keypoint_on))
    c.pixel_mean = tuple(float(v) for v in get(M, "PIXEL_MEAN", c.pixel_mean))
    c.pixel_std = tuple(float(v) for v in get(M, "PIXEL_STD", c.pixel_std))
    c.input_format = str(get(node("INPUT"), "FORMAT", c.input_format))
    c.detections_per_image = int(get(node("TEST"), "DETECTIONS_PER_IMAGE", c.detections_per_image))

    R = node("MODEL", "RESNETS")
    c.depth = int(get(R, "DEPTH", c.depth))
    c.stride_in_1x1 = bool(get(R, "STRIDE_IN_1X1", c.stride_in_1x1))
    c.res2_out_channels = int(get(R, "RES2_OUT_CHANNELS", c.res2_out_channels))
    c.stem_out_channels = int(get(R, "STEM_OUT_CHANNELS", c.stem_out_channels))
    c.num_groups = int(get(R, "NUM_GROUPS", c.num_groups))
    c.width_per_group = int(get(R, "WIDTH_PER_GROUP", c.width_per_group))
    c.res5_dilation = int(get(R, "RES5_DILATION", c.res5_dilation))
    norm = get(R, "NORM", "FrozenBN")
    refuse(norm == "FrozenBN", "MODEL.RESNETS.NORM", norm, "FrozenBN (folded into the convs at load)")
    deform = get(R, "DEFORM_ON_PER_STAGE", [False] * 4)
    refuse(not any(deform), "MODEL.RESNETS.DEFORM_ON_PER_STAGE", deform, "deformable convs are not implemented")
    of = list(get(R, "OUT_FEATURES", ["res2", "res3", "res4", "res5"]))
    refuse(of == ["res2", "res3", "res4", "res5"], "MODEL.RESNETS.OUT_FEATURES", of, "res2..res5")

    F = node("MODEL", "FPN")
    c.fpn_norm = str(get(F, "NORM", c.fpn_norm))
    c.fpn_fuse_type = str(get(F, "FUSE_TYPE", c.fpn_fuse_type))
    c.fpn_out_channels = int(get(F, "OUT_CHANNELS", c.fpn_out_channels))
    fi = list(get(F, "IN_FEATURES", ["res2", "res3", "res4", "res5"]))
    refuse(fi == ["res2", "res3", "res4", "res5"], "MODEL.FPN.IN_FEATURES", fi, "res2..res5 (+ LastLevelMaxPool p6)")

    A = node("MODEL", "ANCHOR_GENERATOR")
    an = get(A, "NAME", "DefaultAnchorGenerator")
    refuse(an == "DefaultAnchorGenerator", "MODEL.ANCHOR_GENERATOR.NAME", an,
           "axis-aligned anchors only (rotated boxes are not on the extract path)")
    def per_level(v):
        # DefaultAnchorGenerator._broadcast_params: a flat list is ONE entry,
        # broadcast to every level; a list of lists has one entry per level
        v = list(v)
        return [list(e) for e in v] if v and isinstance(v[0], (list, tuple)) else [v]

    sizes = per_level(get(A, "SIZES", [[s] for s in c.anchor_sizes]))
    # the kernels hold one anchor size per level
    refuse(all(len(v) == 1 for v in sizes) and len(sizes) in (1, 5), "MODEL.ANCHOR_GENERATOR.SIZES", sizes,
           "one size per level for p2..p6")
    c.anchor_sizes = tuple(float(v[0]) for v in (sizes * 5 if len(sizes) == 1 else sizes))
    ratios = per_level(get(A, "ASPECT_RATIOS", [list(c.aspect_ratios)]))
    refuse(len(ratios) in (1, 5) and all(r == ratios[0] for r in ratios), "MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS",
           ratios, "the same ratios at every level")
    c.aspect_ratios = tuple(float(v) for v in ratios[0])
    c.anchor_offset = float(get(A, "OFFSET", c.anchor_offset))

    P = node("MODEL", "PROPOSAL_GENERATOR")
    pn = get(P, "NAME", "RPN")
    refuse(pn == "RPN", "MODEL.PROPOSAL_GENERATOR.NAME", pn, "RPN only")
    c.rpn_min_box_size = float(get(P, "MIN_SIZE", c.rpn_min_box_size))
    RP = node("MODEL", "RPN")
    hn = get(RP, "HEAD_NAME", "StandardRPNHead")
    refuse(hn == "StandardRPNHead", "MODEL.RPN.HEAD_NAME", hn, "StandardRPNHead only")
    c.rpn_pre_nms_topk_test = int(get(RP, "PRE_NMS_TOPK_TEST", c.rpn_pre_nms_topk_test))
    c.rpn_post_nms_topk_test = int(get(RP, "POST_NMS_TOPK_TEST", c.rpn_post_nms_topk_test))
    c.rpn_nms_thresh = float(get(RP, "NMS_THRESH", c.rpn_nms_thresh))
    c.rpn_bbox_reg_weights = tuple(float(v) for v in get(RP, "BBOX_REG_WEIGHTS", c.rpn_bbox_reg_weights))
    refuse(len(c.rpn_bbox_reg_weights) == 4, "MODEL.RPN.BBOX_REG_WEIGHTS", c.rpn_bbox_reg_weights,
           "four weights (axis-aligned boxes)")
    ri = list(get(RP, "IN_FEATURES", ["p2", "p3", "p4", "p5", "p6"]))
    refuse(ri == ["p2", "p3", "p4", "p5", "p6"], "MODEL.RPN.IN_FEATURES", ri, "p2..p6")

    H = node("MODEL", "ROI_HEADS")
    rn = get(H, "NAME", "StandardROIHeads")
    refuse(rn == "StandardROIHeads", "MODEL.ROI_HEADS.NAME", rn, "StandardROIHeads only")
    c.num_classes = int(get(H, "NUM_CLASSES", c.num_classes))
    c.score_thresh_test = float(get(H, "SCORE_THRESH_TEST", c.score_thresh_test))
    c.nms_thresh_test = float(get(H, "NMS_THRESH_TEST", c.nms_thresh_test))
    hi = list(get(H, "IN_FEATURES", ["p2", "p3", "p4", "p5"]))
    refuse(hi == ["p2", "p3", "p4", "p5"], "MODEL.ROI_HEADS.IN_FEATURES", hi, "p2..p5")

    # the poolers: Detectron2 has one per head; the model handle has one
    # sampling ratio and one alignment mode for all of them
    poolers = {}

    def pooler(node_name, enabled):
        N_ = node("MODEL", node_name)
        pt = get(N_, "POOLER_TYPE", "ROIAlignV2")
        refuse(pt in ("ROIAlignV2", "ROIAlign"), f"MODEL.{node_name}.POOLER_TYPE", pt, "ROIAlignV2 or ROIAlign")
        if enabled:
            poolers[node_name] = (pt, int(get(N_, "POOLER_SAMPLING_RATIO", c.pooler_sampling_ratio)))
        return N_

    B_ = pooler("ROI_BOX_HEAD", True)
    bn = get(B_, "NAME", "FastRCNNConvFCHead")
    refuse(bn == "FastRCNNConvFCHead", "MODEL.ROI_BOX_HEAD.NAME", bn, "FastRCNNConvFCHead only")
    refuse(int(get(B_, "NUM_CONV", 0)) == 0, "MODEL.ROI_BOX_HEAD.NUM_CONV", B_.get("NUM_CONV"), "FC-only box head")
    refuse(get(B_, "NORM", "") == "", "MODEL.ROI_BOX_HEAD.NORM", B_.get("NORM"), "no norm in the box head")
    c.box_pooler_resolution = int(get(B_, "POOLER_RESOLUTION", c.box_pooler_resolution))
    c.box_num_fc = int(get(B_, "NUM_FC", c.box_num_fc))
    c.box_fc_dim = int(get(B_, "FC_DIM", c.box_fc_dim))
    c.box_reg_weights = tuple(float(v) for v in get(B_, "BBOX_REG_WEIGHTS", c.box_reg_weights))
    refuse(len(c.box_reg_weights) == 4, "MODEL.ROI_BOX_HEAD.BBOX_REG_WEIGHTS", c.box_reg_weights,
           "four weights (axis-aligned boxes)")
    K_ = pooler("ROI_MASK_HEAD", c.mask_on)
    mn = get(K_, "NAME", "MaskRCNNConvUpsampleHead")
    refuse(mn == "MaskRCNNConvUpsampleHead", "MODEL.ROI_MASK_HEAD.NAME", mn, "MaskRCNNConvUpsampleHead only")
    refuse(get(K_, "NORM", "") == "", "MODEL.ROI_MASK_HEAD.NORM", K_.get("NORM"), "no norm in the mask head")
    c.mask_pooler_resolution = int(get(K_, "POOLER_RESOLUTION", c.mask_pooler_resolution))
    c.mask_num_conv = int(get(K_, "NUM_CONV", c.mask_num_conv))
    c.mask_conv_dim = int(get(K_, "CONV_DIM", c.mask_conv_dim))
    P_ = pooler("ROI_KEYPOINT_HEAD", c.keypoint_on)
    kn = get(P_, "NAME", "KRCNNConvDeconvUpsampleHead")
    refuse(kn == "KRCNNConvDeconvUpsampleHead", "MODEL.ROI_KEYPOINT_HEAD.NAME", kn, "KRCNNConvDeconvUpsampleHead only")
    c.num_keypoints = int(get(P_, "NUM_KEYPOINTS", c.num_keypoints))
    c.keypoint_pooler_resolution = int(get(P_, "POOLER_RESOLUTION", c.keypoint_pooler_resolution))
    c.keypoint_conv_dims = tuple(int(v) for v in get(P_, "CONV_DIMS", c.keypoint_conv_dims))
    kinds = set(poolers.values())
    refuse(len(kinds) == 1, "MODEL.ROI_*_HEAD.POOLER_TYPE / POOLER_SAMPLING_RATIO", poolers,
           "the same pooler type and sampling ratio for every head")
    pt, sr = kinds.pop()
    c.pooler_aligned = pt == "ROIAlignV2"
    c.pooler_sampling_ratio = sr
