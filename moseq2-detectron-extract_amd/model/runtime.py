"""MI355X-native Mask/Keypoint R-CNN inference runtime: the Python face of the
libmdx model handle (include/mdx.h, csrc/model.hip).

mdx_model_create receives the Detectron2 state dict as an "MDXW" blob
(weights.pack_blob) and the CfgNode hyper-parameters as struct
mdx_model_cfg; it folds FrozenBN, packs every weight into its kernel's layout
and uploads it.  mdx_model_forward enqueues the whole forward -- every layer a
hand-written gfx950 kernel -- on the current HIP stream with no host
synchronisation (fixed shapes: 1000 proposals/image, D detections/image,
counts kept on the device), so it can be captured into a HIP graph and
replayed; its intermediates live in a per-stream device arena.

The layer sequence follows Detectron2's GeneralizedRCNN as configured by the
reference (M/model/config.py:21-94); see oracle/model_ref.py for the CPU
restatement used as the parity checker.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional

import numpy as np
import torch

from .._lib import MdxError, Policy, call, lib, policy_scope
from .config import ModelConfig
from .weights import pack_blob, resnet_stage_specs

# "mixed": fp32 backbone / FPN / RPN / box head, fp16 mask + keypoint heads
# (BASELINE config 5: "Keypoint+Mask heads fp16")
_DT = {"fp32": 0, "fp16": 1, "mixed": 0}
_HEAD_DT = {"fp32": 0, "fp16": 0, "mixed": 1}
_TDT = {0: torch.float32, 1: torch.float16, 2: torch.int32, 3: torch.bfloat16}


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class ModelCfgC(ctypes.Structure):
    """struct mdx_model_cfg (include/mdx.h)."""
    _fields_ = [
        ("depth", ctypes.c_int), ("dtype", ctypes.c_int), ("stem_out_channels", ctypes.c_int),
        ("res2_out_channels", ctypes.c_int), ("width_per_group", ctypes.c_int), ("stride_in_1x1", ctypes.c_int),
        ("fpn_out_channels", ctypes.c_int), ("fpn_fuse_avg", ctypes.c_int), ("gn_groups", ctypes.c_int),
        ("gn_eps", ctypes.c_float), ("n_anchor_sizes", ctypes.c_int), ("anchor_sizes", ctypes.c_float * 5),
        ("n_aspect_ratios", ctypes.c_int), ("aspect_ratios", ctypes.c_float * 8), ("anchor_offset", ctypes.c_float),
        ("rpn_pre_nms_topk", ctypes.c_int), ("rpn_post_nms_topk", ctypes.c_int), ("rpn_nms_thresh", ctypes.c_float),
        ("rpn_min_box_size", ctypes.c_float), ("num_classes", ctypes.c_int), ("score_thresh", ctypes.c_float),
        ("nms_thresh", ctypes.c_float), ("detections_per_image", ctypes.c_int),
        ("box_pooler_resolution", ctypes.c_int), ("box_num_fc", ctypes.c_int), ("box_fc_dim", ctypes.c_int),
        ("box_reg_weights", ctypes.c_float * 4), ("mask_on", ctypes.c_int), ("mask_pooler_resolution", ctypes.c_int),
        ("mask_num_conv", ctypes.c_int), ("mask_conv_dim", ctypes.c_int), ("mask_threshold", ctypes.c_float),
        ("keypoint_on", ctypes.c_int), ("keypoint_pooler_resolution", ctypes.c_int),
        ("n_keypoint_convs", ctypes.c_int), ("keypoint_conv_dims", ctypes.c_int * 16), ("num_keypoints", ctypes.c_int),
        ("pooler_sampling_ratio", ctypes.c_int), ("pooler_aligned", ctypes.c_int),
        ("canonical_box_size", ctypes.c_float), ("canonical_level", ctypes.c_float), ("in_channels", ctypes.c_int),
        ("pixel_mean", ctypes.c_float * 3), ("pixel_std", ctypes.c_float * 3), ("size_divisibility", ctypes.c_int),
        ("rpn_bbox_reg_weights", ctypes.c_float * 4), ("head_dtype", ctypes.c_int),
    ]


class OutputsC(ctypes.Structure):
    """struct mdx_model_outputs (include/mdx.h)."""
    _fields_ = [("boxes", ctypes.c_void_p), ("scores", ctypes.c_void_p), ("classes", ctypes.c_void_p),
                ("ndet", ctypes.c_void_p), ("masks", ctypes.c_void_p), ("mask_plane_stride", ctypes.c_int64),
                ("keypoints", ctypes.c_void_p), ("keypoint_heatmaps", ctypes.c_void_p)]


class ConvRecordC(ctypes.Structure):
    """struct mdx_conv_record (include/mdx.h)."""
    _fields_ = [("kernel", ctypes.c_int), ("ksplit", ctypes.c_int), ("M", ctypes.c_int64), ("N", ctypes.c_int64),
                ("K", ctypes.c_int64), ("flop", ctypes.c_double), ("ms", ctypes.c_double), ("dtype", ctypes.c_int),
                ("reserved", ctypes.c_int)]


def model_cfg_c(cfg: ModelConfig, dtype: str) -> ModelCfgC:
    """ModelConfig (Detectron2 CfgNode keys) -> struct mdx_model_cfg."""
    cfg.validate()
    c = ModelCfgC()
    c.depth, c.dtype = cfg.depth, _DT[dtype]
    c.stem_out_channels, c.res2_out_channels, c.width_per_group = (cfg.stem_out_channels, cfg.res2_out_channels,
                                                                   cfg.width_per_group)
    c.stride_in_1x1 = int(cfg.stride_in_1x1)
    c.fpn_out_channels, c.fpn_fuse_avg, c.gn_groups, c.gn_eps = (cfg.fpn_out_channels,
                                                                 int(cfg.fpn_fuse_type == "avg"), cfg.gn_groups,
                                                                 cfg.gn_eps)
    c.n_anchor_sizes = len(cfg.anchor_sizes)
    c.anchor_sizes[:] = [float(v) for v in cfg.anchor_sizes]
    c.n_aspect_ratios = len(cfg.aspect_ratios)
    for i, v in enumerate(cfg.aspect_ratios):
        c.aspect_ratios[i] = float(v)
    c.anchor_offset = cfg.anchor_offset
    c.rpn_pre_nms_topk, c.rpn_post_nms_topk = cfg.rpn_pre_nms_topk_test, cfg.rpn_post_nms_topk_test
    c.rpn_nms_thresh, c.rpn_min_box_size = cfg.rpn_nms_thresh, cfg.rpn_min_box_size
    c.num_classes, c.score_thresh, c.nms_thresh = cfg.num_classes, cfg.score_thresh_test, cfg.nms_thresh_test
    c.detections_per_image = cfg.detections_per_image
    c.box_pooler_resolution, c.box_num_fc, c.box_fc_dim = (cfg.box_pooler_resolution, cfg.box_num_fc,
                                                           cfg.box_fc_dim)
    c.box_reg_weights[:] = [float(v) for v in cfg.box_reg_weights]
    c.mask_on, c.mask_pooler_resolution = int(cfg.mask_on), cfg.mask_pooler_resolution
    c.mask_num_conv, c.mask_conv_dim, c.mask_threshold = cfg.mask_num_conv, cfg.mask_conv_dim, cfg.mask_threshold
    c.keypoint_on, c.keypoint_pooler_resolution = int(cfg.keypoint_on), cfg.keypoint_pooler_resolution
    c.n_keypoint_convs = len(cfg.keypoint_conv_dims)
    for i, v in enumerate(cfg.keypoint_conv_dims):
        c.keypoint_conv_dims[i] = int(v)
    c.num_keypoints = cfg.num_keypoints
    c.pooler_sampling_ratio, c.pooler_aligned = cfg.pooler_sampling_ratio, int(cfg.pooler_aligned)
    c.canonical_box_size, c.canonical_level = float(cfg.canonical_box_size), float(cfg.canonical_level)
    c.in_channels = cfg.in_channels
    c.pixel_mean[:] = [float(v) for v in (list(cfg.pixel_mean) * 3)[:3]]
    c.pixel_std[:] = [float(v) for v in (list(cfg.pixel_std) * 3)[:3]]
    c.size_divisibility = cfg.size_divisibility
    c.rpn_bbox_reg_weights[:] = [float(v) for v in cfg.rpn_bbox_reg_weights]
    c.head_dtype = _HEAD_DT[dtype]
    return c


class MaskRCNN:
    """The reference model on one GPU behind the libmdx model handle
    (mdx_model_create / mdx_model_forward / mdx_model_destroy).  `policy`:
    fields of the kernel-selection policy (include/mdx.h mdx_policy) this
    handle runs with, over the calling thread's; the handle captures it at
    creation, so handles with different policies run side by side."""

    def __init__(self, cfg: ModelConfig, state_dict: Dict[str, torch.Tensor], device="cuda", dtype: str = "fp32",
                 policy: Optional[dict] = None):
        if not torch.cuda.is_available():
            raise MdxError("MaskRCNN needs an AMD GPU; there is no CPU fallback")
        if dtype not in _DT:
            raise ValueError("dtype must be 'fp32', 'fp16' or 'mixed' (fp32 trunk, fp16 mask + keypoint heads)")
        if cfg.num_classes != 1:
            raise NotImplementedError("the extraction model has one class (ROI_HEADS.NUM_CLASSES=1)")
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        self.tdt = torch.float16 if dtype == "fp16" else torch.float32
        self._ccfg = model_cfg_c(cfg, dtype)
        blob = pack_blob(state_dict)
        h = ctypes.c_void_p()
        with policy_scope(**(policy or {})):
            call("mdx_model_create", blob, len(blob), ctypes.byref(self._ccfg), self.device.index, ctypes.byref(h))
        self._h = h
        self._lib = lib()

    def policy(self) -> dict:
        """The kernel-selection policy this handle runs with."""
        p = Policy()
        call("mdx_model_get_policy", self._h, ctypes.byref(p))
        return p.as_dict()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.mdx_model_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------ forward
    def padded_size(self, h, w):
        d = self.cfg.size_divisibility
        return (h + d - 1) // d * d, (w + d - 1) // d * d

    def reserve(self, B: int, h: int, w: int):
        """Workspace for forwards of up to B frames of h x w on the current
        stream (mdx_model_reserve): before capturing a forward in a graph."""
        call("mdx_model_reserve", self._h, B, h, w, _stream())

    def tensor(self, name: str) -> torch.Tensor:
        """Copy of an intermediate of the last forward on the current stream."""
        shape = (ctypes.c_int64 * 4)()
        dt = ctypes.c_int()
        call("mdx_model_tensor_info", self._h, _stream(), name.encode(), shape, ctypes.byref(dt))
        t = torch.empty(tuple(shape), dtype=_TDT[dt.value], device=self.device)
        call("mdx_model_tensor_copy", self._h, _stream(), name.encode(), _p(t), t.numel() * t.element_size())
        return t

    def debug_fill(self, B: int, h: int, w: int, byte: int):
        """Fill the current stream's workspace with `byte` (testing aid)."""
        call("mdx_model_debug_fill", self._h, B, h, w, int(byte), _stream())

    def profile(self, on: bool) -> bool:
        """Time every conv launch of later forwards (HIP events)."""
        return bool(call("mdx_model_profile", self._h, int(on)))

    def profile_read(self, max_records: int = 4096):
        """[(kernel, ksplit, M, N, K, flop, ms, dtype)] of the last profiled
        forward (the stream must be synchronised; dtype 0 f32, 1 f16)."""
        buf = (ConvRecordC * max_records)()
        n = call("mdx_model_profile_read", self._h, buf, max_records)
        return [(r.kernel, r.ksplit, r.M, r.N, r.K, r.flop, r.ms, r.dtype) for r in buf[:n]]

    @torch.no_grad()
    def forward(self, frames: torch.Tensor, lut: Optional[np.ndarray] = None, intermediates: bool = False):
        """frames: uint8 (B, h, w) device tensor.  lut: 256-entry scale table
        applied first (scale_raw_frames fused), identity if None.  Returns a dict
        of device tensors: boxes (B,D,4) f32, scores (B,D), classes (B,D) i64,
        ndet (B,) i32, masks (B,D,h,w) u8, keypoints (B,D,K,3) f32,
        keypoint_heatmaps (B,D,K,28,28) f32."""
        cfg = self.cfg
        if frames.dim() != 3 or frames.dtype != torch.uint8 or not frames.is_cuda:
            raise ValueError("frames must be a uint8 (B, h, w) GPU tensor")
        frames = frames.contiguous()
        B, h, w = frames.shape
        D, K = cfg.detections_per_image, cfg.num_keypoints
        dev = self.device
        o = OutputsC()
        out = {"boxes": torch.empty((B, D, 4), dtype=torch.float32, device=dev),
               "scores": torch.empty((B, D), dtype=torch.float32, device=dev),
               "classes": torch.empty((B, D), dtype=torch.int64, device=dev),
               "ndet": torch.empty((B,), dtype=torch.int32, device=dev)}
        o.boxes, o.scores, o.classes, o.ndet = (out[k].data_ptr() for k in ("boxes", "scores", "classes", "ndet"))
        if cfg.mask_on:
            plane = (h * w + 15) // 16 * 16  # 16-B aligned planes for the selection kernel
            mbuf = torch.empty((B, D, plane), dtype=torch.uint8, device=dev)
            o.masks, o.mask_plane_stride = mbuf.data_ptr(), plane
            out["masks"] = torch.as_strided(mbuf, (B, D, h, w), (D * plane, plane, w, 1))
            out["mask_planes"] = (mbuf, plane)
        if cfg.keypoint_on:
            S = 4 * cfg.keypoint_pooler_resolution
            out["keypoints"] = torch.empty((B, D, K, 3), dtype=torch.float32, device=dev)
            out["keypoint_heatmaps"] = torch.empty((B, D, K, S, S), dtype=torch.float32, device=dev)
            o.keypoints, o.keypoint_heatmaps = out["keypoints"].data_ptr(), out["keypoint_heatmaps"].data_ptr()
        lut_p = None
        if lut is not None:
            lut = np.ascontiguousarray(lut, np.uint8)
            lut_p = lut.ctypes.data_as(ctypes.c_void_p)
        call("mdx_model_forward", self._h, _p(frames), B, h, w, lut_p, ctypes.byref(o), _stream())
        if intermediates:
            Hp, Wp = self.padded_size(h, w)
            inter = {"input": s2d_to_nhwc(self.tensor("input_s2d"), Hp, Wp, cfg)}
            for k in ("res2", "res3", "res4", "res5", "p2", "p3", "p4", "p5", "p6"):
                inter[k] = self.tensor(k)
            inter["proposals"] = self.tensor("proposals")[..., 0]
            inter["proposal_scores"] = self.tensor("proposal_scores")[..., 0, 0]
            inter["proposal_count"] = self.tensor("proposal_count").view(B)
            bp = self.tensor("box_pooled")
            if bp.dtype == torch.bfloat16:  # split-plane mode: hi + mid + lo planes of each 16 values
                P, C = cfg.box_pooler_resolution, cfg.fpn_out_channels
                bp = bp.float().sum(2).reshape(bp.shape[0], P, P, C)
            inter["box_pooled"] = bp
            inter["box_pred"] = self.tensor("box_pred")[..., 0, 0]
            if cfg.mask_on:
                inter["mask_logits"] = self.tensor("mask_logits")
            out["intermediates"] = inter
        return out


def s2d_to_nhwc(x: torch.Tensor, Hp: int, Wp: int, cfg: Optional[ModelConfig] = None) -> torch.Tensor:
    """(B, Hp/2+1, Wp/2+1, 16) space-to-depth input -> (B, Hp, Wp, 4) NHWC.
    The folded stem's 8-channel form (per phase: scaled pixel, inside flag)
    is expanded to the normalised input (x - mean_c) / std_c inside the image,
    0 outside (cfg's pixel mean / std), channels beyond in_channels zero."""
    B, C = x.shape[0], x.shape[-1]
    t = x.view(B, Hp // 2 + 1, Wp // 2 + 1, 2, 2, C // 4).permute(0, 1, 3, 2, 4, 5)
    t = t.reshape(B, Hp + 2, Wp + 2, C // 4)[:, 1:Hp + 1, 1:Wp + 1]
    if C == 16:
        return t.contiguous()
    if cfg is None:
        raise ValueError("s2d_to_nhwc: the folded 8-channel input needs the model config")
    v, inside = t[..., 0], t[..., 1] > 0
    out = torch.zeros(t.shape[:3] + (4,), dtype=t.dtype, device=t.device)
    for c in range(cfg.in_channels):
        # tensor operands: an IEEE division as in the preprocess kernel (a
        # python-scalar divisor becomes a multiply by its reciprocal)
        mean = torch.full_like(v, cfg.pixel_mean[c])
        std = torch.full_like(v, cfg.pixel_std[c])
        out[..., c] = torch.where(inside, (v - mean) / std, torch.zeros_like(v))
    return out


def flops_per_image(cfg: ModelConfig, h: int = 423, w: int = 511, proposals: int = 1000, dets: int = 4) -> float:
    """Algorithmic FLOPs (2 x MAC) of one image's forward, re-derived from the
    layer list (convolutions, FCs, deconvs; excludes norm/pool/NMS)."""
    d = cfg.size_divisibility
    Hp, Wp = (h + d - 1) // d * d, (w + d - 1) // d * d
    mac = 0
    H, W = Hp // 2, Wp // 2
    mac += H * W * 64 * 3 * 49
    H, W = H // 2, W // 2
    for name, nb, cin, bott, cout, stride in resnet_stage_specs(cfg):
        for b in range(nb):
            s = stride if b == 0 else 1
            ci = cin if b == 0 else cout
            Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
            if b == 0:
                mac += Ho * Wo * cout * ci
            mac += Ho * Wo * bott * ci + Ho * Wo * bott * bott * 9 + Ho * Wo * cout * bott
            H, W = Ho, Wo
    C = cfg.fpn_out_channels
    sizes = {2: (Hp // 4, Wp // 4), 3: (Hp // 8, Wp // 8), 4: (Hp // 16, Wp // 16), 5: (Hp // 32, Wp // 32)}
    cins = {2: 256, 3: 512, 4: 1024, 5: 2048}
    for l, (h_, w_) in sizes.items():
        mac += h_ * w_ * C * cins[l] + h_ * w_ * C * C * 9
    sizes[6] = ((sizes[5][0] + 1) // 2, (sizes[5][1] + 1) // 2)
    A = len(cfg.aspect_ratios)
    for l in range(2, 7):
        h_, w_ = sizes[l]
        mac += h_ * w_ * C * C * 9 + h_ * w_ * C * 5 * A
    R = cfg.box_pooler_resolution
    mac += proposals * (C * R * R * cfg.box_fc_dim + cfg.box_fc_dim * cfg.box_fc_dim + cfg.box_fc_dim * 6)
    M = cfg.mask_pooler_resolution
    mac += dets * (cfg.mask_num_conv * M * M * C * C * 9 + M * M * C * 4 * C + 4 * M * M * C)
    Pk = cfg.keypoint_pooler_resolution
    cin = C
    for dim in cfg.keypoint_conv_dims:
        mac += dets * Pk * Pk * dim * cin * 9
        cin = dim
    mac += dets * Pk * Pk * cfg.num_keypoints * 16 * cin  # ConvTranspose2d(4, s2) as a GEMM
    return 2.0 * mac
