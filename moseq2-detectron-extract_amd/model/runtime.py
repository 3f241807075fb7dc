"""MI355X-native Mask/Keypoint R-CNN inference runtime.

Weights are packed once (FrozenBN folded into the conv, OIHW -> OHWI, the box
head's fc1 columns permuted to the NHWC pooled layout, the mask deconv turned
into a 1x1 GEMM with a pixel-shuffle epilogue) and every layer is one launch
of a hand-written gfx950 kernel through the C ABI (include/mdx.h).  The whole
forward is launched on the current HIP stream with no host synchronisation
(fixed shapes: 1000 proposals/image, D detections/image, counts kept on the
device), so it can be captured into a HIP graph and replayed.

The layer sequence follows Detectron2's GeneralizedRCNN as configured by the
reference (M/model/config.py:21-94); see oracle/model_ref.py for the CPU
restatement used as the parity checker.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from .._lib import MdxError, call
from .config import ModelConfig
from .weights import resnet_stage_specs

# fp32 partial-sum workspace for split-K launches of the small-grid layers
# (res5, ROI heads); the library only splits when the partials fit
SPLITK_WS_BYTES = 64 << 20

_DT = {"fp32": 0, "fp16": 1}


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@dataclass
class Conv:
    w: torch.Tensor            # [Cout][K] packed
    b: Optional[torch.Tensor]  # f32 [Cout]
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    kalg: int = 0              # algorithmic K (MACs per output) when the packing pads it; 0 = k*k*cin


class MaskRCNN:
    """Packed weights + forward of the reference model on one GPU."""

    def __init__(self, cfg: ModelConfig, state_dict: Dict[str, torch.Tensor], device="cuda", dtype: str = "fp16"):
        if not torch.cuda.is_available():
            raise MdxError("MaskRCNN needs an AMD GPU; there is no CPU fallback")
        if dtype not in _DT:
            raise ValueError("dtype must be 'fp16' or 'fp32'")
        if cfg.num_classes != 1:
            raise NotImplementedError("the extraction model has one class (ROI_HEADS.NUM_CLASSES=1)")
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tdt = torch.float16 if dtype == "fp16" else torch.float32
        self.dcode = _DT[dtype]
        self.vec = 8 if dtype == "fp16" else 4
        sd = {k: v.detach().to("cpu", torch.float32) for k, v in state_dict.items()}
        self._pack(sd)
        self._bufs = None
        self._buf_key = None

    # ------------------------------------------------------------ packing
    def _dev(self, t, dt=None):
        return t.to(self.device, dt or self.tdt).contiguous()

    def _conv(self, w, b, stride, pad, cin_pad=None) -> Conv:
        cout, cin, kh, kw = w.shape
        wp = w.permute(0, 2, 3, 1)  # OHWI
        if cin_pad and cin_pad > cin:
            wp = torch.nn.functional.pad(wp, (0, cin_pad - cin))
            cin = cin_pad
        return Conv(self._dev(wp.reshape(cout, -1)), None if b is None else self._dev(b, torch.float32),
                    cin, cout, kh, stride, pad)

    def _conv_bn(self, sd, p, stride, pad, cin_pad=None) -> Conv:
        w = sd[p + ".weight"]
        scale = sd[p + ".norm.weight"] * (sd[p + ".norm.running_var"] + 1e-5).rsqrt()
        bias = sd[p + ".norm.bias"] - sd[p + ".norm.running_mean"] * scale
        return self._conv(w * scale.view(-1, 1, 1, 1), bias, stride, pad, cin_pad)

    def _stem_s2d(self, sd, p) -> Conv:
        """7x7/s2/p3 stem as a 4x4/s1/p1 conv over the space-to-depth input
        (mdx_preprocess_s2d): W'[o][ty][tx][(2dy+dx)*4+c] = W[o][c][2ty+dy][2tx+dx]."""
        w = sd[p + ".weight"]
        scale = sd[p + ".norm.weight"] * (sd[p + ".norm.running_var"] + 1e-5).rsqrt()
        bias = sd[p + ".norm.bias"] - sd[p + ".norm.running_mean"] * scale
        w = w * scale.view(-1, 1, 1, 1)
        cout, cin, kh, kw = w.shape
        assert kh == 7 and kw == 7 and cin <= 4
        w8 = torch.zeros(cout, 4, 8, 8)
        w8[:, :cin, :7, :7] = w
        # [o][c][ty][dy][tx][dx] -> [o][ty][tx][dy][dx][c]
        wp = w8.view(cout, 4, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(cout, 4 * 4 * 16)
        return Conv(self._dev(wp), self._dev(bias, torch.float32), 16, cout, 4, 1, 1, kalg=49 * cin)

    def _pack(self, sd):
        cfg = self.cfg
        bu = "backbone.bottom_up"
        self.stem = self._stem_s2d(sd, f"{bu}.stem.conv1")
        self.blocks: List[dict] = []
        for name, nb, _cin, _bott, _cout, stride in resnet_stage_specs(cfg):
            for b in range(nb):
                p = f"{bu}.{name}.{b}"
                s = stride if b == 0 else 1
                s1, s3 = (s, 1) if cfg.stride_in_1x1 else (1, s)
                blk = {"stage": name,
                       "shortcut": self._conv_bn(sd, f"{p}.shortcut", s, 0) if f"{p}.shortcut.weight" in sd else None,
                       "conv1": self._conv_bn(sd, f"{p}.conv1", s1, 0),
                       "conv2": self._conv_bn(sd, f"{p}.conv2", s3, 1),
                       "conv3": self._conv_bn(sd, f"{p}.conv3", 1, 0)}
                self.blocks.append(blk)
        self.fpn = {}
        gn = cfg.fpn_norm == "GN"
        for l in cfg.fpn_levels:
            for kind, pad in (("lateral", 0), ("output", 1)):
                p = f"backbone.fpn_{kind}{l}"
                c = self._conv(sd[p + ".weight"], sd.get(p + ".bias"), 1, pad)
                g = (self._dev(sd[p + ".norm.weight"], torch.float32), self._dev(sd[p + ".norm.bias"], torch.float32)) \
                    if gn else None
                self.fpn[(kind, l)] = (c, g)
        p = "proposal_generator.rpn_head"
        self.rpn_conv = self._conv(sd[p + ".conv.weight"], sd[p + ".conv.bias"], 1, 1)
        hw = torch.cat([sd[p + ".objectness_logits.weight"], sd[p + ".anchor_deltas.weight"]], 0)
        hb = torch.cat([sd[p + ".objectness_logits.bias"], sd[p + ".anchor_deltas.bias"]], 0)
        self.rpn_head = self._conv(hw, hb, 1, 0)
        self.A = len(cfg.aspect_ratios)
        # anchors: cell anchors computed in double, stored float32 (DefaultAnchorGenerator)
        cells = []
        for size in cfg.anchor_sizes:
            for ar in cfg.aspect_ratios:
                area = float(size) ** 2.0
                w = math.sqrt(area / ar)
                h = ar * w
                cells.append([-w / 2.0, -h / 2.0, w / 2.0, h / 2.0])
        self.cell_anchors = np.ascontiguousarray(np.array(cells, np.float32))
        # box head
        R = cfg.box_pooler_resolution
        C = cfg.fpn_out_channels
        w1 = sd["roi_heads.box_head.fc1.weight"].view(-1, C, R, R).permute(0, 2, 3, 1).reshape(-1, R * R * C)
        self.fc = [self._conv(w1[:, :, None, None], sd["roi_heads.box_head.fc1.bias"], 1, 0)]
        for i in range(1, cfg.box_num_fc):
            self.fc.append(self._conv(sd[f"roi_heads.box_head.fc{i + 1}.weight"][:, :, None, None],
                                      sd[f"roi_heads.box_head.fc{i + 1}.bias"], 1, 0))
        pw = torch.cat([sd["roi_heads.box_predictor.cls_score.weight"], sd["roi_heads.box_predictor.bbox_pred.weight"]])
        pb = torch.cat([sd["roi_heads.box_predictor.cls_score.bias"], sd["roi_heads.box_predictor.bbox_pred.bias"]])
        self.box_pred = self._conv(pw[:, :, None, None], pb, 1, 0)
        # mask head
        if cfg.mask_on:
            self.mask_convs = [self._conv(sd[f"roi_heads.mask_head.mask_fcn{i + 1}.weight"],
                                          sd[f"roi_heads.mask_head.mask_fcn{i + 1}.bias"], 1, 1)
                               for i in range(cfg.mask_num_conv)]
            dw = sd["roi_heads.mask_head.deconv.weight"]  # (Cin, Co, 2, 2)
            cin, co = dw.shape[0], dw.shape[1]
            dwp = dw.permute(2, 3, 1, 0).reshape(4 * co, cin)  # n' = (dy*2+dx)*Co + co
            self.mask_deconv = Conv(self._dev(dwp), self._dev(sd["roi_heads.mask_head.deconv.bias"].repeat(4),
                                                              torch.float32), cin, 4 * co, 1, 1, 0)
            self.mask_pred = self._conv(sd["roi_heads.mask_head.predictor.weight"],
                                        sd["roi_heads.mask_head.predictor.bias"], 1, 0)
        if cfg.keypoint_on:
            self.kp_convs = [self._conv(sd[f"roi_heads.keypoint_head.conv_fcn{i + 1}.weight"],
                                        sd[f"roi_heads.keypoint_head.conv_fcn{i + 1}.bias"], 1, 1)
                             for i in range(len(cfg.keypoint_conv_dims))]
            kw_ = sd["roi_heads.keypoint_head.score_lowres.weight"]  # (Cin, K, 4, 4)
            cin, kk = kw_.shape[0], kw_.shape[1]
            # ConvTranspose2d(k4,s2,p1) = GEMM to (K*16) columns + col2im
            self.kp_deconv = Conv(self._dev(kw_.permute(1, 2, 3, 0).reshape(kk * 16, cin)), None, cin, kk * 16, 1, 1,
                                  0)
            self.kp_deconv_b = self._dev(sd["roi_heads.keypoint_head.score_lowres.bias"], torch.float32)
        self.pixel_mean = np.ascontiguousarray(np.asarray(sd["pixel_mean"].reshape(-1), np.float32))
        self.pixel_std = np.ascontiguousarray(np.asarray(sd["pixel_std"].reshape(-1), np.float32))
        # per-stream workspaces: forwards of different batches may run
        # concurrently on different HIP streams (pipeline.OverlappedExtractor)
        self._ws = {}
        self._keep = {}

    # ------------------------------------------------------------ layers
    def workspace(self, name: str, nbytes: int) -> torch.Tensor:
        """Scratch buffer `name` of >= nbytes owned by the current stream (work
        on one stream is ordered, so reuse within it is safe)."""
        key = (torch.cuda.current_stream().cuda_stream, name)
        t = self._ws.get(key)
        if t is None or t.numel() * 4 < nbytes:
            t = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=self.device)
            self._ws[key] = t
        return t

    def conv(self, x, N, H, W, c: Conv, relu, out=None, residual=None, out_f32=False, out_mode=0):
        OH = (H + 2 * c.pad - c.k) // c.stride + 1
        OW = (W + 2 * c.pad - c.k) // c.stride + 1
        odt = torch.float32 if out_f32 else self.tdt
        if out is None:
            if out_mode == 1:
                out = torch.empty((N, 2 * OH, 2 * OW, c.cout // 4), dtype=odt, device=self.device)
            else:
                out = torch.empty((N, OH, OW, c.cout), dtype=odt, device=self.device)
        ws = self.workspace("splitk", SPLITK_WS_BYTES)
        call("mdx_conv2d_splitk", _p(x), N, H, W, c.cin, _p(c.w), _p(c.b), c.cout, c.k, c.k, c.stride, c.pad,
             _p(residual), int(relu), out_mode, self.dcode, 0 if out_f32 else self.dcode, _p(out), 0,
             _p(ws), SPLITK_WS_BYTES, _stream())
        return out, OH, OW

    def groupnorm(self, x, N, H, W, C, g, up=None, fuse=0):
        out = torch.empty_like(x)
        ws = self.workspace("gn", call("mdx_groupnorm_workspace_bytes", N, H, W, self.cfg.gn_groups))
        call("mdx_groupnorm", _p(x), N, H, W, C, self.cfg.gn_groups, float(self.cfg.gn_eps), _p(g[0]), _p(g[1]),
             _p(up), fuse, self.dcode, _p(out), _p(ws), _stream())
        return out

    # ------------------------------------------------------------ forward
    def padded_size(self, h, w):
        d = self.cfg.size_divisibility
        return (h + d - 1) // d * d, (w + d - 1) // d * d

    def backbone(self, x, B, Hp, Wp):
        cfg = self.cfg
        y, H, W = self.conv(x, B, Hp // 2 + 1, Wp // 2 + 1, self.stem, relu=True)
        pooled = torch.empty((B, (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1, self.stem.cout), dtype=self.tdt,
                             device=self.device)
        call("mdx_maxpool2d", _p(y), B, H, W, self.stem.cout, 3, 2, 1, self.dcode, _p(pooled), _stream())
        x, H, W = pooled, pooled.shape[1], pooled.shape[2]
        res = {}
        for blk in self.blocks:
            if blk["shortcut"] is not None:
                sc, _, _ = self.conv(x, B, H, W, blk["shortcut"], relu=False)
            else:
                sc = x
            t, H1, W1 = self.conv(x, B, H, W, blk["conv1"], relu=True)
            t, H2, W2 = self.conv(t, B, H1, W1, blk["conv2"], relu=True)
            x, H, W = self.conv(t, B, H2, W2, blk["conv3"], relu=True, residual=sc)
            res[blk["stage"]] = (x, H, W)
        # FPN (coarse -> fine), GN, avg fuse
        lv = cfg.fpn_levels
        names = ["res2", "res3", "res4", "res5"]
        C = cfg.fpn_out_channels
        fuse = 2 if cfg.fpn_fuse_type == "avg" else 1
        feats = {}
        prev = None
        for idx in range(len(names) - 1, -1, -1):
            r, H, W = res[names[idx]]
            lc, lg = self.fpn[("lateral", lv[idx])]
            lat, _, _ = self.conv(r, B, H, W, lc, relu=False)
            if lg is not None:
                prev = self.groupnorm(lat, B, H, W, C, lg, up=prev, fuse=0 if prev is None else fuse)
            else:
                raise NotImplementedError("FPN without GN")
            oc, og = self.fpn[("output", lv[idx])]
            o, _, _ = self.conv(prev, B, H, W, oc, relu=False)
            if og is not None:
                o = self.groupnorm(o, B, H, W, C, og)
            feats[lv[idx]] = (o, H, W)
        p5, H5, W5 = feats[lv[-1]]
        H6, W6 = (H5 - 1) // 2 + 1, (W5 - 1) // 2 + 1
        p6 = torch.empty((B, H6, W6, C), dtype=self.tdt, device=self.device)
        call("mdx_maxpool2d", _p(p5), B, H5, W5, C, 1, 2, 0, self.dcode, _p(p6), _stream())
        feats[lv[-1] + 1] = (p6, H6, W6)
        return res, feats

    def rpn(self, feats, B, h, w):
        cfg = self.cfg
        heads, hs, ws, strides = [], [], [], []
        for i, l in enumerate(range(2, 7)):
            f, H, W = feats[l]
            t, _, _ = self.conv(f, B, H, W, self.rpn_conv, relu=True)
            hd, _, _ = self.conv(t, B, H, W, self.rpn_head, relu=False, out_f32=True)
            heads.append(hd); hs.append(H); ws.append(W); strides.append(2 ** l)
        L = len(heads)
        post = cfg.rpn_post_nms_topk_test
        boxes = torch.empty((B, post, 4), dtype=torch.float32, device=self.device)
        scores = torch.empty((B, post), dtype=torch.float32, device=self.device)
        counts = torch.empty((B,), dtype=torch.int32, device=self.device)
        wsb = call("mdx_rpn_workspace_bytes", B, L, cfg.rpn_pre_nms_topk_test)
        ws_ = torch.empty(wsb, dtype=torch.uint8, device=self.device)
        ptrs = (ctypes.c_void_p * L)(*[h_.data_ptr() for h_ in heads])
        ia = lambda v: (ctypes.c_int * len(v))(*v)  # noqa: E731
        call("mdx_rpn_proposals", ptrs, ia(hs), ia(ws), ia(strides), L, B, self.A,
             self.cell_anchors.ctypes.data_as(ctypes.c_void_p), float(cfg.anchor_offset), h, w,
             cfg.rpn_pre_nms_topk_test, post, float(cfg.rpn_nms_thresh), float(cfg.rpn_min_box_size),
             float(cfg.bbox_reg_clamp), _p(boxes), _p(scores), _p(counts), _p(ws_), _stream())
        self._keep[torch.cuda.current_stream().cuda_stream] = (heads, ws_)  # alive until the stream consumes them
        return boxes, scores, counts

    def roi_align(self, feats, rois, counts, per_image, P):
        cfg = self.cfg
        lv = cfg.fpn_levels
        C = cfg.fpn_out_channels
        R = rois.shape[0] * rois.shape[1] if rois.dim() == 3 else rois.shape[0]
        out = torch.empty((R, P, P, C), dtype=self.tdt, device=self.device)
        L = len(lv)
        ptrs = (ctypes.c_void_p * L)(*[feats[l][0].data_ptr() for l in lv])
        fh = (ctypes.c_int * L)(*[feats[l][1] for l in lv])
        fw = (ctypes.c_int * L)(*[feats[l][2] for l in lv])
        sc = (ctypes.c_float * L)(*[1.0 / 2 ** l for l in lv])
        call("mdx_roi_align", ptrs, fh, fw, sc, L, lv[0], C, _p(rois), _p(counts), R, per_image, P,
             cfg.pooler_sampling_ratio, int(cfg.pooler_aligned), float(cfg.canonical_box_size),
             float(cfg.canonical_level), self.dcode, _p(out), _stream())
        return out

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
        Hp, Wp = self.padded_size(h, w)
        lut = np.arange(256, dtype=np.uint8) if lut is None else np.ascontiguousarray(lut, np.uint8)
        x = torch.empty((B, Hp // 2 + 1, Wp // 2 + 1, 16), dtype=self.tdt, device=self.device)
        C = 3 if cfg.input_format == "RGB" else 1
        call("mdx_preprocess_s2d", _p(frames), B, h, w, lut.ctypes.data_as(ctypes.c_void_p),
             self.pixel_mean.ctypes.data_as(ctypes.c_void_p), self.pixel_std.ctypes.data_as(ctypes.c_void_p),
             C, Hp, Wp, self.dcode, _p(x), _stream())
        inter = {"input": s2d_to_nhwc(x, Hp, Wp)} if intermediates else None
        res, feats = self.backbone(x, B, Hp, Wp)
        if intermediates:
            inter.update({k: v[0] for k, v in res.items()})
            inter.update({f"p{k}": v[0] for k, v in feats.items()})
        props, pscores, pcount = self.rpn(feats, B, h, w)
        if intermediates:
            inter.update(proposals=props, proposal_scores=pscores, proposal_count=pcount)
        Rp = props.shape[1]
        P = cfg.box_pooler_resolution
        pooled = self.roi_align(feats, props, pcount, Rp, P)
        y = pooled.view(B * Rp, 1, 1, -1)
        for fc in self.fc:
            y, _, _ = self.conv(y, B * Rp, 1, 1, fc, relu=True)
        pred, _, _ = self.conv(y, B * Rp, 1, 1, self.box_pred, relu=False, out_f32=True)
        if intermediates:
            inter.update(box_pooled=pooled, box_pred=pred)
        D = cfg.detections_per_image
        det_boxes = torch.empty((B, D, 4), dtype=torch.float32, device=self.device)
        det_scores = torch.empty((B, D), dtype=torch.float32, device=self.device)
        det_classes = torch.empty((B, D), dtype=torch.int64, device=self.device)
        ndet = torch.empty((B,), dtype=torch.int32, device=self.device)
        rw = np.ascontiguousarray(np.asarray(cfg.box_reg_weights, np.float32))
        call("mdx_box_postprocess", _p(pred), pred.shape[-1], _p(props), _p(pcount), B, Rp, D,
             float(cfg.score_thresh_test), float(cfg.nms_thresh_test), h, w, rw.ctypes.data_as(ctypes.c_void_p),
             float(cfg.bbox_reg_clamp), _p(det_boxes), _p(det_scores), _p(det_classes), _p(ndet), _stream())
        out = {"boxes": det_boxes, "scores": det_scores, "classes": det_classes, "ndet": ndet}
        R2 = B * D
        if cfg.mask_on:
            M = cfg.mask_pooler_resolution
            t = self.roi_align(feats, det_boxes, ndet, D, M)
            for c in self.mask_convs:
                t, _, _ = self.conv(t, R2, M, M, c, relu=True)
            t, _, _ = self.conv(t, R2, M, M, self.mask_deconv, relu=True, out_mode=1)
            logits, _, _ = self.conv(t, R2, 2 * M, 2 * M, self.mask_pred, relu=False, out_f32=True)
            plane = (h * w + 15) // 16 * 16  # 16-B aligned planes for the selection kernel
            mbuf = torch.empty((B, D, plane), dtype=torch.uint8, device=self.device)
            call("mdx_paste_masks", _p(logits), _p(det_boxes), _p(ndet), B, D, 2 * M, h, w, plane,
                 float(cfg.mask_threshold), _p(mbuf), _stream())
            out["masks"] = torch.as_strided(mbuf, (B, D, h, w), (D * plane, plane, w, 1))
            out["mask_planes"] = (mbuf, plane)
            if intermediates:
                inter["mask_logits"] = logits
        if cfg.keypoint_on:
            Pk = cfg.keypoint_pooler_resolution
            t = self.roi_align(feats, det_boxes, ndet, D, Pk)
            for c in self.kp_convs:
                t, _, _ = self.conv(t, R2, Pk, Pk, c, relu=True)
            K = cfg.num_keypoints
            y, _, _ = self.conv(t, R2, Pk, Pk, self.kp_deconv, relu=False, out_f32=True)
            low = torch.empty((R2, K, 2 * Pk, 2 * Pk), dtype=torch.float32, device=self.device)
            call("mdx_deconv_col2im", _p(y), _p(self.kp_deconv_b), R2, Pk, Pk, K, _p(low), _stream())
            hm = torch.empty((R2, K, 4 * Pk, 4 * Pk), dtype=torch.float32, device=self.device)
            call("mdx_upsample_bilinear2x", _p(low), R2 * K, 2 * Pk, 2 * Pk, _p(hm), _stream())
            kps = torch.empty((B, D, K, 3), dtype=torch.float32, device=self.device)
            call("mdx_heatmaps_to_keypoints", _p(hm), _p(det_boxes), _p(ndet), B, D, K, 4 * Pk, _p(kps), _stream())
            out["keypoints"] = kps
            out["keypoint_heatmaps"] = hm.view(B, D, K, 4 * Pk, 4 * Pk)
        if intermediates:
            out["intermediates"] = inter
        return out


def s2d_to_nhwc(x: torch.Tensor, Hp: int, Wp: int) -> torch.Tensor:
    """(B, Hp/2+1, Wp/2+1, 16) space-to-depth input -> (B, Hp, Wp, 4) NHWC."""
    B = x.shape[0]
    t = x.view(B, Hp // 2 + 1, Wp // 2 + 1, 2, 2, 4).permute(0, 1, 3, 2, 4, 5)
    t = t.reshape(B, Hp + 2, Wp + 2, 4)
    return t[:, 1:Hp + 1, 1:Wp + 1].contiguous()


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
