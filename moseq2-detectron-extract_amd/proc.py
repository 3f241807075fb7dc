"""Frame ops of the extraction hot path, MI355X-native.

Same names, argument meaning and error behaviour as the reference's
``moseq2_detectron_extract/proc/proc.py`` (M/proc/proc.py) so callers drop in:

=========================  =============================  ===========================
this module                reference                      kernel (csrc/)
=========================  =============================  ===========================
prep_raw_frames            M/proc/proc.py:129-172         k_prep + k_inpaint
find_invalid_pixels        M/proc/proc.py:175-186         (k_prep's invalid output)
fill_invalid_pixels        M/proc/proc.py:189-210         k_inpaint
scale_raw_frames           M/proc/proc.py:214-234         k_scale (256-entry LUT)
clean_frames               M/proc/proc.py:480-515         k_clean (fused LDS tiles)
get_frame_features         M/proc/proc.py:237-302,518-549 k_moments
crop_and_rotate_frame(s)   M/proc/proc.py:305-340         k_crop
get_bbox / apply_roi       M/proc/roi.py:215-254          (host bbox; crop fused in k_prep)
=========================  =============================  ===========================

Inputs may be numpy arrays (copied to the current GPU, result copied back, as
the reference returns numpy) or CUDA/HIP ``torch.Tensor`` s (results stay in
HBM).  There is no CPU fallback: without a GPU every op raises MdxError.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from ._lib import MdxError, call

_U8 = "uint8"


# ---------------------------------------------------------------------------
# plumbing
# ---------------------------------------------------------------------------
def _torch():
    import torch
    if not torch.cuda.is_available():
        raise MdxError("moseq2_detectron_extract_amd needs an AMD GPU (torch.cuda.is_available() is False); "
                       "there is no CPU fallback")
    return torch


def _stream():
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _to_dev(x, dtype):
    """numpy / torch -> contiguous device tensor of `dtype` (torch dtype)."""
    torch = _torch()
    if isinstance(x, torch.Tensor):
        t = x
        if not t.is_cuda:
            t = t.to("cuda", non_blocking=False)
    else:
        t = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def _is_np(x):
    return isinstance(x, np.ndarray)


def _ret(t, as_numpy):
    return t.cpu().numpy() if as_numpy else t


def get_bbox(roi) -> Optional[np.ndarray]:
    """((y_min, x_min), (y_max, x_max)) of roi > 0, or None (M/proc/roi.py:239-254)."""
    r = roi.detach().cpu().numpy() if hasattr(roi, "detach") else np.asarray(roi)
    y, x = np.where(r > 0)
    if len(y) == 0:
        return None
    return np.array([[y.min(), x.min()], [y.max(), x.max()]])


def ellipse_strel(ksize=(9, 9)) -> np.ndarray:
    """cv2.getStructuringElement(cv2.MORPH_ELLIPSE, ksize) (OpenCV's formula)."""
    w, h = ksize
    r, c = h // 2, w // 2
    inv_r2 = 1.0 / (r * r) if r else 0.0
    k = np.zeros((h, w), np.uint8)
    for i in range(h):
        dy = i - r
        if abs(dy) <= r:
            dx = int(np.rint(c * np.sqrt((r * r - dy * dy) * inv_r2)))
            k[i, max(c - dx, 0):min(c + dx + 1, w)] = 1
    return k


def rect_strel(ksize=(5, 5)) -> np.ndarray:
    return np.ones((ksize[1], ksize[0]), np.uint8)


ELLIPSE9 = ellipse_strel((9, 9))
RECT5 = rect_strel((5, 5))


# ---------------------------------------------------------------------------
# prep
# ---------------------------------------------------------------------------
class FramePrep:
    """Session-resident state of prep_raw_frames: background (float64) and ROI
    live in HBM once; each call is one fused kernel (+ inpaint)."""

    def __init__(self, bground_im=None, roi=None, vmin=None, vmax=None, fix_invalid_pixels=True, frame_shape=None):
        torch = _torch()
        self.bg = None if bground_im is None else _to_dev(bground_im, torch.float64)
        self.roi = None
        self.bbox = None
        if roi is not None:
            self.roi = _to_dev((roi.detach().cpu().numpy() if hasattr(roi, "detach") else np.asarray(roi)) > 0,
                               torch.uint8)
            self.bbox = get_bbox(roi)
        self.vmin, self.vmax = vmin, vmax
        self.fix_invalid_pixels = fix_invalid_pixels
        self._ws = None
        self._errors = None  # this prep's device count of unconverged inpaint frames (inpaint_errors)

    def inpaint_errors(self) -> int:
        """Frames of THIS prep's calls whose inpaint labelling did not
        converge (left un-inpainted; mdx_inpaint_ns_counted).  Synchronises
        the current stream."""
        return 0 if self._errors is None else int(self._errors.item())

    def crop(self, H, W):
        if self.bbox is None:
            return 0, H, 0, W
        b = self.bbox
        return int(b[0, 0]), int(b[1, 0]), int(b[0, 1]), int(b[1, 1])

    def __call__(self, frames, out=None, invalid_out=None, return_invalid=False):
        torch = _torch()
        as_np = _is_np(frames)
        raw = _to_dev(frames, torch.int16)
        if raw.dim() != 3:
            raise ValueError(f"frames must be (nframes, height, width); got {tuple(raw.shape)}")
        n, H, W = raw.shape
        y0, y1, x0, x1 = self.crop(H, W)
        oh, ow = y1 - y0, x1 - x0
        if out is None:
            out = torch.empty((n, oh, ow), dtype=torch.uint8, device=raw.device)
        inv = None
        if return_invalid:
            inv = invalid_out if invalid_out is not None else torch.empty_like(out)
        flags = (1 if self.vmin is not None else 0) | (2 if self.vmax is not None else 0)
        args = (_ptr(raw), n, H, W, _ptr(self.bg), _ptr(self.roi), y0, y1, x0, x1, flags, float(self.vmin or 0.0),
                float(self.vmax or 0.0), _ptr(out), _ptr(inv))
        if self.fix_invalid_pixels and n > 0 and oh > 0 and ow > 0:
            # one call: the invalid pixels go straight to the inpaint
            # workspace as bit images (mdx_prep_inpaint)
            ws = _inpaint_workspace(self, n, oh, ow, raw.device)
            call("mdx_prep_inpaint", *args, 3, _ptr(ws), _ptr(_error_counter(self, raw.device)), _stream())
        else:
            call("mdx_prep_frames", *args, _stream())
        if return_invalid:
            return _ret(out, as_np), _ret(inv, as_np)
        return _ret(out, as_np)


def prep_raw_frames(frames, bground_im=None, roi=None, vmin=None, vmax=None, dtype=_U8,
                    fix_invalid_pixels=True):
    """Background-subtract, ROI-mask/crop, clamp, cast to uint8, inpaint invalid
    (raw == 0) pixels.  Reference: M/proc/proc.py:129-172."""
    if np.dtype(dtype) != np.uint8:
        raise NotImplementedError("prep_raw_frames: only dtype='uint8' (the extract path's) is implemented")
    return FramePrep(bground_im, roi, vmin, vmax, fix_invalid_pixels)(frames)


def find_invalid_pixels(frames):
    """Mask of Kinect-invalid (== 0) pixels, uint8 (M/proc/proc.py:175-186)."""
    prep = FramePrep(None, None, None, None, fix_invalid_pixels=False)
    _, inv = prep(frames, return_invalid=True)
    return inv


def _inpaint_workspace(owner, n, H, W, device):
    """The owner's inpaint workspace for n frames of H x W (a fresh one if no
    owner): sparse per-frame slots, set up once per frame shape; each call
    leaves it ready for the next (mdx_inpaint_workspace_init)."""
    torch = _torch()
    nbytes = call("mdx_inpaint_workspace_bytes", n, H, W)
    ws = getattr(owner, "_ws", None) if owner is not None else None
    if ws is None or ws.numel() < nbytes or getattr(owner, "_ws_shape", None) != (H, W):
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        call("mdx_inpaint_workspace_init", _ptr(ws), ws.numel(), H, W, _stream())
        if owner is not None:
            owner._ws, owner._ws_shape = ws, (H, W)
    return ws


def _error_counter(owner, device):
    """The owner's own device count of unconverged inpaint frames."""
    if getattr(owner, "_errors", None) is None:
        owner._errors = _torch().zeros((1,), dtype=_torch().int32, device=device)
    return owner._errors


def fill_invalid_pixels(frames, invalid_mask, _workspace_owner=None):
    """In-place NS inpaint of every frame (cv2.inpaint(f, m, 3, INPAINT_NS)),
    M/proc/proc.py:189-210.  Device tensors are filled in place; numpy input
    returns a filled copy."""
    torch = _torch()
    as_np = _is_np(frames)
    f = _to_dev(frames, torch.uint8) if as_np or not frames.is_cuda else frames
    if f.dtype != torch.uint8:
        raise NotImplementedError("fill_invalid_pixels: uint8 frames only")
    m = _to_dev(invalid_mask, torch.uint8)
    if tuple(m.shape) != tuple(f.shape):
        raise AssertionError("frames and invalid_mask shapes differ")
    n, H, W = f.shape
    if n == 0:
        return _ret(f, as_np)
    ws = _inpaint_workspace(_workspace_owner, n, H, W, f.device)
    err = _error_counter(_workspace_owner, f.device) if _workspace_owner is not None else None
    call("mdx_inpaint_ns_counted", _ptr(f), _ptr(m), n, H, W, 3, _ptr(ws), _ptr(err), _stream())
    return _ret(f, as_np)


# ---------------------------------------------------------------------------
# scale
# ---------------------------------------------------------------------------
def scale_lut(vmin, vmax) -> np.ndarray:
    lut = np.empty(256, np.uint8)
    int_vmin = isinstance(vmin, (int, np.integer)) and not isinstance(vmin, bool)
    call("mdx_build_scale_lut", float(vmin), float(vmax), int(int_vmin), lut.ctypes.data_as(ctypes.c_void_p))
    return lut


def scale_raw_frames(frames, vmin, vmax, dtype=_U8):
    """Linear scale to the uint8 range, M/proc/proc.py:214-234 (float64 math
    through a host-built 256-entry table, applied on the GPU)."""
    if np.dtype(dtype) != np.uint8:
        raise NotImplementedError("scale_raw_frames: only dtype='uint8' is implemented")
    torch = _torch()
    as_np = _is_np(frames)
    src = frames if (not as_np and frames.dtype == torch.uint8) else None
    if src is None:
        if as_np and np.asarray(frames).dtype != np.uint8:
            raise NotImplementedError("scale_raw_frames: uint8 frames only (the extract path's input)")
        src = _to_dev(frames, torch.uint8)
    src = src.contiguous()
    out = torch.empty_like(src)
    lut = scale_lut(vmin, vmax)
    call("mdx_scale_frames", _ptr(src), src.numel(), lut.ctypes.data_as(ctypes.c_void_p), _ptr(out), _stream())
    return _ret(out, as_np)


# ---------------------------------------------------------------------------
# clean
# ---------------------------------------------------------------------------
def clean_frames(frames, prefilter_space=(3,), prefilter_time=None, strel_tail=ELLIPSE9, iters_tail=None,
                 frame_dtype=_U8, strel_min=RECT5, iters_min=None, progress_bar=True):
    """Median filter then morphological opening, M/proc/proc.py:480-515."""
    if np.dtype(frame_dtype) != np.uint8:
        raise NotImplementedError("clean_frames: frame_dtype='uint8' only")
    if iters_min is not None and iters_min > 0:
        raise NotImplementedError("clean_frames: iters_min (pre-erosion) is not on the extract path")
    if prefilter_time is not None:
        raise NotImplementedError("clean_frames: prefilter_time (temporal median) is not on the extract path")
    med = 0
    if prefilter_space is not None and np.all(np.array(prefilter_space) > 0):
        ps = list(prefilter_space)
        if ps != [3]:
            raise NotImplementedError(f"clean_frames: prefilter_space={prefilter_space}; only (3,) is implemented")
        med = 3
    iters = int(iters_tail) if iters_tail is not None and iters_tail > 0 else 0
    torch = _torch()
    as_np = _is_np(frames)
    src = _to_dev(frames, torch.uint8)
    n, H, W = src.shape
    out = torch.empty_like(src)
    if med == 0 and iters == 0:
        out.copy_(src)
        return _ret(out, as_np)
    st = np.ascontiguousarray(np.asarray(strel_tail) != 0, np.uint8)
    ws = torch.empty(call("mdx_clean_workspace_bytes", n, H, W), dtype=torch.uint8, device=src.device)
    call("mdx_clean_frames", _ptr(src), n, H, W, med, st.ctypes.data_as(ctypes.c_void_p), st.shape[0], st.shape[1],
         iters, _ptr(out), _ptr(ws), _stream())
    return _ret(out, as_np)


# ---------------------------------------------------------------------------
# moments
# ---------------------------------------------------------------------------
def frame_moments(frames, mask=None, frame_threshold=10.0):
    """Device-resident features: dict of float64 tensors centroid (n,2),
    orientation (n,), axis_length (n,2), area (n,)."""
    torch = _torch()
    src = _to_dev(frames, torch.uint8)
    n, H, W = src.shape
    m = None if mask is None else _to_dev(mask, torch.uint8)
    if m is not None and tuple(m.shape) != (n, H, W):
        raise ValueError("mask shape must match frames")
    cen = torch.empty((n, 2), dtype=torch.float64, device=src.device)
    ori = torch.empty((n,), dtype=torch.float64, device=src.device)
    ax = torch.empty((n, 2), dtype=torch.float64, device=src.device)
    area = torch.empty((n,), dtype=torch.float64, device=src.device)
    ws = torch.empty(max(1, call("mdx_frame_moments_workspace_bytes", n, H, W)), dtype=torch.uint8,
                     device=src.device)  # the bit-packed blob masks (packed over every CU)
    call("mdx_frame_moments_ws", _ptr(src), _ptr(m), n, H, W, float(frame_threshold), _ptr(cen), _ptr(ori), _ptr(ax),
         _ptr(area), _ptr(ws), _stream())
    return {"centroid": cen, "orientation": ori, "axis_length": ax, "area": area}


def get_frame_features(frames, frame_threshold=10, mask=np.array([]), mask_threshold=-30, use_cc=False,
                       progress_bar=True) -> Tuple[dict, object]:
    """Largest-blob moments per frame, M/proc/proc.py:237-302.

    Returns (features, masks) like the reference.  For uint8 frames use_cc is a
    no-op in the reference (frames > mask_threshold is all-true for
    mask_threshold < 0), so it is accepted and ignored under that condition.
    features['contour'] is not materialised (nothing on the extract path
    reads it)."""
    torch = _torch()
    as_np = _is_np(frames)
    has_mask = mask is not None and ((hasattr(mask, "numel") and mask.numel() > 0) or
                                     (not hasattr(mask, "numel") and np.asarray(mask).size > 0))
    if use_cc and not mask_threshold < 0:
        raise NotImplementedError("get_frame_features: use_cc with mask_threshold >= 0 is not implemented")
    feats = frame_moments(frames, mask if has_mask else None, float(frame_threshold))
    if has_mask:
        masks = mask
    else:
        src = _to_dev(frames, torch.uint8)
        masks = (src > frame_threshold).to(torch.uint8)
        masks = masks.cpu().numpy() if as_np else masks
    out = {k: (v.cpu().numpy() if as_np else v) for k, v in feats.items() if k != "area"}
    out["contour"] = []
    return out, masks


# ---------------------------------------------------------------------------
# crop and rotate
# ---------------------------------------------------------------------------
def crop_and_rotate_frames(frames, centers, angles, crop_size=(80, 80), frames2=None, return_window=False):
    """Batched crop_and_rotate_frame for every frame (and frames2 with the same
    centres/angles, e.g. the d2 masks).  Returns uint8 (n, crop_h, crop_w)
    (a tuple with frames2's crops; with return_window, also the int32 (n, 4)
    crop windows (xmin, xmax, ymin, ymax), -1 where the crop is zeros)."""
    torch = _torch()
    as_np = _is_np(frames)
    src0 = _to_dev(frames, torch.uint8)
    n, H, W = src0.shape
    src1 = None if frames2 is None else _to_dev(frames2, torch.uint8)
    c = _to_dev(np.asarray(centers, np.float64) if not hasattr(centers, "dtype") or _is_np(centers) else centers,
                torch.float64).reshape(n, 2).contiguous()
    a = _to_dev(np.asarray(angles, np.float64) if not hasattr(angles, "dtype") or _is_np(angles) else angles,
                torch.float64).reshape(n).contiguous()
    cw, ch = int(crop_size[0]), int(crop_size[1])
    o0 = torch.empty((n, ch, cw), dtype=torch.uint8, device=src0.device)
    o1 = None if src1 is None else torch.empty_like(o0)
    win = torch.empty((n, 4), dtype=torch.int32, device=src0.device) if return_window else None
    call("mdx_crop_rotate", _ptr(src0), _ptr(src1), n, H, W, _ptr(c), _ptr(a), cw, ch, _ptr(o0), _ptr(o1),
         _ptr(win), _stream())
    out = (_ret(o0, as_np),) + (() if src1 is None else (_ret(o1, as_np),)) + \
        (() if win is None else (_ret(win, as_np),))
    return out[0] if len(out) == 1 else out


def crop_and_rotate_frame(frame, center, angle, crop_size=(80, 80)):
    """Single-frame form of the reference (M/proc/proc.py:305-340)."""
    f = frame[None] if not hasattr(frame, "unsqueeze") else frame.unsqueeze(0)
    out = crop_and_rotate_frames(f, np.asarray(center, np.float64).reshape(1, 2),
                                 np.asarray([angle], np.float64), crop_size)
    return out[0]
