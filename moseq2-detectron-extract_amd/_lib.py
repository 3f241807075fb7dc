"""ctypes binding of the in-tree HIP library ``libmdx.so`` (C ABI: include/mdx.h).

There is no CPU fallback: if the library is missing or the device is not a
GPU, every op raises :class:`MdxError`.  ``torch`` is imported before the
library is opened so that ``libmdx.so``'s ``libamdhip64.so.7`` dependency binds
to the HIP runtime PyTorch already loaded (one runtime, shared streams).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MDX_LIB_VARIANT=<name> loads libmdx_<name>.so (an instrumented build, debugging only)
LIB_PATH = os.path.join(_HERE, "libmdx.so" if not os.environ.get("MDX_LIB_VARIANT") else
                        f"libmdx_{os.environ['MDX_LIB_VARIANT']}.so")
_LIB = None


class MdxError(RuntimeError):
    pass


P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F64 = ctypes.c_double
F32 = ctypes.c_float

# name -> (restype, argtypes); mirrors include/mdx.h
SIGNATURES = {
    "mdx_last_error": (ctypes.c_char_p, []),
    "mdx_version": (ctypes.c_char_p, []),
    "mdx_prep_frames": (I32, [P, I64, I32, I32, P, P, I32, I32, I32, I32, I32, F64, F64, P, P, P]),
    "mdx_inpaint_workspace_bytes": (I64, [I64, I32, I32]),
    "mdx_inpaint_workspace_init": (I32, [P, I64, I32, I32, P]),
    "mdx_inpaint_sparse_capacity": (I32, [I32, I32]),
    "mdx_prep_inpaint": (I32, [P, I64, I32, I32, P, P, I32, I32, I32, I32, I32, F64, F64, P, P, I32, P, P, P]),
    "mdx_inpaint_ns": (I32, [P, P, I64, I32, I32, I32, P, P]),
    "mdx_inpaint_errors": (I32, [I32]),
    "mdx_inpaint_ns_counted": (I32, [P, P, I64, I32, I32, I32, P, P, P]),
    "mdx_build_scale_lut": (I32, [F64, F64, I32, P]),
    "mdx_scale_frames": (I32, [P, I64, P, P, P]),
    "mdx_clean_workspace_bytes": (I64, [I64, I32, I32]),
    "mdx_clean_frames": (I32, [P, I64, I32, I32, I32, P, I32, I32, I32, P, P, P]),
    "mdx_clean_set_mode": (I32, [I32]),
    "mdx_frame_moments": (I32, [P, P, I64, I32, I32, F64, P, P, P, P, P]),
    "mdx_frame_moments_workspace_bytes": (I64, [I64, I32, I32]),
    "mdx_frame_moments_ws": (I32, [P, P, I64, I32, I32, F64, P, P, P, P, P, P]),
    "mdx_crop_rotate": (I32, [P, P, I64, I32, I32, P, P, I32, I32, P, P, P, P]),
    "mdx_frame_scalars": (I32, [P, P, I64, I32, I32, F64, F64, P, I32, P, P, P, P, P]),
    "mdx_bground_median": (I32, [P, I64, I32, I32, I32, P, P, P]),
    "mdx_iterative_filter_angles": (I32, [P, I64, I32, F64, I32, P, P]),
    "mdx_flips_from_keypoints": (I32, [P, I64, I32, P, P, P, P, P]),
    "mdx_finalize_angles": (I32, [P, P, P, P, I64, I32, P, P]),
    "mdx_conv2d": (I32, [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, P, I32, I32, I32, I32, P, P]),
    "mdx_winograd_weights": (I32, [P, I32, I32, I32, P]),
    "mdx_winograd_workspace_bytes": (I64, [I32, I32, I32, I32, I32, I32]),
    "mdx_conv3x3_winograd": (I32, [P, I32, I32, I32, I32, P, P, I32, I32, I32, P, P, I64, P]),
    "mdx_conv3x3_winograd_x6": (I32, [P, I32, I32, I32, I32, P, P, P, I32, I32, I32, P, P, I64, P]),
    "mdx_winograd_tile": (I32, [I32, I32, I32]),
    "mdx_x6_plane_bytes": (I64, [I64, I32]),
    "mdx_split_x6": (I32, [P, I64, I32, I64, P, P]),
    "mdx_gemm_x6": (I32, [P, P, P, I32, I32, I32, P, I32, P, P]),
    "mdx_conv2d_last_plan": (I32, [P, P]),
    "mdx_conv2d_workspace_bytes": (I64, [I32, I32, I32, I32, I32, I32, I32, I32, I32]),
    "mdx_conv2d_splitk": (I32, [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, P, I32, I32, I32, I32, P, I32,
                                P, I64, P]),
    "mdx_format_tsv_rows": (I64, [P, P, I32, I64, P, I64]),
    "mdx_conv2d_dual": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, P, P, I32, I32, I32, P, P, I64, P]),
    "mdx_preprocess": (I32, [P, I32, I32, I32, P, P, P, I32, I32, I32, I32, I32, P, P]),
    "mdx_preprocess_s2d": (I32, [P, I32, I32, I32, P, P, P, I32, I32, I32, I32, P, P]),
    "mdx_preprocess_s2d_folded": (I32, [P, I32, I32, I32, P, I32, I32, I32, P, P]),
    "mdx_maxpool2d": (I32, [P, I32, I32, I32, I32, I32, I32, I32, I32, P, P]),
    "mdx_convert": (I32, [P, I64, I32, P, I32, P]),
    "mdx_groupnorm_workspace_bytes": (I64, [I32, I32, I32, I32]),
    "mdx_groupnorm": (I32, [P, I32, I32, I32, I32, I32, F32, P, P, P, I32, I32, P, P, P]),
    "mdx_rpn_workspace_bytes": (I64, [I32, I32, I32]),
    "mdx_rpn_proposals": (I32, [P, P, P, P, I32, I32, I32, P, F32, I32, I32, I32, I32, F32, F32, F32,
                                P, P, P, P, P, P]),
    "mdx_roi_align": (I32, [P, P, P, P, I32, I32, I32, P, P, I32, I32, I32, I32, I32, F32, F32, I32, P, P]),
    "mdx_roi_align_ex": (I32, [P, P, P, P, I32, I32, I32, P, P, I32, I32, I32, I32, I32, F32, F32, I32, P, P, P]),
    "mdx_box_postprocess": (I32, [P, I32, P, P, I32, I32, I32, F32, F32, I32, I32, P, F32, P, P, P, P, P]),
    "mdx_paste_masks": (I32, [P, P, P, I32, I32, I32, I32, I32, I64, F32, P, P]),
    "mdx_deconv_col2im": (I32, [P, P, I32, I32, I32, I32, P, P]),
    "mdx_upsample_bilinear2x": (I32, [P, I32, I32, I32, P, P]),
    "mdx_heatmaps_to_keypoints": (I32, [P, P, P, I32, I32, I32, I32, P, P]),
    "mdx_mask_nms_select": (I32, [P, I64, P, P, P, I32, I32, I32, I32, I32, F32, P, P, P, P, P]),
    "mdx_mask_centers": (I32, [P, I64, P, P, P, I32, I32, I32, I32, P, P]),
    "mdx_gather_planes": (I32, [P, P, P, I64, I32, P]),
    "mdx_instance_tracker_create": (P, [I32]),
    "mdx_instance_tracker_destroy": (I32, [P]),
    "mdx_instance_tracker_select": (I32, [P, P, P, I64, I32, I64, P, P]),
    "mdx_tracking_create": (P, [I32]),
    "mdx_tracking_destroy": (I32, [P]),
    "mdx_tracking_state": (I32, [P, I32, P, P, I64]),
    "mdx_tracking_track": (I32, [P, I64, I32, P, P, P, P, P, P, P, P]),
    "mdx_model_create": (I32, [ctypes.c_char_p, I64, P, I32, P]),
    "mdx_model_destroy": (I32, [P]),
    "mdx_model_reserve": (I32, [P, I32, I32, I32, P]),
    "mdx_model_forward": (I32, [P, P, I32, I32, I32, P, P, P]),
    "mdx_model_tensor_info": (I32, [P, P, ctypes.c_char_p, P, P]),
    "mdx_model_tensor_copy": (I32, [P, P, ctypes.c_char_p, P, I64]),
    "mdx_model_profile": (I32, [P, I32]),
    "mdx_model_debug_fill": (I32, [P, I32, I32, I32, I32, P]),
    "mdx_model_debug_arena": (I32, [P, P, ctypes.c_char_p, P, P, P, I64]),
    "mdx_model_profile_read": (I32, [P, P, I32]),
    "mdx_model_get_policy": (I32, [P, P]),
    "mdx_policy_defaults": (I32, [P]),
    "mdx_policy_get": (I32, [P]),
    "mdx_policy_set": (I32, [P]),
}

# include/mdx.h mdx_policy, field for field (tests/test_abi.py checks the order
# against the header)
POLICY_FIELDS = ("winograd", "winograd_min_cin", "winograd_dma", "winograd_dma_min_wgs", "wino_slice_mb",
                 "fp32_split", "x3_narrow", "x3_single_stage", "large_tiles", "dma128", "dma128_min_tiles",
                 "dma128_interleave", "dma_f32", "pointwise", "single_stage", "direct_epilogue", "narrow_kmax",
                 "head_f32", "stream1x1", "stream1x1_min_m", "stem_fold", "fuse_shortcut", "rpn_sliced", "roi_mode",
                 "roi_xcd_order", "roi_sorted", "f16_pingpong")


class Policy(ctypes.Structure):
    """mdx_policy (include/mdx.h): the kernel-selection policy."""
    _fields_ = [(f, ctypes.c_int) for f in POLICY_FIELDS]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f in POLICY_FIELDS}


def policy() -> dict:
    """The calling thread's policy (mdx_policy_get)."""
    p = Policy()
    call("mdx_policy_get", ctypes.byref(p))
    return p.as_dict()


def policy_defaults() -> dict:
    p = Policy()
    call("mdx_policy_defaults", ctypes.byref(p))
    return p.as_dict()


def set_policy(**fields) -> dict:
    """Change fields of the calling thread's policy (model handles created
    afterwards on this thread capture it); returns the previous policy."""
    old = policy()
    bad = set(fields) - set(POLICY_FIELDS)
    if bad:
        raise KeyError(f"unknown policy field(s): {sorted(bad)}")
    p = Policy(**{**old, **fields})
    call("mdx_policy_set", ctypes.byref(p))
    return old


class policy_scope:
    """with policy_scope(winograd=4): ... -- the thread's policy with these
    fields changed, restored on exit."""

    def __init__(self, **fields):
        self.fields = fields

    def __enter__(self):
        self.old = set_policy(**self.fields)
        return self

    def __exit__(self, *exc):
        p = Policy(**self.old)
        call("mdx_policy_set", ctypes.byref(p))


def knob(field: str, value: int, *more):
    """Set one policy field (and, for the (mode, threshold) pairs, the
    threshold field after it in POLICY_FIELDS) on the calling thread; returns
    the field's previous value."""
    old = policy()
    upd = {field: value}
    if more:
        upd[POLICY_FIELDS[POLICY_FIELDS.index(field) + 1]] = more[0]
    set_policy(**upd)
    return old[field]


def lib():
    """Open (once) and return the library; raises MdxError if unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (binds libamdhip64.so.7 first)
    if not os.path.exists(LIB_PATH):
        raise MdxError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                       "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def call(name: str, *args) -> int:
    L = lib()
    rc = getattr(L, name)(*args)
    if isinstance(rc, int) and rc < 0 and SIGNATURES[name][0] is I32:
        raise MdxError(f"{name} failed ({rc}): {L.mdx_last_error().decode()}")
    return rc
