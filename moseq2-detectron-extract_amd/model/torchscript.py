"""Weights-only import of a TorchScript model archive (``model.ts``).

The reference can load an exported TorchScript model
(``Predictor.from_torchscript``, M/model/predict.py:46-51; exported by
M/model/deploy.py:77-121 as a ScriptableAdapter whose ``model`` attribute is
the Detectron2 GeneralizedRCNN; post-processed by ``outputs_to_instances``,
M/model/util.py:45-62).  The native runtime does not run the archive's
TorchScript graph: it reads the module tree's parameters, buffers and scalar
attributes out of ``<archive>/data.pkl`` with a restricted unpickler that
builds nothing but plain containers and tensors (every ``__torch__.*`` class
becomes an inert attribute record; any other global is refused), and feeds the
Detectron2 state dict into the model handle like a ``model_final.pth``.  No
code from the archive is executed.
"""
from __future__ import annotations

import io
import pickle
import zipfile
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np
import torch

from .config import ModelConfig

_STORAGE_DTYPES = {
    "FloatStorage": torch.float32, "DoubleStorage": torch.float64, "HalfStorage": torch.float16,
    "BFloat16Storage": torch.bfloat16, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8, "BoolStorage": torch.bool,
}


class TSObject:
    """Inert stand-in for a scripted module / class instance: its pickled
    attribute dict, nothing else."""
    qualname = "__torch__"

    def __setstate__(self, state):
        self.attrs = dict(state) if isinstance(state, dict) else {}

    def __getattr__(self, name):
        if name == "attrs":
            return {}
        raise AttributeError(name)


class _StorageType:
    def __init__(self, dtype):
        self.dtype = dtype


class _TypedStorage:
    def __init__(self, flat: torch.Tensor):
        self.flat = flat
        self.dtype = flat.dtype


def _rebuild_tensor_v2(storage, offset, size, stride, requires_grad=False, hooks=None, metadata=None):
    if not isinstance(storage, _TypedStorage):
        raise pickle.UnpicklingError("TorchScript import: tensor without a storage")
    return storage.flat.as_strided(tuple(size), tuple(stride), int(offset)).clone()


def _identity(x, *_a, **_k):
    return x


class _Unpickler(pickle.Unpickler):
    def __init__(self, data: bytes, zf: zipfile.ZipFile, prefix: str):
        super().__init__(io.BytesIO(data))
        self.zf = zf
        self.prefix = prefix
        self.storages: Dict[str, torch.Tensor] = {}
        self.classes: Dict[str, type] = {}

    def find_class(self, module, name):
        if module == "__torch__" or module.startswith("__torch__."):
            qual = f"{module}.{name}"
            if qual not in self.classes:
                self.classes[qual] = type(name, (TSObject,), {"qualname": qual})
            return self.classes[qual]
        if module == "torch" and name in _STORAGE_DTYPES:
            return _StorageType(_STORAGE_DTYPES[name])
        if module == "torch._utils" and name == "_rebuild_tensor_v2":
            return _rebuild_tensor_v2
        if module == "collections" and name == "OrderedDict":
            return OrderedDict
        if module == "torch.jit._pickle" and name in ("build_intlist", "build_tensorlist", "build_doublelist",
                                                       "build_boollist", "restore_type_tag"):
            return _identity
        raise pickle.UnpicklingError(f"TorchScript import: refusing global {module}.{name}")

    def persistent_load(self, pid):
        if not (isinstance(pid, tuple) and len(pid) >= 5 and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"TorchScript import: unexpected persistent id {pid!r}")
        stype, key, _loc, numel = pid[1], str(pid[2]), pid[3], int(pid[4])
        if not isinstance(stype, _StorageType):
            raise pickle.UnpicklingError(f"TorchScript import: storage of unknown type {stype!r}")
        dtype = stype.dtype
        if key not in self.storages:
            raw = self.zf.read(f"{self.prefix}data/{key}")
            itemsize = torch.empty((), dtype=dtype).element_size()
            buf = np.frombuffer(raw, dtype=np.uint8, count=numel * itemsize).copy()
            self.storages[key] = torch.from_numpy(buf).view(dtype)
        return _TypedStorage(self.storages[key])


def read_archive(path: str) -> TSObject:
    """The archive's root module record (restricted unpickling of data.pkl)."""
    with zipfile.ZipFile(path) as zf:
        pk = [n for n in zf.namelist() if n.endswith("/data.pkl") and n.count("/") == 1]
        if not pk:
            raise ValueError(f"{path}: not a TorchScript archive (no <name>/data.pkl)")
        prefix = pk[0][:-len("data.pkl")]
        if (prefix + "byteorder") in zf.namelist() and zf.read(prefix + "byteorder").strip() not in (b"little",):
            raise ValueError(f"{path}: big-endian archive")
        root = _Unpickler(zf.read(pk[0]), zf, prefix).load()
    if not isinstance(root, TSObject):
        raise ValueError(f"{path}: data.pkl does not hold a module")
    return root


def flatten(root: TSObject) -> Tuple["OrderedDict[str, torch.Tensor]", Dict[str, object]]:
    """(tensors by dotted name, scalar attributes by dotted name) of the module tree."""
    tensors: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    scalars: Dict[str, object] = {}

    def walk(obj, pfx):
        for k, v in obj.attrs.items():
            if isinstance(v, torch.Tensor):
                tensors[pfx + k] = v
            elif isinstance(v, TSObject):
                walk(v, pfx + k + ".")
            elif isinstance(v, (bool, int, float, str)) or v is None:
                scalars[pfx + k] = v
            elif isinstance(v, (list, tuple)) and all(isinstance(t, torch.Tensor) for t in v):
                for i, t in enumerate(v):
                    tensors[f"{pfx}{k}.{i}"] = t
            elif isinstance(v, dict):
                scalars[pfx + k] = v

    walk(root, "")
    return tensors, scalars


def load_torchscript(path: str) -> Tuple["OrderedDict[str, torch.Tensor]", Dict[str, object]]:
    """Detectron2 state dict + scalar attributes of an exported model: the
    ScriptableAdapter's ``model.`` prefix is removed."""
    tensors, scalars = flatten(read_archive(path))
    if tensors and all(k.startswith("model.") for k in tensors):
        tensors = OrderedDict((k[len("model."):], v) for k, v in tensors.items())
        scalars = {k[len("model."):] if k.startswith("model.") else k: v for k, v in scalars.items()}
    return tensors, scalars


def infer_config(sd: Dict[str, torch.Tensor], scalars: Dict[str, object] = None, **overrides) -> ModelConfig:
    """ModelConfig of a Detectron2 state dict (architecture from the tensor
    names / shapes; thresholds from the scripted modules' attributes when
    present: FastRCNNOutputLayers.test_score_thresh / test_nms_thresh /
    test_topk_per_image, RPN nms_thresh / min_box_size)."""
    scalars = scalars or {}
    c = ModelConfig()
    bu = "backbone.bottom_up"
    nres4 = len({k.split(".")[3] for k in sd if k.startswith(f"{bu}.res4.")})
    c.depth = {6: 50, 23: 101}.get(nres4, 50)
    w = sd[f"{bu}.stem.conv1.weight"]
    c.stem_out_channels = int(w.shape[0])
    c.input_format = "RGB" if int(w.shape[1]) == 3 else "L"
    c.width_per_group = int(sd[f"{bu}.res2.0.conv1.weight"].shape[0])
    c.res2_out_channels = int(sd[f"{bu}.res2.0.conv3.weight"].shape[0])
    c.fpn_out_channels = int(sd["backbone.fpn_output2.weight"].shape[0])
    c.fpn_norm = "GN" if "backbone.fpn_output2.norm.weight" in sd else ""
    c.num_classes = int(sd["roi_heads.box_predictor.cls_score.weight"].shape[0]) - 1
    c.box_num_fc = len([k for k in sd if k.startswith("roi_heads.box_head.fc") and k.endswith(".weight")])
    c.box_fc_dim = int(sd["roi_heads.box_head.fc1.weight"].shape[0])
    c.mask_on = "roi_heads.mask_head.predictor.weight" in sd
    if c.mask_on:
        c.mask_num_conv = len([k for k in sd if k.startswith("roi_heads.mask_head.mask_fcn") and k.endswith(".weight")])
        c.mask_conv_dim = int(sd["roi_heads.mask_head.deconv.weight"].shape[1])
    c.keypoint_on = "roi_heads.keypoint_head.score_lowres.weight" in sd
    if c.keypoint_on:
        n = len([k for k in sd if k.startswith("roi_heads.keypoint_head.conv_fcn") and k.endswith(".weight")])
        c.keypoint_conv_dims = tuple(int(sd[f"roi_heads.keypoint_head.conv_fcn{i + 1}.weight"].shape[0])
                                     for i in range(n))
        c.num_keypoints = int(sd["roi_heads.keypoint_head.score_lowres.weight"].shape[1])
    A = int(sd["proposal_generator.rpn_head.objectness_logits.weight"].shape[0])
    if A != len(c.aspect_ratios):
        raise NotImplementedError(f"{A} anchors per location (expected {len(c.aspect_ratios)})")
    if "pixel_mean" in sd:
        c.pixel_mean = tuple(float(v) for v in sd["pixel_mean"].reshape(-1))
        c.pixel_std = tuple(float(v) for v in sd["pixel_std"].reshape(-1))
    g = scalars.get
    bp = "roi_heads.box_predictor."
    c.score_thresh_test = float(g(bp + "test_score_thresh", c.score_thresh_test))
    c.nms_thresh_test = float(g(bp + "test_nms_thresh", c.nms_thresh_test))
    c.detections_per_image = int(g(bp + "test_topk_per_image", c.detections_per_image))
    c.rpn_nms_thresh = float(g("proposal_generator.nms_thresh", c.rpn_nms_thresh))
    c.rpn_min_box_size = float(g("proposal_generator.min_box_size", c.rpn_min_box_size))
    for k, v in overrides.items():
        setattr(c, k, v)
    return c
