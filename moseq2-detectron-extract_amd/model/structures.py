"""Minimal Detectron2-compatible result containers.

The reference's downstream code reads model outputs through Detectron2's
``Instances``/``Boxes`` API (M/pipeline/process_features_step.py:63-160,
M/proc/proc.py:657-685, M/model/util.py:65-76).  Detectron2 is not a runtime
dependency here, so these classes provide the same surface: field access,
``len``, boolean/index selection, ``to(device)``, ``Instances.cat``,
``Boxes.tensor`` / ``get_centers()`` / ``area()``.
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple

import torch


class Boxes:
    def __init__(self, tensor: torch.Tensor):
        if not isinstance(tensor, torch.Tensor):
            tensor = torch.as_tensor(tensor, dtype=torch.float32)
        self.tensor = tensor.reshape(-1, 4)

    def __len__(self):
        return self.tensor.shape[0]

    def __getitem__(self, item):
        t = self.tensor[item]
        return Boxes(t.view(1, -1) if t.dim() == 1 else t)

    def to(self, *args, **kwargs):
        return Boxes(self.tensor.to(*args, **kwargs))

    def clone(self):
        return Boxes(self.tensor.clone())

    def get_centers(self) -> torch.Tensor:
        return (self.tensor[:, :2] + self.tensor[:, 2:]) / 2

    def area(self) -> torch.Tensor:
        b = self.tensor
        return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])

    @property
    def device(self):
        return self.tensor.device

    @staticmethod
    def cat(boxes_list: List["Boxes"]) -> "Boxes":
        return Boxes(torch.cat([b.tensor for b in boxes_list], dim=0))

    def __repr__(self):
        return f"Boxes({self.tensor!r})"


class Instances:
    """Per-image detection results (Detectron2 ``Instances`` surface)."""

    def __init__(self, image_size: Tuple[int, int], **kwargs: Any):
        object.__setattr__(self, "_image_size", (int(image_size[0]), int(image_size[1])))
        object.__setattr__(self, "_fields", {})
        for k, v in kwargs.items():
            self.set(k, v)

    @property
    def image_size(self) -> Tuple[int, int]:
        return self._image_size

    def __setattr__(self, name, val):
        if name.startswith("_"):
            object.__setattr__(self, name, val)
        else:
            self.set(name, val)

    def __getattr__(self, name):
        if name == "_fields" or name not in self._fields:
            raise AttributeError(f"Cannot find field '{name}' in the given Instances!")
        return self._fields[name]

    def set(self, name: str, value: Any) -> None:
        n = len(value)
        if len(self._fields):
            assert len(self) == n, f"Adding a field of length {n} to a Instances of length {len(self)}"
        self._fields[name] = value

    def has(self, name: str) -> bool:
        return name in self._fields

    def remove(self, name: str) -> None:
        del self._fields[name]

    def get(self, name: str) -> Any:
        return self._fields[name]

    def get_fields(self) -> Dict[str, Any]:
        return self._fields

    def to(self, *args, **kwargs) -> "Instances":
        ret = Instances(self._image_size)
        for k, v in self._fields.items():
            if hasattr(v, "to"):
                v = v.to(*args, **kwargs)
            ret.set(k, v)
        return ret

    def __getitem__(self, item) -> "Instances":
        if isinstance(item, int):
            if item >= len(self) or item < -len(self):
                raise IndexError("Instances index out of range!")
            item = slice(item, None, len(self)) if item == -1 else slice(item, item + 1)
        ret = Instances(self._image_size)
        for k, v in self._fields.items():
            if isinstance(item, (list, tuple)) or (hasattr(item, "dtype") and not isinstance(item, slice)):
                if isinstance(v, Boxes):
                    ret.set(k, Boxes(v.tensor[torch.as_tensor(item)]))
                else:
                    ret.set(k, v[torch.as_tensor(item)])
            else:
                ret.set(k, v[item])
        return ret

    def __len__(self) -> int:
        for v in self._fields.values():
            return len(v)
        raise NotImplementedError("Empty Instances does not support __len__!")

    def __iter__(self):
        raise NotImplementedError("`Instances` object is not iterable!")

    @staticmethod
    def cat(instance_lists: List["Instances"]) -> "Instances":
        assert len(instance_lists) > 0
        if len(instance_lists) == 1:
            return instance_lists[0]
        image_size = instance_lists[0].image_size
        ret = Instances(image_size)
        for k in instance_lists[0]._fields.keys():
            values = [i.get(k) for i in instance_lists]
            v0 = values[0]
            if isinstance(v0, torch.Tensor):
                values = torch.cat(values, dim=0)
            elif isinstance(v0, Boxes):
                values = Boxes.cat(values)
            elif isinstance(v0, list):
                values = [x for v in values for x in v]
            else:
                raise ValueError(f"Unsupported type {type(v0)} for concatenation")
            ret.set(k, values)
        return ret

    def __repr__(self):
        s = f"Instances(num_instances={len(self) if self._fields else 0}, image_height={self._image_size[0]}, " \
            f"image_width={self._image_size[1]}, fields=[{', '.join(self._fields.keys())}])"
        return s


def create_empty_instances(width: int, height: int, nkeypoints: int) -> Instances:
    """M/model/util.py:65-76."""
    return Instances(
        (height, width),
        pred_boxes=Boxes(torch.empty(size=(0, 4), dtype=torch.float32)),
        scores=torch.empty(size=(0,), dtype=torch.float32),
        pred_classes=torch.empty(size=(0,), dtype=torch.int64),
        pred_masks=torch.empty(size=(0, height, width), dtype=torch.bool),
        pred_keypoints=torch.empty(size=(0, nkeypoints, 3), dtype=torch.float32),
        pred_keypoints_heatmaps=torch.empty(size=(0, nkeypoints, 28, 28), dtype=torch.float32),
    )
