"""Mask/Keypoint R-CNN forward of the extraction hot path (M/model/)."""
from .config import ModelConfig  # noqa: F401
from .structures import Boxes, Instances, create_empty_instances  # noqa: F401
from .weights import load_state_dict, synthetic_state_dict  # noqa: F401


def __getattr__(name):
    # the runtime needs torch + the HIP library; import lazily
    if name in ("MaskRCNN", "flops_per_image"):
        from . import runtime
        return getattr(runtime, name)
    if name in ("Predictor", "outputs_to_instances"):
        from . import predict
        return getattr(predict, name)
    raise AttributeError(name)
