"""A Detectron2 ``config.yaml`` as ``cfg.dump()`` writes it for the
reference's model (get_base_config, M/model/config.py:21-94, on COCO
keypoint_rcnn_R_50_FPN_3x, plus add_dataset_cfg's keypoint count and pixel
statistics) -- the inference-relevant subtree, with Detectron2's default
values for the keys the reference does not set.  Test data, written by hand
from Detectron2's published defaults (config/defaults.py); Detectron2 is not
importable here."""
import copy

BASE = {
    "MODEL": {
        "META_ARCHITECTURE": "GeneralizedRCNN",
        "WEIGHTS": "",
        "MASK_ON": True,
        "KEYPOINT_ON": True,
        "DEVICE": "cuda",
        "PIXEL_MEAN": [1.12, 1.12, 1.12],
        "PIXEL_STD": [5.79, 5.79, 5.79],
        "LOAD_PROPOSALS": False,
        "BACKBONE": {"NAME": "build_resnet_fpn_backbone", "FREEZE_AT": 0},
        "RESNETS": {"DEPTH": 50, "OUT_FEATURES": ["res2", "res3", "res4", "res5"], "NUM_GROUPS": 1,
                    "NORM": "FrozenBN", "WIDTH_PER_GROUP": 64, "STRIDE_IN_1X1": True, "RES5_DILATION": 1,
                    "RES2_OUT_CHANNELS": 256, "STEM_OUT_CHANNELS": 64,
                    "DEFORM_ON_PER_STAGE": [False, False, False, False], "DEFORM_MODULATED": False,
                    "DEFORM_NUM_GROUPS": 1},
        "FPN": {"IN_FEATURES": ["res2", "res3", "res4", "res5"], "OUT_CHANNELS": 256, "NORM": "GN",
                "FUSE_TYPE": "avg"},
        "PROPOSAL_GENERATOR": {"NAME": "RPN", "MIN_SIZE": 0},
        "ANCHOR_GENERATOR": {"NAME": "DefaultAnchorGenerator", "SIZES": [[32], [64], [128], [256], [512]],
                             "ASPECT_RATIOS": [[0.5, 1.0, 2.0]], "ANGLES": [[-90, 0, 90]], "OFFSET": 0.0},
        "RPN": {"HEAD_NAME": "StandardRPNHead", "IN_FEATURES": ["p2", "p3", "p4", "p5", "p6"],
                "BOUNDARY_THRESH": -1, "IOU_THRESHOLDS": [0.3, 0.7], "IOU_LABELS": [0, -1, 1],
                "BATCH_SIZE_PER_IMAGE": 256, "POSITIVE_FRACTION": 0.5, "BBOX_REG_LOSS_TYPE": "smooth_l1",
                "BBOX_REG_LOSS_WEIGHT": 1.0, "BBOX_REG_WEIGHTS": [1.0, 1.0, 1.0, 1.0], "SMOOTH_L1_BETA": 0.0,
                "LOSS_WEIGHT": 1.0, "PRE_NMS_TOPK_TRAIN": 2000, "PRE_NMS_TOPK_TEST": 1000,
                "POST_NMS_TOPK_TRAIN": 1500, "POST_NMS_TOPK_TEST": 1000, "NMS_THRESH": 0.7, "CONV_DIMS": [-1]},
        "ROI_HEADS": {"NAME": "StandardROIHeads", "NUM_CLASSES": 1, "IN_FEATURES": ["p2", "p3", "p4", "p5"],
                      "IOU_THRESHOLDS": [0.5], "IOU_LABELS": [0, 1], "BATCH_SIZE_PER_IMAGE": 256,
                      "POSITIVE_FRACTION": 0.5, "SCORE_THRESH_TEST": 0.05, "NMS_THRESH_TEST": 0.5,
                      "PROPOSAL_APPEND_GT": True},
        "ROI_BOX_HEAD": {"NAME": "FastRCNNConvFCHead", "BBOX_REG_LOSS_TYPE": "smooth_l1",
                         "BBOX_REG_LOSS_WEIGHT": 1.0, "BBOX_REG_WEIGHTS": [10.0, 10.0, 5.0, 5.0],
                         "SMOOTH_L1_BETA": 0.5, "POOLER_RESOLUTION": 7, "POOLER_SAMPLING_RATIO": 0,
                         "POOLER_TYPE": "ROIAlignV2", "NUM_FC": 2, "FC_DIM": 1024, "NUM_CONV": 0, "CONV_DIM": 256,
                         "NORM": "", "CLS_AGNOSTIC_BBOX_REG": False, "TRAIN_ON_PRED_BOXES": False,
                         "USE_FED_LOSS": False, "USE_SIGMOID_CE": False, "FED_LOSS_FREQ_WEIGHT_POWER": 0.5,
                         "FED_LOSS_NUM_CLASSES": 50},
        "ROI_MASK_HEAD": {"NAME": "MaskRCNNConvUpsampleHead", "POOLER_RESOLUTION": 14, "POOLER_SAMPLING_RATIO": 0,
                          "NUM_CONV": 4, "CONV_DIM": 256, "NORM": "", "CLS_AGNOSTIC_MASK": False,
                          "POOLER_TYPE": "ROIAlignV2"},
        "ROI_KEYPOINT_HEAD": {"NAME": "KRCNNConvDeconvUpsampleHead", "POOLER_RESOLUTION": 7,
                              "POOLER_SAMPLING_RATIO": 0, "CONV_DIMS": [512] * 8, "NUM_KEYPOINTS": 8,
                              "MIN_KEYPOINTS_PER_IMAGE": 1, "NORMALIZE_LOSS_BY_VISIBLE_KEYPOINTS": True,
                              "LOSS_WEIGHT": 1.0, "POOLER_TYPE": "ROIAlignV2"},
    },
    "INPUT": {"FORMAT": "RGB", "MIN_SIZE_TRAIN": [240], "MAX_SIZE_TRAIN": 250, "MIN_SIZE_TEST": 240,
              "MAX_SIZE_TEST": 250, "RANDOM_FLIP": "none", "MASK_FORMAT": "polygon"},
    "TEST": {"DETECTIONS_PER_IMAGE": 1, "EVAL_PERIOD": 1000, "KEYPOINT_OKS_SIGMAS": [0.026, 0.035, 0.035, 0.079,
                                                                                      0.107, 0.107, 0.089, 0.026]},
    "SOLVER": {"IMS_PER_BATCH": 8, "BASE_LR": 0.0025, "MAX_ITER": 100000, "AMP": {"ENABLED": True}},
    "OUTPUT_DIR": "./models/output_4",
    "VERSION": 2,
}


def d2_config(**paths):
    """BASE with overrides given as dotted keys, e.g.
    d2_config(**{"MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS": [[0.5, 1, 2, 3, 4]]})."""
    c = copy.deepcopy(BASE)
    for k, v in paths.items():
        node = c
        parts = k.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return c


def write_model_dir(d, cfg: dict, sd, iteration: int = 99999):
    """A trained model directory as DefaultTrainer leaves it: config.yaml,
    model_<iter>.pth ({'model': state_dict, 'iteration': ...}) and the
    last_checkpoint file naming it."""
    import os
    import torch
    import yaml
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "config.yaml"), "w", encoding="utf-8") as fh:
        yaml.safe_dump(cfg, fh)
    name = f"model_{iteration:07d}.pth"
    torch.save({"model": dict(sd), "iteration": iteration, "optimizer": {"state": {}, "param_groups": []}},
               os.path.join(d, name))
    with open(os.path.join(d, "last_checkpoint"), "w", encoding="utf-8") as fh:
        fh.write(name)
    return os.path.join(d, name)
