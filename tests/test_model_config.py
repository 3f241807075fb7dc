"""Drop-in model construction from a trained model directory (SURVEY §8(b)
"Model wrapper"): Predictor.from_config / from_model_dir read a Detectron2
config.yaml (M/pipeline/inference_step.py:35-52), load MODEL.WEIGHTS
(M/model/predict.py:31-44, weights-only) and refuse what the native kernels
do not implement.  Host side only: the GPU half (the same directory through
the native forward, against the oracle) is
tests/test_predictor_parity.py::test_predictor_from_model_dir_matches_oracle."""
import os

import numpy as np
import pytest
import torch

from _d2_config import d2_config, write_model_dir


@pytest.fixture(scope="module")
def small_sd(mdx):
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    return synthetic_state_dict(ModelConfig(), 3)


def test_model_dir_loads_weights_and_honours_config(mdx, small_sd, tmp_path):
    from moseq2_detectron_extract_amd.model.predict import model_dir_config, resolve_model
    ck = write_model_dir(tmp_path / "m", d2_config(**{"MODEL.ROI_HEADS.NMS_THRESH_TEST": 0.45,
                                                       "MODEL.RPN.POST_NMS_TOPK_TEST": 500}), small_sd)
    cfg = model_dir_config(str(tmp_path / "m"), "last", instance_threshold=0.3, allowed_detections=2)
    assert cfg.weights == ck
    # the CLI overrides win over the file, the file over the base config
    assert (cfg.score_thresh_test, cfg.detections_per_image) == (0.3, 2)
    assert (cfg.nms_thresh_test, cfg.rpn_post_nms_topk_test) == (0.45, 500)
    assert cfg.box_reg_weights == (10.0, 10.0, 5.0, 5.0) and cfg.rpn_bbox_reg_weights == (1.0, 1.0, 1.0, 1.0)
    cfg2, sd = resolve_model(cfg)
    assert list(sd) == list(small_sd)
    assert all(torch.equal(sd[k], small_sd[k]) for k in sd)
    # a specific iteration (get_specific_checkpoint)
    assert model_dir_config(str(tmp_path / "m"), 99999).weights == ck
    with pytest.raises(FileNotFoundError):
        model_dir_config(str(tmp_path / "m"), 12345)


def test_every_cfg_key_reaches_the_abi(mdx):
    """Non-default values of every key struct mdx_model_cfg carries travel
    from the yaml into the C struct."""
    from moseq2_detectron_extract_amd.model import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import model_cfg_c
    y = d2_config(**{
        "MODEL.RESNETS.DEPTH": 101, "MODEL.RESNETS.STRIDE_IN_1X1": False,
        "MODEL.FPN.FUSE_TYPE": "sum", "MODEL.FPN.OUT_CHANNELS": 128,
        "MODEL.ANCHOR_GENERATOR.SIZES": [[16], [40], [100], [250], [600]],
        "MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS": [[0.5, 1.0, 2.0, 3.0, 4.0]],
        "MODEL.ANCHOR_GENERATOR.OFFSET": 0.5,
        "MODEL.PROPOSAL_GENERATOR.MIN_SIZE": 2,
        "MODEL.RPN.PRE_NMS_TOPK_TEST": 600, "MODEL.RPN.POST_NMS_TOPK_TEST": 300, "MODEL.RPN.NMS_THRESH": 0.6,
        "MODEL.RPN.BBOX_REG_WEIGHTS": [2.0, 2.0, 1.0, 1.0],
        "MODEL.ROI_HEADS.SCORE_THRESH_TEST": 0.25, "MODEL.ROI_HEADS.NMS_THRESH_TEST": 0.4,
        "MODEL.ROI_BOX_HEAD.POOLER_RESOLUTION": 5, "MODEL.ROI_BOX_HEAD.NUM_FC": 1,
        "MODEL.ROI_BOX_HEAD.FC_DIM": 512, "MODEL.ROI_BOX_HEAD.BBOX_REG_WEIGHTS": [5.0, 5.0, 2.0, 2.0],
        "MODEL.ROI_BOX_HEAD.POOLER_SAMPLING_RATIO": 2, "MODEL.ROI_MASK_HEAD.POOLER_SAMPLING_RATIO": 2,
        "MODEL.ROI_KEYPOINT_HEAD.POOLER_SAMPLING_RATIO": 2,
        "MODEL.ROI_MASK_HEAD.POOLER_RESOLUTION": 12, "MODEL.ROI_MASK_HEAD.NUM_CONV": 2,
        "MODEL.ROI_MASK_HEAD.CONV_DIM": 128,
        "MODEL.ROI_KEYPOINT_HEAD.POOLER_RESOLUTION": 6, "MODEL.ROI_KEYPOINT_HEAD.CONV_DIMS": [256] * 4,
        "MODEL.ROI_KEYPOINT_HEAD.NUM_KEYPOINTS": 6,
        "MODEL.PIXEL_MEAN": [2.0, 2.0, 2.0], "MODEL.PIXEL_STD": [4.0, 4.0, 4.0],
        "TEST.DETECTIONS_PER_IMAGE": 3})
    c = ModelConfig.from_yaml(y)
    s = model_cfg_c(c, "fp32")
    assert (s.depth, s.stride_in_1x1, s.fpn_fuse_avg, s.fpn_out_channels) == (101, 0, 0, 128)
    assert list(s.anchor_sizes) == [16, 40, 100, 250, 600]
    assert s.n_aspect_ratios == 5 and list(s.aspect_ratios)[:5] == [0.5, 1.0, 2.0, 3.0, 4.0]
    assert (s.anchor_offset, s.rpn_min_box_size) == (0.5, 2.0)
    assert (s.rpn_pre_nms_topk, s.rpn_post_nms_topk) == (600, 300)
    assert abs(s.rpn_nms_thresh - 0.6) < 1e-7 and list(s.rpn_bbox_reg_weights) == [2, 2, 1, 1]
    assert abs(s.score_thresh - 0.25) < 1e-7 and abs(s.nms_thresh - 0.4) < 1e-7
    assert (s.box_pooler_resolution, s.box_num_fc, s.box_fc_dim) == (5, 1, 512)
    assert list(s.box_reg_weights) == [5, 5, 2, 2] and s.pooler_sampling_ratio == 2 and s.pooler_aligned == 1
    assert (s.mask_pooler_resolution, s.mask_num_conv, s.mask_conv_dim) == (12, 2, 128)
    assert (s.keypoint_pooler_resolution, s.n_keypoint_convs, s.num_keypoints) == (6, 4, 6)
    assert list(s.keypoint_conv_dims)[:4] == [256] * 4
    assert list(s.pixel_mean) == [2, 2, 2] and list(s.pixel_std) == [4, 4, 4] and s.detections_per_image == 3
    # a flat list of ratios is one entry broadcast to every level (Detectron2 _broadcast_params)
    assert ModelConfig.from_yaml(d2_config(**{"MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS": [0.5, 1, 2]})
                                 ).aspect_ratios == (0.5, 1.0, 2.0)
    assert ModelConfig.from_yaml(d2_config(**{"INPUT.FORMAT": "L", "MODEL.PIXEL_MEAN": [1.12],
                                              "MODEL.PIXEL_STD": [5.79]})).in_channels == 1
    # 'L' with the base config's three means: Detectron2's stem takes len(PIXEL_MEAN) = 3 channels
    # (ADVICE r4), so the state dict must carry a (64, 3, 7, 7) stem and does
    from moseq2_detectron_extract_amd.model.weights import state_dict_spec
    c3 = ModelConfig.from_yaml(d2_config(**{"INPUT.FORMAT": "L", "MODEL.PIXEL_MEAN": [1.12] * 3,
                                            "MODEL.PIXEL_STD": [5.79] * 3}))
    assert c3.in_channels == 3
    assert [shape for name, shape, _ in state_dict_spec(c3) if name.endswith("stem.conv1.weight")] == [(64, 3, 7, 7)]
    with pytest.raises(NotImplementedError, match="PIXEL_STD"):
        ModelConfig.from_yaml(d2_config(**{"INPUT.FORMAT": "L", "MODEL.PIXEL_MEAN": [1.12] * 3,
                                           "MODEL.PIXEL_STD": [5.79]}))


@pytest.mark.parametrize("key,val", [
    ("MODEL.ANCHOR_GENERATOR.NAME", "RotatedAnchorGenerator"),           # add_rotated_bbox_support
    ("MODEL.ROI_HEADS.NAME", "RROIHeads"),
    ("MODEL.PROPOSAL_GENERATOR.NAME", "RRPN"),
    ("MODEL.ROI_BOX_HEAD.POOLER_TYPE", "ROIAlignRotated"),
    ("MODEL.ROI_BOX_HEAD.BBOX_REG_WEIGHTS", [1, 1, 1, 1, 1]),
    ("MODEL.ANCHOR_GENERATOR.SIZES", [[32, 64, 128, 256, 512]]),          # 5 sizes at every level
    ("MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS", [[0.5, 1, 2, 3, 4, 5, 6, 7, 8]]),
    ("MODEL.ROI_MASK_HEAD.POOLER_SAMPLING_RATIO", 2),                     # heads disagree
    ("MODEL.RESNETS.NORM", "BN"),
    ("MODEL.RESNETS.DEFORM_ON_PER_STAGE", [False, True, True, True]),
    ("MODEL.FPN.NORM", ""),
    ("MODEL.ROI_BOX_HEAD.NUM_CONV", 4),
    ("MODEL.ROI_HEADS.NUM_CLASSES", 2),
    ("MODEL.RESNETS.DEPTH", 152),
    ("INPUT.FORMAT", "YUV"),
])
def test_unsupported_settings_are_refused(mdx, key, val):
    from moseq2_detectron_extract_amd.model import ModelConfig
    with pytest.raises(NotImplementedError, match=key.split(".")[-1] if "SAMPLING" not in key else "POOLER"):
        ModelConfig.from_yaml(d2_config(**{key: val}))


def test_weights_resolution_errors(mdx, small_sd, tmp_path):
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    from moseq2_detectron_extract_amd.model.predict import resolve_model
    # MODEL.WEIGHTS empty and no weights given: no silent random weights
    with pytest.raises(ValueError, match="MODEL.WEIGHTS is empty"):
        resolve_model(ModelConfig.from_yaml(d2_config()))
    # an explicit request for the seeded synthetic weights
    cfg, sd = resolve_model(ModelConfig(), "synthetic", seed=3)
    assert all(torch.equal(sd[k], small_sd[k]) for k in small_sd)
    # MODEL.WEIGHTS naming a missing file
    with pytest.raises(FileNotFoundError):
        resolve_model(d2_config(**{"MODEL.WEIGHTS": str(tmp_path / "nope.pth")}))
    # Detectron2's pickled .pkl format is not unpickled
    (tmp_path / "model.pkl").write_bytes(b"not loaded")
    with pytest.raises(ValueError, match="pickle"):
        resolve_model(d2_config(**{"MODEL.WEIGHTS": str(tmp_path / "model.pkl")}))
    # a checkpoint of another architecture: 5 aspect ratios in the yaml, a
    # 3-anchor RPN head in the checkpoint
    ck = write_model_dir(tmp_path / "m5", d2_config(**{"MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS":
                                                        [[0.5, 1.0, 2.0, 3.0, 4.0]]}), small_sd)
    y = d2_config(**{"MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS": [[0.5, 1.0, 2.0, 3.0, 4.0]], "MODEL.WEIGHTS": ck})
    with pytest.raises(ValueError, match="objectness_logits"):
        resolve_model(y)
    # ... and the matching 5-ratio checkpoint loads
    c5 = ModelConfig.from_yaml(y)
    sd5 = synthetic_state_dict(c5, 4)
    torch.save({"model": dict(sd5)}, ck)
    cfg, sd = resolve_model(y)
    assert len(cfg.aspect_ratios) == 5 and sd["proposal_generator.rpn_head.anchor_deltas.weight"].shape[0] == 20
    # missing parameters
    part = {k: v for k, v in small_sd.items() if "keypoint_head" not in k}
    with pytest.raises(ValueError, match="missing"):
        resolve_model(ModelConfig(), part)


def test_predictor_needs_the_gpu(mdx, small_sd):
    """No CPU fallback: the constructor fails loudly without a GPU."""
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from moseq2_detectron_extract_amd._lib import MdxError
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    with pytest.raises(MdxError):
        Predictor.from_config(ModelConfig(), small_sd)
