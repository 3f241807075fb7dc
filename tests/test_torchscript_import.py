"""Weights-only import of a TorchScript archive (model/torchscript.py;
reference: Predictor.from_torchscript M/model/predict.py:46-51, export
M/model/deploy.py:77-121).  An archive with the exported model's module tree
(ScriptableAdapter.model = GeneralizedRCNN: the Detectron2 parameter / buffer
names, FastRCNNOutputLayers' test thresholds as attributes) is written with
torch.jit.save here; the restricted unpickler must return exactly its tensors
and refuse any global outside the TorchScript / tensor set."""
import pickle
import zipfile

import pytest
import torch

from _ts_archive import write_archive


@pytest.fixture(scope="module")
def archive(tmp_path_factory, mdx):
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    cfg = ModelConfig(depth=101)
    sd = synthetic_state_dict(cfg, 5)
    scalars = {"roi_heads.box_predictor.test_score_thresh": 0.25, "roi_heads.box_predictor.test_topk_per_image": 3,
               "roi_heads.box_predictor.test_nms_thresh": 0.45}
    path = write_archive(tmp_path_factory.mktemp("ts") / "model.ts", sd, scalars)
    return path, sd


def test_state_dict_roundtrip(archive):
    from moseq2_detectron_extract_amd.model.torchscript import load_torchscript
    path, sd = archive
    got, scalars = load_torchscript(path)
    assert set(got) == set(sd)
    for k in sd:
        assert got[k].dtype == torch.float32 and torch.equal(got[k], sd[k]), k
    assert scalars["roi_heads.box_predictor.test_score_thresh"] == 0.25


def test_infer_config(archive):
    from moseq2_detectron_extract_amd.model.torchscript import infer_config, load_torchscript
    path, _ = archive
    sd, scalars = load_torchscript(path)
    c = infer_config(sd, scalars)
    assert c.depth == 101 and c.num_keypoints == 8 and c.keypoint_conv_dims == (512,) * 8
    assert c.mask_on and c.keypoint_on and c.fpn_norm == "GN" and c.input_format == "RGB"
    assert c.score_thresh_test == 0.25 and c.detections_per_image == 3 and c.nms_thresh_test == 0.45
    assert infer_config(sd, scalars, score_thresh_test=0.5).score_thresh_test == 0.5


def test_refuses_foreign_globals(tmp_path, mdx):
    """A data.pkl naming anything outside the TorchScript/tensor globals is
    refused before any object is built."""
    from moseq2_detectron_extract_amd.model.torchscript import read_archive
    evil = pickle.dumps(zipfile.ZipFile)  # a global the importer must not resolve
    p = tmp_path / "bad.ts"
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("bad/data.pkl", evil)
        z.writestr("bad/byteorder", "little")
    with pytest.raises(pickle.UnpicklingError, match="refusing global"):
        read_archive(str(p))
    p2 = tmp_path / "notts.ts"
    with zipfile.ZipFile(p2, "w") as z:
        z.writestr("x.txt", "hi")
    with pytest.raises(ValueError):
        read_archive(str(p2))


@pytest.mark.gpu
def test_torchscript_predictor_equals_config_predictor(archive):
    """The imported archive runs on the native kernels exactly like the same
    weights given as a state dict."""
    import numpy as np
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    path, sd = archive
    ts = Predictor.from_torchscript(path, dtype="fp32", score_thresh_test=0.0)
    assert ts.is_torchscript and ts.model.cfg.depth == 101
    ref = Predictor.from_config(ModelConfig(depth=101, score_thresh_test=0.0, nms_thresh_test=0.45,
                                            detections_per_image=3), weights=sd, dtype="fp32")
    img = np.random.default_rng(3).integers(0, 256, size=(2, 96, 128, 1), dtype=np.uint8)
    a, b = ts(img), ref(img)
    for x, y in zip(a, b):
        xi, yi = x["instances"], y["instances"]
        assert len(xi) == len(yi)
        torch.testing.assert_close(xi.pred_boxes.tensor, yi.pred_boxes.tensor, rtol=0, atol=0)
        torch.testing.assert_close(xi.pred_keypoints, yi.pred_keypoints, rtol=0, atol=0)
