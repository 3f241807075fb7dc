"""A4: the drop-in Predictor against the oracle, through the reference's call
contract (M/model/predict.py:46-102; TorchScript post-processing
M/model/util.py:45-62).  Full 512x424 synthetic frames (ROI crop 423x511,
the production shape), uint8 (N,H,W,1) numpy in -> list of
{'instances': Instances}; every Instances field the reference's downstream
code reads (pred_boxes, scores, pred_classes, pred_masks,
pred_keypoints, pred_keypoint_heatmaps) is compared with
oracle/model_ref.py's restatement of Detectron2's inference on the same
frames, for both constructors: ``from_config`` (the default dtype, which is
the reference's fp32) and ``from_torchscript`` on an archive written here.

Tolerances (fp32, as tests/test_parity_full.py): same detection count and
classes; every oracle box matched by a box of IoU >= 0.98 and |score diff|
<= 1e-3; matched masks differ in <= max(4, 3 % of the union) pixels;
>= 90 % of keypoints within 1 px, keypoint scores (heatmap-maximum logits,
up to ~50) within 1e-3 absolute + 1e-4 relative;
heatmap logits within 1e-3 of the largest |logit|."""
import numpy as np
import pytest
import torch

from _ts_archive import write_archive

pytestmark = pytest.mark.gpu

N = 4
SEED = 77


@pytest.fixture(scope="module")
def case(mdx, tmp_path_factory):
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    from oracle import frameops as O
    from oracle import model_ref as R
    cfg = ModelConfig(score_thresh_test=0.0)
    sd = synthetic_state_dict(cfg, 0)
    s = synth.SyntheticSession(N, seed=SEED)
    prepped, _ = O.prep_raw_frames(s.frames(0, N), s.bground_im, s.roi, 0, 100)
    img = np.ascontiguousarray(O.scale_raw_frames(prepped, 0, 100)[..., None])  # (N,423,511,1) uint8
    want, _ = R.forward(sd, cfg, img, keep_intermediates=False)
    scalars = {"roi_heads.box_predictor.test_score_thresh": 0.0, "roi_heads.box_predictor.test_topk_per_image": 4,
               "roi_heads.box_predictor.test_nms_thresh": 0.5}
    path = write_archive(tmp_path_factory.mktemp("ts") / "model.ts", sd, scalars)
    return cfg, sd, img, want, path


def _iou(a, b):
    x1 = np.maximum(a[:, None, 0], b[None, :, 0]); y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2]); y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]); ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + ab[None, :] - inter)


def _check(preds, want, hw):
    assert isinstance(preds, list) and len(preds) == len(want)
    for p, w in zip(preds, want):
        assert set(p) == {"instances"}
        ins = p["instances"].to("cpu")
        assert ins.image_size == hw
        n = len(ins)
        assert n == len(w["pred_boxes"]) and n >= 1
        gb, wb = ins.pred_boxes.tensor.numpy(), w["pred_boxes"].numpy()
        iou = _iou(wb, gb)
        m = iou.argmax(1)
        assert iou.max(1).min() >= 0.98
        np.testing.assert_allclose(ins.scores.numpy()[m], w["scores"].numpy(), atol=1e-3, rtol=0)
        assert ins.pred_classes.dtype == torch.int64
        np.testing.assert_array_equal(ins.pred_classes.numpy()[m], w["pred_classes"].numpy())
        gm, wm = ins.pred_masks.numpy()[m], w["pred_masks"].numpy()
        assert ins.pred_masks.dtype == torch.bool and gm.shape == wm.shape == (n,) + hw
        for j in range(n):
            diff, union = np.logical_xor(gm[j], wm[j]).sum(), np.logical_or(gm[j], wm[j]).sum()
            assert diff <= max(4, 0.03 * union), (j, diff, union)
        gk, wk = ins.pred_keypoints.numpy()[m], w["pred_keypoints"].numpy()
        assert gk.shape == wk.shape == (n, 8, 3)
        assert (np.abs(gk[..., :2] - wk[..., :2]).max(-1) < 1.0).mean() >= 0.9
        np.testing.assert_allclose(gk[..., 2], wk[..., 2], atol=1e-3, rtol=1e-4)
        gh, wh = ins.pred_keypoint_heatmaps.numpy()[m], w["pred_keypoint_heatmaps"].numpy()
        assert gh.shape == wh.shape == (n, 8, 28, 28)
        assert np.abs(gh - wh).max() <= 1e-3 * np.abs(wh).max()


def test_predictor_from_config_matches_oracle(case):
    from moseq2_detectron_extract_amd.model import Predictor
    cfg, sd, img, want, _ = case
    pred = Predictor.from_config(cfg, weights=sd)  # reference constructor, default dtype
    assert pred.model.dtype == "fp32" and not pred.is_torchscript
    assert pred.device.type == "cuda"
    _check(pred(img), want, img.shape[1:3])
    # one (H,W,C) image -> one dict; an RGB-replicated frame and a device
    # tensor give the same Instances as the 1-channel numpy batch
    one = pred(img[1])
    assert isinstance(one, dict)
    _check([one], want[1:2], img.shape[1:3])
    rgb = pred(np.repeat(img[:2], 3, axis=3))
    dev = pred(torch.from_numpy(img[:2]).cuda())
    base = pred(img[:2])
    for a, b, c in zip(rgb, dev, base):
        for f in ("pred_boxes", "scores", "pred_masks", "pred_keypoints", "pred_keypoint_heatmaps"):
            x, y, z = (getattr(t["instances"], f) for t in (a, b, c))
            x, y, z = (t.tensor if f == "pred_boxes" else t for t in (x, y, z))
            assert torch.equal(x, z) and torch.equal(y, z), f


def test_predictor_from_torchscript_matches_oracle(case):
    """M/model/predict.py:46-51 + M/model/util.py:45-62: the archive's
    weights and test thresholds drive the same native forward."""
    from moseq2_detectron_extract_amd.model import Predictor
    cfg, _, img, want, path = case
    pred = Predictor.from_torchscript(path)
    assert pred.is_torchscript and pred.model.dtype == "fp32"
    c = pred.model.cfg
    assert (c.depth, c.score_thresh_test, c.detections_per_image, c.nms_thresh_test) == (50, 0.0, 4, 0.5)
    _check(pred(img), want, img.shape[1:3])
