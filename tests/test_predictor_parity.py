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

from _d2_config import d2_config, write_model_dir
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
    # the same weights as a trained model directory (config.yaml dumped by
    # Detectron2, model_XXXXXXX.pth, last_checkpoint)
    mdir = tmp_path_factory.mktemp("model_dir")
    write_model_dir(mdir, d2_config(), sd)
    return cfg, sd, img, want, path, str(mdir)


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
    cfg, sd, img, want, _, _ = case
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
    cfg, _, img, want, path, _ = case
    pred = Predictor.from_torchscript(path)
    assert pred.is_torchscript and pred.model.dtype == "fp32"
    c = pred.model.cfg
    assert (c.depth, c.score_thresh_test, c.detections_per_image, c.nms_thresh_test) == (50, 0.0, 4, 0.5)
    _check(pred(img), want, img.shape[1:3])


def test_predictor_from_model_dir_matches_oracle(case):
    """The reference's model-directory path (M/pipeline/inference_step.py:35-52):
    <dir>/config.yaml read, MODEL.WEIGHTS = the last checkpoint, loaded
    weights-only, --instance-threshold / --allowed-detections applied, then
    Predictor.from_config(cfg) with no weights argument."""
    from moseq2_detectron_extract_amd.model import Predictor
    from moseq2_detectron_extract_amd.model.predict import model_dir_config
    _, _, img, want, _, mdir = case
    cfg = model_dir_config(mdir, "last", instance_threshold=0.0, allowed_detections=4)
    assert cfg.weights.endswith(".pth")
    pred = Predictor.from_config(cfg)
    _check(pred(img), want, img.shape[1:3])
    pred2 = Predictor.from_model_dir(mdir, instance_threshold=0.0, allowed_detections=4)
    a, b = pred(img[:1]), pred2(img[:1])
    assert torch.equal(a[0]["instances"].pred_boxes.tensor, b[0]["instances"].pred_boxes.tensor)


def test_two_policies_concurrently_on_two_streams(case):
    """Per-handle kernel selection (include/mdx.h, mdx_policy): a predictor
    built with direct 3x3 convolutions (winograd 0) and one built with F(6,3)
    Winograd and another ROI-align mode, created side by side on one thread,
    their forwards enqueued on two streams with no synchronisation between
    them, three times over.  Each handle keeps the policy it was created
    with, each concurrent result equals that handle's serial result bit for
    bit, each matches the oracle, and the thread's own policy is untouched."""
    from moseq2_detectron_extract_amd._lib import policy
    from moseq2_detectron_extract_amd.model import Predictor
    cfg, sd, img, want, _, _ = case
    before = policy()
    pa = Predictor.from_config(cfg, weights=sd, policy={"winograd": 0})
    pb = Predictor.from_config(cfg, weights=sd, policy={"winograd": 6, "roi_mode": 7})
    assert policy() == before
    assert pa.model.policy()["winograd"] == 0 and pa.model.policy()["roi_mode"] == before["roi_mode"]
    assert pb.model.policy()["winograd"] == 6 and pb.model.policy()["roi_mode"] == 7
    _check(pa(img), want, img.shape[1:3])
    _check(pb(img), want, img.shape[1:3])
    x = torch.from_numpy(img[..., 0]).cuda()
    keys = ("boxes", "scores", "classes", "ndet", "keypoints", "keypoint_heatmaps")

    def snap(o):
        return {k: o[k].clone() for k in keys} | {"masks": o["masks"].clone()}
    serial_a, serial_b = snap(pa.model.forward(x)), snap(pb.model.forward(x))
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    sa.wait_stream(torch.cuda.current_stream())
    sb.wait_stream(torch.cuda.current_stream())
    runs = []
    for _ in range(3):
        with torch.cuda.stream(sa):
            ra = snap(pa.model.forward(x))
        with torch.cuda.stream(sb):
            rb = snap(pb.model.forward(x))
        runs.append((ra, rb))
    torch.cuda.synchronize()
    for ra, rb in runs:
        for k in serial_a:
            assert torch.equal(ra[k], serial_a[k]), ("winograd 0", k)
            assert torch.equal(rb[k], serial_b[k]), ("winograd 6", k)
    # the two policies run different 3x3 kernels: close, not identical
    assert not torch.equal(serial_a["keypoint_heatmaps"], serial_b["keypoint_heatmaps"])
    assert policy() == before


def test_predictor_non_default_anchors_match_oracle(mdx, tmp_path):
    """A model directory whose config differs from the zoo defaults in the
    anchor generator (the reference notebook's five aspect ratios, other
    sizes and offset) and the RPN / box regression weights: the native
    forward follows the file, as the oracle does."""
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor, synthetic_state_dict
    from oracle import frameops as O
    from oracle import model_ref as R
    y = d2_config(**{"MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS": [[0.5, 1.0, 2.0, 3.0, 4.0]],
                     "MODEL.ANCHOR_GENERATOR.SIZES": [[24], [48], [96], [192], [384]],
                     "MODEL.ANCHOR_GENERATOR.OFFSET": 0.5,
                     "MODEL.RPN.BBOX_REG_WEIGHTS": [2.0, 2.0, 1.0, 1.0],
                     "MODEL.ROI_BOX_HEAD.BBOX_REG_WEIGHTS": [8.0, 8.0, 4.0, 4.0],
                     "MODEL.ROI_HEADS.SCORE_THRESH_TEST": 0.0, "TEST.DETECTIONS_PER_IMAGE": 4})
    cfg = ModelConfig.from_yaml(y)
    sd = synthetic_state_dict(cfg, 2)
    write_model_dir(tmp_path / "m", y, sd)
    s = synth.SyntheticSession(2, seed=SEED + 1)
    prepped, _ = O.prep_raw_frames(s.frames(0, 2), s.bground_im, s.roi, 0, 100)
    img = np.ascontiguousarray(O.scale_raw_frames(prepped, 0, 100)[..., None])
    want, _ = R.forward(sd, cfg, img, keep_intermediates=False)
    pred = Predictor.from_model_dir(str(tmp_path / "m"), instance_threshold=0.0, allowed_detections=4)
    assert len(pred.model.cfg.aspect_ratios) == 5
    _check(pred(img), want, img.shape[1:3])
