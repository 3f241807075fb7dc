"""BASELINE config 3 at its stated shape: extract.extract_session over a
synthetic session written as depth.dat, in chunks of 1000 frames (three of
them), fp32 (the reference's precision), tracking on (the reference's
default, M/cli.py:366), instance selection on, with the result writers --
the reference's extraction unit (M/extract.py:96-137,
M/pipeline/process_features_step.py:56-199).  The session's outputs are
compared with the oracle chain:

* chunk 1 (frames 1000-1999) through the oracle frame ops: prepped frames,
  cleaned frames bit for bit; moments of the selected masks: centroid and
  axis lengths bit for bit, orientation to 1e-14 rad;
* the host step over all three chunks: the restated pykalman / flip chain
  (oracle/kalman_ref.py, as tests/test_tracking.py) on the device features
  gives the session's centroids (1e-8 px), angles (1e-7 deg) and flips
  (exactly);
* chunk 1's crops: the oracle crop at the session's pose byte for byte, and
  at the restated pose on >= 99.5 % of the frames byte for byte;
* chunk 1's scalars: the oracle reductions through the same host code;
* the model on 32 frames of chunk 1 against the oracle forward: detection
  count, boxes (IoU >= 0.98), and -- where one instance survives mask NMS,
  so selection is the identity -- the selected mask within max(4 px, 3 %).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, CHUNK = 3000, 1000


@pytest.fixture(scope="module")
def session(mdx, tmp_path_factory):
    from moseq2_detectron_extract_amd import synth
    s = synth.SyntheticSession(N, seed=9)
    d = tmp_path_factory.mktemp("config3")
    s.write(str(d), workers=max(1, min(16, len(os.sched_getaffinity(0)))))
    return s, d


def _iou(a, b):
    x1 = np.maximum(a[:, None, 0], b[None, :, 0]); y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2]); y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]); ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + ab[None, :] - inter)


def test_config3_session_matches_oracle_chain(session):
    from moseq2_detectron_extract_amd import features as F
    from moseq2_detectron_extract_amd.extract import extract_session
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor, synthetic_state_dict
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import kalman_ref as R
    from oracle import model_ref as MR
    s, d = session
    mcfg = ModelConfig(score_thresh_test=0.0)
    sd = synthetic_state_dict(mcfg, 0)
    pred = Predictor.from_config(mcfg, weights=sd)
    assert pred.model.dtype == "fp32"
    cfg = ExtractConfig(chunk_size=CHUNK, use_tracking=True)
    path = str(d / "depth.dat")
    out = extract_session(path, s.bground_im, s.roi, pred, cfg, true_depth=s.true_depth, output_dir=str(d / "out"))
    assert out["frames"].shape == (N, 80, 80)
    np.testing.assert_array_equal(out["frame_idxs"], np.arange(N))
    written = os.listdir(d / "out")
    assert any(f.startswith("results_00") for f in written) and any(f.endswith(".tsv") for f in written), written

    # the device features of every chunk through the same extractor code
    # (instance tracker carried), then the session's own host step
    raw_all = np.memmap(path, dtype="<i2", mode="r", shape=(N, 424, 512))
    ex = GPUExtractor(s.bground_im, s.roi, pred, cfg)
    states, hosts = [], []
    for c0 in range(0, N, CHUNK):
        st, host = ex.features_pass(torch.from_numpy(np.ascontiguousarray(raw_all[c0:c0 + CHUNK])).cuda())
        ex.select_instances(st, host)
        states.append(st)
        hosts.append(host)
    torch.cuda.synchronize()

    # oracle frame ops on chunk 1
    c, a = 1, CHUNK
    raw = np.ascontiguousarray(raw_all[a:a + CHUNK])
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    np.testing.assert_array_equal(states[c]["prepped"].cpu().numpy(), prepped)
    cl = O.clean_frames(prepped, iters_tail=3)
    np.testing.assert_array_equal(states[c]["cleaned"].cpu().numpy(), cl)
    d2 = states[c]["d2"].cpu().numpy()
    fw = O.get_frame_features(cl, 3, mask=d2)
    np.testing.assert_array_equal(hosts[c]["centroid"], fw["centroid"])
    np.testing.assert_array_equal(hosts[c]["axis_length"], fw["axis_length"])
    np.testing.assert_allclose(hosts[c]["orientation"], fw["orientation"], rtol=0, atol=1e-14)
    assert np.isfinite(fw["centroid"]).all(axis=1).mean() > 0.5  # real contours, not NaN against NaN

    # the host step over the three chunks: restated tracking chain
    Ar, Cr = R.point_tracker_matrices()
    Aa, Ca = R.angle_tracker_matrices()
    rp, ra = R.RefTracker(Ar, Cr), R.RefTracker(Aa, Ca)
    rest = []
    for k, host in enumerate(hosts):
        cen, kp, ori, axl = host["centroid"], host["keypoints"], host["orientation"], host["axis_length"]
        Z = R.point_format(cen, kp[:, :, :2])
        if rp.kf is None:
            rp.initialize(R.point_init_mean(cen, kp[:, :, :2]), Z)
        xs = rp.smooth_update(Z)
        sc = xs[:, 0:6:3]
        wk = np.array(kp, dtype=float)
        wk[:, :7, :2] = xs[:, 6::3].reshape(len(xs), 8, 2)[:, :7]
        ang = F.clamp_angles_deg(-np.rad2deg(ori))
        fl, _ = F.flips_from_keypoints(wk, sc, ang, np.max(axl, axis=1))
        ang[fl] = F.clamp_angles_deg(ang[fl] + 180)
        scores = F.compute_keypoint_alignment_scores(F.rotate_points_batch(np.copy(wk[:, :7, :2]), sc, ang))
        wang, wfl = R.angle_loop_ref(ra, ang, fl, scores)
        sl = slice(k * CHUNK, (k + 1) * CHUNK)
        np.testing.assert_allclose(out["scalars/centroid_x_px"][sl], sc[:, 0], rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(out["scalars/centroid_y_px"][sl], sc[:, 1], rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(np.rad2deg(out["scalars/angle"][sl]), wang, rtol=0, atol=1e-7)
        np.testing.assert_array_equal(out["flips"][sl], wfl)
        rest.append((sc, wk, wang))

    # chunk 1's crops and scalars
    sl = slice(a, a + CHUNK)
    cen_s = np.column_stack([out["scalars/centroid_x_px"][sl], out["scalars/centroid_y_px"][sl]])
    ang_s = np.rad2deg(out["scalars/angle"][sl])
    np.testing.assert_array_equal(out["frames"][sl], O.crop_and_rotate_frames(prepped, cen_s, ang_s))
    np.testing.assert_array_equal(out["frames_mask"][sl], O.crop_and_rotate_frames(d2, cen_s, ang_s))
    sc, wk, wang = rest[c]
    same = (out["frames"][sl] == O.crop_and_rotate_frames(prepped, sc, wang)).all(axis=(1, 2))
    assert same.mean() >= 0.995, same.mean()
    area, hmean, _ = FR.frame_scalars_ref(prepped, d2, 0, 100)
    track = {"centroid": cen_s, "orientation": ang_s, "axis_length": hosts[c]["axis_length"]}
    want = F.compute_scalars(None, track, 0, 100, s.true_depth, reductions=(area, hmean))
    for k in ("area_px", "height_ave_mm", "width_px", "length_px", "velocity_2d_px", "centroid_x_mm"):
        np.testing.assert_array_equal(out[f"scalars/{k}"][sl], want[k], err_msg=k)

    # the model on 32 frames spread over chunk 1 against the oracle forward
    idx = np.arange(0, CHUNK, CHUNK // 32)
    img = O.scale_raw_frames(prepped[idx], 0, 100)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    want, _ = MR.forward(sd, mcfg, img[..., None], keep_intermediates=False)
    got = pred.model.forward(torch.from_numpy(np.ascontiguousarray(img)).cuda())
    nkeep = states[c]["nkeep"]
    for j, i in enumerate(idx):
        w = want[j]
        n = int(got["ndet"][j])
        assert n == len(w["pred_boxes"])
        assert _iou(w["pred_boxes"].numpy(), got["boxes"][j, :n].cpu().numpy()).max(1).min() >= 0.98
        keep = FR.nms_mask_instances(w["pred_masks"].numpy(), w["scores"].numpy())
        if int(nkeep[i]) == 1 and len(keep) == 1:
            wm = w["pred_masks"][keep[0]].numpy()
            diff, union = np.logical_xor(wm, d2[i] > 0).sum(), np.logical_or(wm, d2[i] > 0).sum()
            assert diff <= max(4, 0.03 * union), (i, diff, union)


def test_sessions_share_primed_streams(session):
    """A second session through the same predictor borrows the first one's
    stream set (pipeline._checkout_streams: the model's per-stream
    workspaces, no second priming forward) and gives the same results."""
    from moseq2_detectron_extract_amd import pipeline as P
    from moseq2_detectron_extract_amd.extract import extract_session
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    s, d = session
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), weights="synthetic")
    cfg = P.ExtractConfig(chunk_size=500, use_tracking=True)
    path = str(d / "depth.dat")
    outs = []
    for _ in range(2):
        outs.append(extract_session(path, s.bground_im, s.roi, pred, cfg, true_depth=s.true_depth,
                                    frame_trim=(0, N - 1200)))
        pool = P._STREAM_POOLS[pred]
        assert len(pool) == 1 and pool[0].primed
    assert outs[0].keys() == outs[1].keys()
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_concurrent_sessions_one_predictor(session):
    """Two sessions extracted at once from two threads through one predictor
    borrow two stream sets (pipeline._checkout_streams hands a busy set to
    nobody else; the model keeps a workspace per stream) and give the same
    arrays as one session alone."""
    import threading
    from moseq2_detectron_extract_amd import pipeline as P
    from moseq2_detectron_extract_amd.extract import extract_session
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    s, d = session
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), weights="synthetic")
    cfg = P.ExtractConfig(chunk_size=400, use_tracking=True)
    path = str(d / "depth.dat")
    kw = dict(true_depth=s.true_depth, frame_trim=(0, N - 800))
    want = extract_session(path, s.bground_im, s.roi, pred, cfg, **kw)
    got, errs = [None, None], []

    def run(i):
        try:
            torch.cuda.set_device(0)
            got[i] = extract_session(path, s.bground_im, s.roi, pred, cfg, **kw)
        except BaseException as e:  # surfaced below
            errs.append(e)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert len(P._STREAM_POOLS[pred]) == 2
    for g in got:
        assert g.keys() == want.keys()
        for k in want:
            np.testing.assert_array_equal(g[k], want[k], err_msg=k)
