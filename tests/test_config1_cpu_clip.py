"""BASELINE config 1: a 16-frame 512x424 synthetic depth clip through the
CPU path end to end (plumbing, no GPU): the .dat frame source, the oracle's
frame ops and fp32 Mask/Keypoint R-CNN (the CPU statement of the reference's
Detectron2 path), mask NMS + instance 0, clean / moments, the product's host
angle step (no-tracking branch in libmdx host code) and tracking branch,
scalars, keypoint tables, crops, and the result writers -- the h5 tree and
keypoints TSV the reference's ResultWriterStep produces
(M/pipeline/write_results_step.py, M/io/result.py:14-130).  Checks the data
dict keys / dtypes / shapes and the written datasets."""
import os

import numpy as np
import pytest


@pytest.mark.parametrize("use_tracking", [False, True])
def test_sixteen_frame_clip_cpu(mdx, tmp_path, use_tracking):
    import torch
    from moseq2_detectron_extract_amd import features as F
    from moseq2_detectron_extract_amd import results as RS
    from moseq2_detectron_extract_amd import session as S
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd import tracking as TR
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import model_ref as R

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    n = 16
    s = synth.SyntheticSession(n, seed=16)
    s.write(str(tmp_path))
    raw = S.read_frames_raw(str(tmp_path / "depth.dat"))
    assert raw.shape == (n, 424, 512) and raw.dtype == np.int16
    np.testing.assert_array_equal(raw, s.frames(0, n))
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    scaled = O.scale_raw_frames(prepped, 0, 100)
    cfg = ModelConfig(score_thresh_test=0.5, detections_per_image=4)
    sd = synthetic_state_dict(cfg, 0)
    res, _ = R.forward(sd, cfg, scaled[..., None], keep_intermediates=False)
    assert len(res) == n
    h, w = prepped.shape[1:]
    d2 = np.zeros((n, h, w), np.uint8)
    kp = np.full((n, 8, 3), np.nan)
    nins = np.zeros(n, np.int64)
    for i, r in enumerate(res):
        assert r["pred_masks"].shape[1:] == (h, w) and r["pred_keypoints"].shape[1:] == (8, 3)
        keep = FR.nms_mask_instances(r["pred_masks"].numpy(), r["scores"].numpy())
        nins[i] = len(keep)
        if keep:
            d2[i] = r["pred_masks"][keep[0]].numpy()
            kp[i] = r["pred_keypoints"][keep[0]].numpy()
    cleaned = O.clean_frames(prepped, iters_tail=3)
    feats = O.get_frame_features(cleaned, 3, mask=d2)
    if use_tracking:
        p, a = TR.make_trackers()
        cen, kp2, ang, flips = TR.track_features(p, a, feats["centroid"], kp, feats["orientation"],
                                                 feats["axis_length"])
    else:
        ang, flips = F.finalize_angles(feats["orientation"], feats["axis_length"], feats["centroid"], kp)
        cen, kp2 = feats["centroid"], kp
    assert ang.shape == (n,) and flips.dtype == bool
    area, hmean, z = FR.frame_scalars_ref(prepped, d2, 0, 100, keypoints=kp2, z_frames=cleaned)
    track = {"centroid": cen, "orientation": ang, "axis_length": feats["axis_length"]}
    scalars = F.compute_scalars(None, track, 0, 100, s.true_depth, reductions=(area, hmean))
    kpd = F.keypoints_to_dict(kp2, None, cen, ang, true_depth=s.true_depth, z_data=z)
    depth = O.crop_and_rotate_frames(prepped, cen, ang)
    mask = O.crop_and_rotate_frames(d2, cen, ang)
    data = {"chunk": prepped, "frame_idxs": np.arange(n), "offset": 0,
            "features": {"cleaned_frames": cleaned, "masks": d2, "features": track, "flips": flips,
                         "keypoints": kp2, "num_instances": nins},
            "scalars": scalars, "keypoints": kpd, "depth_frames": depth, "mask_frames": mask}
    assert set(data["scalars"]) == set(F.scalar_attributes())
    assert set(data["keypoints"]) == set(F.keypoint_attributes())
    assert depth.shape == (n, 80, 80) and depth.dtype == np.uint8 and mask.dtype == np.uint8
    # writers: h5 tree (npz without h5py) + keypoints TSV
    out = tmp_path / "out"
    out.mkdir()
    hf = RS.open_results(str(out))
    RS.create_extract_h5(hf, {"nframes": n, "crop_size": (80, 80), "frame_dtype": "uint8",
                              "timestamps": np.arange(n) * (1000 / 30), "flip_classifier": "keypoints",
                              "true_depth": s.true_depth, "roi": s.roi, "first_frame": raw[0],
                              "bground_im": s.bground_im},
                         {"uuid": "clip16", "parameters": {"chunk_size": n}, "metadata": {}})
    RS.write_extracted_chunk_to_h5(hf, data)
    tsv = RS.KeypointsTSVWriter(str(out))
    tsv.write(data)
    hf.close()
    saved = dict(np.load(str(out / "results_00.npz"))) if (out / "results_00.npz").exists() else None
    if saved is not None:
        np.testing.assert_array_equal(saved["frames"], depth)
        np.testing.assert_array_equal(saved["frames_mask"], mask.astype(bool))
        np.testing.assert_array_equal(saved["metadata/extraction/flips"], flips)
        np.testing.assert_array_equal(saved["scalars/centroid_x_px"], np.asarray(cen[:, 0], np.float32))
    assert (out / "keypoints_00.tsv").read_text().count("\n") == n + 1
