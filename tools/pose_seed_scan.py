"""Pick the seeded synthetic weights of tests/test_parity_full.py: per weight
seed, the number of the batch's frames whose ORACLE chain carries a non-NaN
pose (selected mask -> clean -> moments), i.e. frames the full-frame parity
test compares downstream.  CPU only (oracle/), the test's session seed.
Usage: python tools/pose_seed_scan.py DEPTH B wseed [wseed ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, synthetic_state_dict
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import model_ref as R
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    depth, B = int(sys.argv[1]), int(sys.argv[2])
    s = synth.SyntheticSession(B, seed=77)
    raw = s.frames(0, B)
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    scaled = O.scale_raw_frames(prepped, 0, 100)
    cl = O.clean_frames(prepped, iters_tail=3)
    for ws in (int(v) for v in sys.argv[3:]):
        cfg = ModelConfig(depth=depth, score_thresh_test=0.0)
        sd = synthetic_state_dict(cfg, ws)
        d2 = np.zeros(prepped.shape, np.uint8)
        nkeep, near = [], []
        try:
            for a in range(0, B, 8):
                w, _ = R.forward(sd, cfg, scaled[a:a + 8, ..., None])
                for j, x in enumerate(w):
                    keep = FR.nms_mask_instances(x["pred_masks"].numpy(), x["scores"].numpy()) \
                        if len(x["scores"]) else []
                    nkeep.append(len(keep))
                    if keep:
                        d2[a + j] = x["pred_masks"][keep[0]].numpy()
                        # pixels of the selected mask's pasted probability this close to the
                        # 0.5 threshold: where an fp32 rounding difference can flip a pixel
                        p = x["pred_mask_probs"][keep[0]].numpy()
                        near.append(int((np.abs(p - 0.5) < 1e-5).sum()))
                    else:
                        near.append(0)
        except Exception as e:  # a seed the oracle chain cannot run (e.g. no detection at all)
            print(json.dumps({"depth": depth, "B": B, "wseed": ws, "error": repr(e)[:200]}), flush=True)
            continue
        fw = O.get_frame_features(cl, 3, mask=d2)
        ok = np.isfinite(fw["centroid"][:, 0])
        # pose sensitivity: flip each near-threshold pixel of the selected mask
        # alone and re-measure the oracle pose (a frame whose angle moves by
        # more than the fp32 tolerance of tests/test_parity_full.py -- 1 deg --
        # or whose centroid moves by more than 0.5 px fails there as soon as
        # the GPU rounds that pixel the other way)
        risky = []
        for f in range(B):
            if not near[f] or not ok[f]:
                continue
            ang0 = np.rad2deg(fw["orientation"][f])
            worst = 0.0
            # the near pixels of frame f (recomputed from its oracle probabilities)
            w, _ = R.forward(sd, cfg, scaled[f:f + 1, ..., None])
            keep = FR.nms_mask_instances(w[0]["pred_masks"].numpy(), w[0]["scores"].numpy())
            p = w[0]["pred_mask_probs"][keep[0]].numpy()
            for yx in np.argwhere(np.abs(p - 0.5) < 1e-5)[:16]:
                m = d2[f:f + 1].copy()
                m[0, yx[0], yx[1]] ^= 1
                g = O.get_frame_features(cl[f:f + 1], 3, mask=m)
                da = abs(((np.rad2deg(g["orientation"][0]) - ang0) + 90) % 180 - 90)
                dc = float(np.abs(g["centroid"][0] - fw["centroid"][f]).max())
                worst = max(worst, da if dc <= 0.5 else 999.0)
            if worst > 1.0:
                risky.append([f, round(worst, 3)])
        print(json.dumps({"depth": depth, "B": B, "wseed": ws, "non_nan_poses": int(ok.sum()),
                          "nkeep_hist": np.bincount(nkeep, minlength=5).tolist(),
                          "frames_with_near_threshold_px": int((np.asarray(near) > 0).sum()),
                          "pose_risky_frames": risky,
                          "near_threshold_px": near,
                          "mask_px": [int(v) for v in d2.reshape(B, -1).sum(1)]}), flush=True)


if __name__ == "__main__":
    main()
