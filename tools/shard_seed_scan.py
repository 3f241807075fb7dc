"""Pick synthetic sessions for tests/test_shard_gpu.py: per (session seed,
weight seed), the fraction of frames with a non-NaN centroid and the number
of frames after the rank boundary whose instance pick names a frame before
it (the tail hand-off between ranks), one process, the test's chunking.
Usage: python tools/shard_seed_scan.py NFR CHUNK BOUNDARY seed[:wseed] ..."""
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
    from moseq2_detectron_extract_amd.instances import InstanceTracker, select_chunk
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
    nfr, chunk, bnd = (int(v) for v in sys.argv[1:4])
    preds = {}
    for spec in sys.argv[4:]:
        seed, wseed = (int(v) for v in (spec.split(":") + ["0"])[:2])
        if wseed not in preds:
            preds[wseed] = Predictor.from_config(ModelConfig(score_thresh_test=0.0), weights="synthetic", seed=wseed)
        s = synth.SyntheticSession(nfr, seed=seed)
        ex = GPUExtractor(s.bground_im, s.roi, preds[wseed],
                          ExtractConfig(chunk_size=chunk, batch_size=16, use_tracking=True, select_instances=True))
        raw = torch.from_numpy(s.frames(0, nfr)).cuda()
        tr = InstanceTracker(1)
        cen_ok, cross, nk_all, changes, trk_ok = 0, 0, [], 0, 0
        for a in range(0, nfr, chunk):
            st, host = ex.features_pass(raw[a:a + chunk])
            cen_ok += int(np.isfinite(host["centroid"][:, 0]).sum())
            nk = st["nkeep"]
            nk_all.extend(nk.tolist())
            ch = select_chunk(tr, nk, host["centers"], a)
            cen_t = ex.host_angles(host)[0]  # the Kalman tracking branch (pre-selection features)
            trk_ok += int(np.isfinite(cen_t[:, 0]).sum())
            changes += len(ch)
            cross += sum(1 for f, sel in ch.items() if a + f >= bnd and any(g < bnd for g, _ in sel))
        print(json.dumps({"seed": seed, "wseed": wseed, "centroid_frac": round(cen_ok / nfr, 3),
                          "tracked_centroid_frac": round(trk_ok / nfr, 3),
                          "nkeep_hist": np.bincount(nk_all, minlength=5).tolist(), "changed_frames": changes,
                          "cross_boundary_picks": cross}), flush=True)


if __name__ == "__main__":
    main()
