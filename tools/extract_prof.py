"""Per-stage wall time of process_chunk on a synthetic chunk (sync at each
stage boundary).  Usage: python tools/extract_prof.py [chunk] [tracking]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    tracking = bool(int(sys.argv[2])) if len(sys.argv) > 2 else False
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
    s = synth.SyntheticSession(n, seed=9)
    raw = torch.from_numpy(s.frames(0, n)).cuda()
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype="fp16")
    ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(chunk_size=n, use_tracking=tracking))
    for rep in range(3):
        T = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prepped = ex.prep(raw)
        torch.cuda.synchronize(); t1 = time.perf_counter(); T["prep"] = t1 - t0
        inf = ex.infer(prepped)
        torch.cuda.synchronize(); t2 = time.perf_counter(); T["infer"] = t2 - t1
        cleaned, feats = ex.features(prepped, inf["d2_mask"])
        torch.cuda.synchronize(); t3 = time.perf_counter(); T["clean+moments"] = t3 - t2
        host = {"centroid": feats["centroid"].cpu().numpy(), "orientation": feats["orientation"].cpu().numpy(),
                "axis_length": feats["axis_length"].cpu().numpy(), "keypoints": inf["sel_keypoints"].cpu().numpy()}
        t4 = time.perf_counter(); T["d2h"] = t4 - t3
        cen, kp, ang, fl = ex.host_angles(host)
        t5 = time.perf_counter(); T["host_angles"] = t5 - t4
        st = {"prepped": prepped, "d2": inf["d2_mask"], "cleaned": cleaned, "nkeep": inf["nkeep"].cpu().numpy()}
        d = ex.finish_chunk(st, cen, kp, ang, fl, host["axis_length"], None, 0, s.true_depth)
        torch.cuda.synchronize(); t6 = time.perf_counter(); T["finish"] = t6 - t5
        tot = t6 - t0
        print(f"rep {rep}: total {tot*1e3:.0f} ms ({n/tot:.0f} fps): " +
              " ".join(f"{k} {v*1e3:.0f}" for k, v in T.items()), flush=True)


if __name__ == "__main__":
    main()
