"""Full extract loop (BASELINE config 3 shape) on one GPU: a synthetic session
written as depth.dat, then extract.extract_session chunk by chunk (frame
source -> device hot path -> host angle / tracking step -> crops, scalars,
keypoints).  Prints frames/s with tracking off and on.
Usage: python tools/extract_bench.py [nframes] [chunk] [fp32|fp16] [model_streams]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    dtype = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    streams = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.extract import extract_session
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig
    s = synth.SyntheticSession(n, seed=9)
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dtype, weights="synthetic")
    res = {"nframes": n, "chunk": chunk, "dtype": dtype, "model_streams": streams}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        t0 = time.perf_counter()
        s.write(td)
        res["write_s"] = round(time.perf_counter() - t0, 2)
        path = os.path.join(td, "depth.dat")
        # warm-up on a short prefix (model plans, allocator)
        extract_session(path, s.bground_im, s.roi, pred, ExtractConfig(chunk_size=64, use_tracking=False),
                        true_depth=s.true_depth, frame_trim=(0, n - 64))
        for rep in range(int(os.environ.get("EXTRACT_REPS", "2"))):
            for overlap in (True,) if os.environ.get("EXTRACT_OVERLAP_ONLY") else (False, True):
                for tracking in (False, True):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    out = extract_session(path, s.bground_im, s.roi, pred,
                                          ExtractConfig(chunk_size=chunk, use_tracking=tracking, overlap_host=overlap,
                                                        model_streams=streams),
                                          true_depth=s.true_depth)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    assert out["frames"].shape[0] == n
                    res[f"overlap{int(overlap)}_tracking{int(tracking)}_fps_{rep}"] = round(n / dt, 1)
                    print(json.dumps(res), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
