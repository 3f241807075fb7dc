"""Host-side issue time of the bench step vs its wall time: is the Python /
ctypes launch path keeping ahead of the GPU?  Usage: python tools/hostbench.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor
    B = 32
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype="fp16", seed=0)
    sess = synth.SyntheticSession(2 * B, seed=1000)
    raw = torch.from_numpy(sess.frames(0, 2 * B)).cuda()
    ex = GPUExtractor(sess.bground_im, sess.roi, pred, ExtractConfig(batch_size=B))
    for depth in (1, 2):
        pipe = OverlappedExtractor(ex, depth)
        for i in range(4):
            pipe.submit(raw[(i % 2) * B:(i % 2) * B + B])
        pipe.flush()
        torch.cuda.synchronize()
        n = 20
        host = 0.0
        t0 = time.perf_counter()
        for i in range(n):
            h0 = time.perf_counter()
            pipe.submit(raw[(i % 2) * B:(i % 2) * B + B])
            host += time.perf_counter() - h0
        pipe.flush()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"model streams {depth}: wall {wall / n * 1e3:.2f} ms/step, host issue {host / n * 1e3:.2f} ms/step",
              flush=True)
    # one forward alone, serial
    prepped, cleaned = ex.front(raw[:B])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ex.infer(prepped)
    h = time.perf_counter() - t0
    torch.cuda.synchronize()
    w = time.perf_counter() - t0
    print(f"infer alone: host issue {h / 10 * 1e3:.2f} ms, wall {w / 10 * 1e3:.2f} ms per batch", flush=True)


if __name__ == "__main__":
    main()
