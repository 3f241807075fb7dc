import os, sys, time, json, tempfile
sys.path.insert(0, '/root/repo')
import numpy as np, torch, mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd import synth, pipeline
from moseq2_detectron_extract_amd.extract import extract_session
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor
T = {"features_pass": [], "host_angles": [], "finish_chunk": []}
for name in T:
    orig = getattr(GPUExtractor, name)
    def wrap(self, *a, _o=orig, _n=name, **k):
        t = time.perf_counter(); r = _o(self, *a, **k); T[_n].append(round((time.perf_counter() - t) * 1e3, 1)); return r
    setattr(GPUExtractor, name, wrap)
n = 3000
s = synth.SyntheticSession(n, seed=9)
pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype="fp16")
with tempfile.TemporaryDirectory(dir="/tmp") as td:
    s.write(td)
    path = os.path.join(td, "depth.dat")
    extract_session(path, s.bground_im, s.roi, pred, ExtractConfig(chunk_size=64, use_tracking=False), true_depth=s.true_depth, frame_trim=(0, n - 64))
    for k in T: T[k].clear()
    t0 = time.perf_counter()
    extract_session(path, s.bground_im, s.roi, pred, ExtractConfig(chunk_size=1000, use_tracking=False), true_depth=s.true_depth)
    print("total ms", (time.perf_counter() - t0) * 1e3)
    print(json.dumps(T))
