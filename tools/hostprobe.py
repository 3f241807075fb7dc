"""Host-side issue timing of the overlapped pipeline: per submit, the time
spent issuing tail / model / front (no synchronisation inside the loop), to
see whether the host blocks."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mdx_pkg  # noqa: E402

mdx_pkg.load()
from moseq2_detectron_extract_amd import synth  # noqa: E402
from moseq2_detectron_extract_amd.model import ModelConfig, Predictor  # noqa: E402
from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor  # noqa: E402

B = 32
pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype="fp16", seed=0)
sess = synth.SyntheticSession(2 * B, seed=1000)
raw_all = torch.from_numpy(sess.frames(0, 2 * B)).cuda()
ex = GPUExtractor(sess.bground_im, sess.roi, pred, ExtractConfig(batch_size=B))
pipe = OverlappedExtractor(ex, int(sys.argv[1]) if len(sys.argv) > 1 else 2)
T = {"tail": [], "model": [], "front": []}
orig = {k: getattr(pipe, "_" + k) for k in T}


def wrap(k):
    def f(*a):
        t = time.perf_counter()
        r = orig[k](*a)
        T[k].append(time.perf_counter() - t)
        return r
    return f


for k in T:
    setattr(pipe, "_" + k, wrap(k))
for i in range(6):
    pipe.submit(raw_all[(i % 2) * B:(i % 2) * B + B])
pipe.flush()
torch.cuda.synchronize()
for k in T:
    T[k].clear()
t0 = time.perf_counter()
sub = []
for i in range(30):
    a = time.perf_counter()
    pipe.submit(raw_all[(i % 2) * B:(i % 2) * B + B])
    sub.append(time.perf_counter() - a)
pipe.flush()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"issue loop {1e3 * (t1 - t0) / 30:.2f} ms/step, wall {1e3 * (t2 - t0) / 30:.2f} ms/step")
print("submit ms:", " ".join(f"{1e3 * s:.1f}" for s in sub))
for k, v in T.items():
    print(k, "ms:", " ".join(f"{1e3 * s:.1f}" for s in v[:30]))
