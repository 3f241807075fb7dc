"""Soak test of the stream-pipelined loop: every output of OverlappedExtractor
(5 streams, two forwards in flight, frame stages beside them) compared bit
for bit with the serial step on the same batch, over many steps.
Usage: python tools/determinism.py [fp32|fp16] [steps] [batch] [model_streams]
(DET_SPLIT=6: the fp32 layers as bf16 plane products, set before the handle
is created so it carries the weight planes)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    ms = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor
    nb = 4
    s = synth.SyntheticSession(nb * B, seed=21)
    raw = torch.from_numpy(s.frames(0, nb * B)).cuda()
    batches = [raw[i * B:(i + 1) * B] for i in range(nb)]
    if os.environ.get("DET_SPLIT"):
        from moseq2_detectron_extract_amd._lib import call
        from moseq2_detectron_extract_amd._lib import knob
        knob("fp32_split", int(os.environ["DET_SPLIT"]))
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype=dtype, weights="synthetic")
    ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(batch_size=B))
    keys = ("depth_frames", "mask_frames", "centroid", "angle", "keypoints", "ndet")
    want = []
    for b in batches:
        r = ex.step_device(b)
        torch.cuda.synchronize()
        want.append({k: r[k].clone() for k in keys})
    pipe = OverlappedExtractor(ex, ms)
    pipe.prime(batches[0])
    bad, done, t0 = [], 0, time.time()

    def check(r):
        nonlocal done
        w = want[done % nb]
        torch.cuda.current_stream().wait_event(r["ready"])
        diff = [k for k in keys if not torch.equal(torch.nan_to_num(r[k].double(), nan=-7.0),
                                                   torch.nan_to_num(w[k].double(), nan=-7.0))]
        if diff:
            bad.append((done, diff))
        done += 1

    for i in range(steps):
        r = pipe.submit(batches[i % nb])
        if r is not None:
            check(r)
        if i % 50 == 49:
            print(json.dumps({"dtype": dtype, "steps": done, "mismatches": len(bad), "s": round(time.time() - t0, 1)}),
                  flush=True)
    for r in pipe.flush():
        check(r)
    torch.cuda.synchronize()
    print(json.dumps({"dtype": dtype, "batch": B, "steps": done, "mismatches": len(bad), "first": bad[:5],
                      "s": round(time.time() - t0, 1)}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
