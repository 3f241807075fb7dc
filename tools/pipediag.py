"""Which stage differs between the multi-stream pipeline and the serial step?
Usage: python tools/pipediag.py [model_streams] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor
    ms = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    s = synth.SyntheticSession(12, seed=5)
    raw = torch.from_numpy(s.frames(0, 12)).cuda()
    pred = Predictor.from_config(ModelConfig(score_thresh_test=0.0), dtype="fp16")
    ex = GPUExtractor(s.bground_im, s.roi, pred, ExtractConfig(batch_size=4))
    batches = [raw[i:i + 4] for i in range(0, 12, 4)]
    want = [ex.step_device(b) for b in batches]
    wantinf = [ex.infer(ex.prep(b)) for b in batches]
    torch.cuda.synchronize()
    stash = []
    orig_infer = ex.infer

    def spy(prepped):
        o = orig_infer(prepped)
        stash.append((prepped, o))
        return o
    for rep in range(reps):
        stash.clear()
        ex.infer = spy
        pipe = OverlappedExtractor(ex, ms)
        got = [r for r in (pipe.submit(b) for b in batches) if r is not None]
        got.extend(pipe.flush())
        torch.cuda.synchronize()
        bad = []
        for bi, (w, g) in enumerate(zip(want, got)):
            for k in ("depth_frames", "mask_frames", "centroid", "angle", "keypoints", "ndet"):
                if not torch.equal(torch.nan_to_num(g[k].float(), 7.0), torch.nan_to_num(w[k].float(), 7.0)):
                    bad.append((bi, k))
        ex.infer = orig_infer
        for bi, (pp, o) in enumerate(stash):
            w = wantinf[bi]
            diff = [k for k in ("boxes", "scores", "ndet", "keypoints", "d2_mask", "sel_keypoints") if not torch.equal(
                torch.nan_to_num(o[k].float(), 7.0), torch.nan_to_num(w[k].float(), 7.0))]
            pw = ex.prep(batches[bi])
            if not torch.equal(pp, pw):
                diff.append("prepped")
            if diff:
                bad.append((bi, "infer", diff))
        print(f"streams {ms} rep {rep}: mismatches {bad}", flush=True)
    # serial repeatability of the forward itself
    again = [ex.infer(ex.prep(b)) for b in batches]
    torch.cuda.synchronize()
    for bi, (a, b) in enumerate(zip(wantinf, again)):
        diff = [k for k in ("boxes", "scores", "d2_mask", "sel_keypoints") if not torch.equal(
            torch.nan_to_num(a[k].float(), 7.0), torch.nan_to_num(b[k].float(), 7.0))]
        print(f"serial infer repeat batch {bi}: differs in {diff}", flush=True)


if __name__ == "__main__":
    main()
