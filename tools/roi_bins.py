"""Tap-count histogram of the box pooler on the bench workload: the model's
proposals for one 32-frame batch (R50-FPN, synthetic session), each assigned
to its pyramid level as the pooler does, and per bin the number of map rows /
columns its adaptive sample grid touches (the (nr, nc) of k_roi_align_sep).
Usage: python tools/roi_bins.py"""
import collections
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def axis_taps(start, size, P, n, extent):
    """rows (or columns) touched by each of the P bins along one axis"""
    out = []
    for p in range(P):
        lo = hi = None
        for i in range(n):
            v = start + p * size + (i + 0.5) * size / n
            if v < -1.0 or v > extent:
                continue
            v = max(v, 0.0)
            l = int(math.floor(v))
            if l >= extent - 1:
                l = h = extent - 1
            else:
                h = l + 1
            lo = l if lo is None else min(lo, l)
            hi = h if hi is None else max(hi, h)
        out.append(0 if lo is None else hi - lo + 1)
    return out


def main():
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import proc, synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    cfg = ModelConfig(score_thresh_test=0.0)
    m = Predictor.from_config(cfg, dtype="fp32", seed=0, weights="synthetic").model
    sess = synth.SyntheticSession(32, seed=1000)
    raw = torch.from_numpy(sess.frames(0, 32)).cuda()
    prepped = proc.FramePrep(sess.bground_im, sess.roi, 0, 100, True)(raw)
    it = m.forward(prepped, proc.scale_lut(0, 100), intermediates=True)["intermediates"]
    props = it["proposals"].reshape(32, -1, 4).cpu().numpy()
    cnt = it["proposal_count"].reshape(-1).cpu().numpy()
    sizes = {2: (112, 128), 3: (56, 64), 4: (28, 32), 5: (14, 16)}
    hist = collections.Counter()
    levels = collections.Counter()
    for b in range(32):
        for x1, y1, x2, y2 in props[b, :int(cnt[b])]:
            s = math.sqrt(max((x2 - x1) * (y2 - y1), 0.0))
            lv = int(min(max(math.floor(4 + math.log2(s / 224 + 1e-8)), 2), 5)) if s > 0 else 2
            levels[lv] += 1
            sc = 1.0 / 2 ** lv
            H, W = sizes[lv]
            rs_w, rs_h = x1 * sc - 0.5, y1 * sc - 0.5
            bw, bh = (x2 - x1) * sc / 7, (y2 - y1) * sc / 7
            gh, gw = max(1, math.ceil(bh)), max(1, math.ceil(bw))
            rows = axis_taps(rs_h, bh, 7, gh, H)
            cols = axis_taps(rs_w, bw, 7, gw, W)
            for r in rows:
                for c in cols:
                    hist[(r, c)] += 1
    tot = sum(hist.values())
    print(json.dumps({"levels": dict(levels), "bins": tot}))
    for (r, c), n in sorted(hist.items(), key=lambda kv: -kv[1])[:20]:
        print(json.dumps({"nr": r, "nc": c, "frac": round(n / tot, 4)}))
    le3 = sum(n for (r, c), n in hist.items() if r <= 3 and c <= 3) / tot
    le4 = sum(n for (r, c), n in hist.items() if r <= 4 and c <= 4) / tot
    print(json.dumps({"frac_le_3x3": round(le3, 4), "frac_le_4x4": round(le4, 4)}))


if __name__ == "__main__":
    main()
