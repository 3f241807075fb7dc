"""Instance selection across frames: the product's
norfair-semantics tracker (moseq2_detectron_extract_amd.instances) against the
object-level restatement in oracle/norfair_ref.py.  Parity unpinned against
norfair itself (absent, unpinned; see the oracle's header)."""
import numpy as np
import pytest

import mdx_pkg

mdx_pkg.load()
from moseq2_detectron_extract_amd import instances as I  # noqa: E402
from oracle import norfair_ref as R  # noqa: E402


def _scenario(seed, n=400, max_det=4):
    """Per frame a list of (id, centre): 1-3 'animals' on random walks (some
    leaving and re-entering), occasional spurious detections, jumps, empty
    frames and duplicate detections of one animal."""
    rng = np.random.default_rng(seed)
    na = int(rng.integers(1, 4))
    pos = rng.uniform(50, 400, (na, 2))
    present = np.ones(na, bool)
    frames = []
    for f in range(n):
        pos += rng.normal(0, 4, pos.shape)
        if rng.random() < 0.02:
            pos[rng.integers(na)] += rng.normal(0, 80, 2)  # a jump past the threshold
        flip = rng.random(na) < 0.03
        present ^= flip
        dets = [pos[a].copy() for a in range(na) if present[a]]
        if rng.random() < 0.1:
            dets.append(rng.uniform(0, 450, 2))  # spurious
        if dets and rng.random() < 0.05:
            dets.append(dets[0] + rng.normal(0, 2, 2))  # duplicate of one animal
        if rng.random() < 0.03:
            dets = []
        rng.shuffle(dets)
        frames.append([((f, s), c) for s, c in enumerate(dets[:max_det])])
    return frames


def _product(frames, expected=1):
    """The per-frame Python statement."""
    tr = I.InstanceTrackerPy(expected)
    out = []
    for dets in frames:
        sel = tr.select([c for _, c in dets], [i for i, _ in dets])
        out.append([i for i, _ in dets] if sel is None else sel)
    return out


def _native(frames, expected=1, chunk=97, D=4):
    """The native tracker, chunk by chunk (state carried)."""
    tr = I.InstanceTracker(expected)
    out = []
    for c0 in range(0, len(frames), chunk):
        fr = frames[c0:c0 + chunk]
        nk = np.array([len(d) for d in fr])
        cen = np.full((len(fr), D, 2), np.nan)
        for f, d in enumerate(fr):
            for s, (_, c) in enumerate(d):
                cen[f, s] = c
        ch = I.select_chunk(tr, nk, cen, c0)
        out.extend(ch.get(f, [(c0 + f, s) for s in range(nk[f])]) for f in range(len(fr)))
    return out


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("expected", [1, 2])
def test_tracker_matches_restatement(seed, expected):
    frames = _scenario(seed)
    ref = R.select_instances(frames, expected)
    assert _product(frames, expected) == ref
    assert _native(frames, expected) == ref


def test_selection_changes_something():
    """The scenarios exercise the non-identity branch, including picks of an
    earlier frame's detection."""
    changed = older = 0
    for seed in range(12):
        frames = _scenario(seed)
        for f, (dets, sel) in enumerate(zip(frames, _product(frames))):
            if sel != [i for i, _ in dets]:
                changed += 1
                older += any(i[0] != f for i in sel)
    assert changed > 50 and older > 0


def test_single_animal_is_identity():
    rng = np.random.default_rng(3)
    p = np.array([200.0, 200.0])
    frames = []
    for f in range(300):
        p += rng.normal(0, 3, 2)
        frames.append([((f, 0), p.copy())] if rng.random() > 0.05 else [])
    assert _product(frames) == [[i for i, _ in d] for d in frames]


def test_select_chunk_carries_state():
    """select_chunk over two chunks == one pass over the session."""
    frames = _scenario(5, n=300)
    D = 4
    n = len(frames)
    nkeep = np.array([len(d) for d in frames])
    cen = np.full((n, D, 2), np.nan)
    for f, d in enumerate(frames):
        for s, (_, c) in enumerate(d):
            cen[f, s] = c
    tr = I.InstanceTrackerPy(1)
    ch = I.select_chunk(tr, nkeep[:150], cen[:150], 0)
    ch.update({f + 150: v for f, v in I.select_chunk(tr, nkeep[150:], cen[150:], 150).items()})
    ref = R.select_instances(frames, 1)
    for f in range(n):
        want = ref[f]
        got = ch.get(f, [(f, s) for s in range(nkeep[f])])
        assert got == want, f


def test_center_of_mass_restatement():
    from scipy import ndimage
    rng = np.random.default_rng(0)
    m = rng.random((37, 53)) < 0.2
    assert np.array_equal(R.center_of_mass(m), np.array(ndimage.center_of_mass(m)))


# ----------------------------------------------------------------- GPU path
def _disc_masks(rng, B, D, h, w):
    """Frames of <= D disc masks: two animals on random walks, a shifted
    duplicate of the first (suppressed by mask NMS), a random spurious disc,
    and now and then an empty mask (box-centre fallback)."""
    yy, xx = np.mgrid[:h, :w]
    rad = 36 if h < 100 else 900
    masks = np.zeros((B, D, h, w), np.uint8)
    scores = np.zeros((B, D), np.float32)
    boxes = np.zeros((B, D, 4), np.float32)
    ndet = np.zeros(B, np.int32)
    a = np.array([20.0, 30.0])
    b = np.array([40.0, 70.0])
    for f in range(B):
        a = np.clip(a + rng.normal(0, 2, 2), 8, [h - 8, w - 8])
        b = np.clip(b + rng.normal(0, 2, 2), 8, [h - 8, w - 8])
        cands = [(a, 0.9), (b, 0.8) if rng.random() < 0.7 else None, (a + 2, 0.7),
                 (rng.uniform(8, [h - 8, w - 8]), 0.6) if rng.random() < 0.3 else None]
        cands = [c for c in cands if c is not None][: int(rng.integers(0, D + 1))]
        for s, (c, sc) in enumerate(cands):
            if rng.random() > 0.05:
                masks[f, s] = ((yy - c[0]) ** 2 + (xx - c[1]) ** 2 <= rad).astype(np.uint8)
            scores[f, s] = sc
            boxes[f, s] = [c[1] - 6, c[0] - 6, c[1] + 6.5, c[0] + 6.5]
        ndet[f] = len(cands)
    return masks, scores, boxes, ndet


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(64, 96), (64, 101), (37, 53), (423, 511)])
def test_mask_centers_kernel(h, w):
    """Bit-exact vs scipy's center_of_mass formula: rows a multiple of 16 B,
    16-B words wrapping onto the next row (w = 101, 511), and unaligned planes
    (h*w % 16 != 0: the byte path)."""
    import torch
    from moseq2_detectron_extract_amd.pipeline import mask_centers, mask_nms_select
    rng = np.random.default_rng(1)
    B, D, K = (48 if h < 100 else 6), 4, 8
    masks, scores, boxes, ndet = _disc_masks(rng, B, D, h, w)
    out = {"masks": torch.from_numpy(masks).cuda(), "scores": torch.from_numpy(scores).cuda(),
           "ndet": torch.from_numpy(ndet).cuda(), "boxes": torch.from_numpy(boxes).cuda(),
           "keypoints": torch.zeros((B, D, K, 3), dtype=torch.float32, device="cuda")}
    _, _, nkeep, keep = mask_nms_select(out, 0.5)
    cen = mask_centers(out, keep, nkeep).cpu().numpy()
    nkeep, keep = nkeep.cpu().numpy(), keep.cpu().numpy()
    fallback = 0
    for f in range(B):
        for s in range(D):
            if s >= nkeep[f]:
                assert np.isnan(cen[f, s]).all()
                continue
            j = keep[f, s]
            if masks[f, j].any():
                want = R.center_of_mass(masks[f, j])
            else:
                bx = boxes[f, j]
                want = np.array([(bx[0] + bx[2]) / np.float32(2), (bx[1] + bx[3]) / np.float32(2)], np.float64)
                fallback += 1
            assert np.array_equal(cen[f, s], want), (f, s)
    assert fallback > 0 or h > 100


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,bs,host_tail", [(48, 16, False), (2, 2, False), (3, 1, True), (48, 16, True)])
def test_extractor_select_instances_two_chunks(chunk, bs, host_tail):
    """GPUExtractor.select_instances over a session of chunks (tracker state
    and the preceding chunks' last detections carried) == the oracle's
    selection.  chunk < POINTWISE_HIT_COUNTER_MAX: a pick can refer to a frame
    two chunks back (the merged tail).  host_tail: the carried planes live in
    host memory, as pass_tail_forward receives them over a gloo group -- a
    cross-chunk pick must still reach the device gather."""
    import torch
    from moseq2_detectron_extract_amd.pipeline import (ExtractConfig, GPUExtractor, mask_centers,
                                                         mask_nms_select)
    rng = np.random.default_rng(2)
    B, D, h, w, K = 96, 4, 64, 96, 8
    masks, scores, boxes, ndet = _disc_masks(rng, B, D, h, w)
    kps = rng.normal(0, 10, (B, D, K, 3)).astype(np.float32)
    ex = GPUExtractor.__new__(GPUExtractor)
    ex.cfg = ExtractConfig()
    ex.instance_tracker = I.InstanceTracker(1)
    ex._frames_seen, ex._tail_dets = 0, {}
    frames, got_d2, got_kp, got_n = [], [], [], []
    for c0 in range(0, B, chunk):
        if host_tail:
            ex._tail_dets = {g: (p.cpu(), k, r) for g, (p, k, r) in ex._tail_dets.items()}
        outs = []
        for i in range(c0, c0 + chunk, bs):
            o = {"masks": torch.from_numpy(masks[i:i + bs]).cuda(), "scores": torch.from_numpy(scores[i:i + bs]).cuda(),
                 "ndet": torch.from_numpy(ndet[i:i + bs]).cuda(), "boxes": torch.from_numpy(boxes[i:i + bs]).cuda(),
                 "keypoints": torch.from_numpy(kps[i:i + bs]).cuda()}
            sel, kp, nk, keep = mask_nms_select(o, 0.5)
            o.update(d2_mask=sel, sel_keypoints=kp, nkeep=nk, keep_idx=keep, centers=mask_centers(o, keep, nk))
            outs.append(o)
        keys = ("keypoints", "d2_mask", "sel_keypoints", "nkeep", "keep_idx", "centers")
        inf = {k: torch.cat([o[k] for o in outs]) for k in keys} | {"masks": [o["masks"] for o in outs]}
        keep_h, nk_h, cen_h = inf["keep_idx"].cpu().numpy(), inf["nkeep"].cpu().numpy(), inf["centers"].cpu().numpy()
        for f in range(chunk):
            frames.append([((c0 + f, keep_h[f, s]), cen_h[f, s]) for s in range(nk_h[f])])
        # what features_pass hands to the host step (moments of a blank frame)
        state = {"d2": inf["d2_mask"], "cleaned": torch.zeros_like(inf["d2_mask"]), "nkeep": nk_h,
                 "inf": {k: inf[k] for k in ("masks", "keypoints", "keep_idx", "sel_keypoints")}}
        host = {"centers": cen_h, "keypoints": inf["sel_keypoints"].cpu().numpy()}
        ex.select_instances(state, host)
        got_n.append(state["nkeep"])
        got_d2.append(state["d2"].cpu().numpy())
        got_kp.append(host["keypoints"])
    got_d2, got_kp, got_n = np.concatenate(got_d2), np.concatenate(got_kp), np.concatenate(got_n)
    ref = R.select_instances(frames, 1)
    changed = 0
    for f in range(B):
        sel = ref[f]
        assert got_n[f] == len(sel), f
        if sel:
            g, j = sel[0]
            changed += not frames[f] or (g, j) != frames[f][0][0]
            assert np.array_equal(got_d2[f], masks[g, j]), f
            assert np.array_equal(got_kp[f], kps[g, j].astype(np.float64)), f
        else:
            assert not got_d2[f].any() and np.isnan(got_kp[f]).all(), f
    assert changed > 0
