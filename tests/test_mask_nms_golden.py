"""Mask-IoU NMS + instance 0 (A14/A16) against fixtures produced by the
reference's own ProcessFeaturesStep.__nms_mask_instances
(M/pipeline/process_features_step.py:63-113; tests/golden/make_golden_nms.py
runs it under stubs): empty masks dropped, duplicates / heavy overlaps
suppressed with the reference's deletion quirk, 0-5 instances.  Cases with
EXACTLY equal scores are excluded: the reference orders them with
np.argsort's default (unstable) kind, whose tie order depends on the numpy
version and CPU (numpy >= 2 sorts with x86-simd-sort on AVX-512 hosts; the
fixtures were made with numpy 2.2 here) -- not a property of the reference's
algorithm.  The port breaks ties by instance index (stable order), which is
what numpy's insertion sort for small arrays gave before SIMD sorting."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gn():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ref_mask_nms.npz")))


def _cases(gn):
    for i in range(int(gn["ncases"])):
        m, s = gn[f"masks_{i}"], gn[f"scores_{i}"]
        live = s[m.reshape(len(s), -1).any(axis=1)] if len(s) else s
        if len(np.unique(live)) != len(live):  # exact score tie: numpy-version-dependent order
            continue
        yield m, s, gn[f"picks_{i}"].tolist()


def test_fixture_coverage(gn):
    cs = list(_cases(gn))
    assert len(cs) >= 100
    assert any(len(p) < len(s) for _, s, p in cs)            # suppressions happen
    assert any(not m.reshape(len(s), -1).any(1).all() for m, s, _ in cs if len(s))  # empty masks


def test_oracle_matches_reference(gn):
    from oracle import features_ref as FR
    for masks, scores, picks in _cases(gn):
        assert FR.nms_mask_instances(masks, scores) == picks


@pytest.mark.gpu
def test_gpu_mask_nms_matches_reference(mdx, gn):
    """mdx_mask_nms_select on every fixture case, batched per frame size."""
    import torch
    from moseq2_detectron_extract_amd.pipeline import mask_nms_select
    groups = {}
    for masks, scores, picks in _cases(gn):
        groups.setdefault(masks.shape[1:], []).append((masks, scores, picks))
    K, D = 8, 5
    for (h, w), cs in groups.items():
        B = len(cs)
        mk = np.zeros((B, D, h, w), np.uint8)
        sc = np.zeros((B, D), np.float32)
        nd = np.zeros(B, np.int32)
        for b, (m, s, _) in enumerate(cs):
            mk[b, :len(s)] = m
            sc[b, :len(s)] = s
            nd[b] = len(s)
        kp = np.random.default_rng(0).random((B, D, K, 3)).astype(np.float32)
        out = {"masks": torch.from_numpy(mk).cuda(), "scores": torch.from_numpy(sc).cuda(),
               "ndet": torch.from_numpy(nd).cuda(), "keypoints": torch.from_numpy(kp).cuda()}
        sel, kps, nkeep, keep = mask_nms_select(out, 0.5)
        for b, (m, s, picks) in enumerate(cs):
            assert keep[b, :int(nkeep[b])].cpu().tolist() == picks, (h, w, b)
            want = m[picks[0]].astype(np.uint8) if picks else np.zeros((h, w), np.uint8)
            np.testing.assert_array_equal(sel[b].cpu().numpy(), want)
