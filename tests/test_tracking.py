"""Tracking branch (tracking.py) against the loop-level pykalman restatement
in oracle/kalman_ref.py.  pykalman is absent from this image and the
reference's tests hold no fixture for it, so this is PARITY UNPINNED against
the reference itself; the reference's own documented examples
(kalman.py:31-35, 70-72) are pinned exactly.  Tolerance: the product inverts
with np.linalg.inv where pykalman calls scipy.linalg.pinv, so states agree to
1e-8 relative (decisions -- flips -- exactly)."""
import os
import sys

import numpy as np
import numpy.ma as ma
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def T():
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import tracking
    return tracking


@pytest.fixture(scope="module")
def R():
    from oracle import kalman_ref
    return kalman_ref


def _traj(n, seed=0, nan_frames=(), flip_every=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    cen = np.stack([200 + 50 * np.sin(t / 50), 200 + 40 * np.cos(t / 70)], 1) + rng.normal(0, 1, (n, 2))
    ang = (t * 0.7 + 30) % 360
    kp = np.zeros((n, 8, 3))
    for k in range(8):
        d = (3.5 - k) * 6
        kp[:, k, 0] = cen[:, 0] + d * np.cos(np.deg2rad(ang))
        kp[:, k, 1] = cen[:, 1] - d * np.sin(np.deg2rad(ang))
        kp[:, k, 2] = 0.9
    kp[:, :, :2] += rng.normal(0, 1, (n, 8, 2))
    obs = ang.copy()
    if flip_every:
        obs[::flip_every] += 180
    ori = -np.deg2rad(obs)
    axl = np.stack([np.full(n, 40.0), np.full(n, 15.0)], 1) + rng.normal(0, 0.5, (n, 2))
    for f in nan_frames:
        cen[f] = np.nan
        kp[f] = np.nan
        ori[f] = np.nan
        axl[f] = np.nan
    return cen, kp, ori, axl


def test_reference_documented_examples(T):
    data = np.array([0, 1, 3, 4, 8, 9, 10])
    steps = np.array([1, 2, 1, 4, 1, 1])
    full = T.expand_missing_entries(data, steps)
    np.testing.assert_array_equal(ma.getmaskarray(full),
                                  [False, False, True, False, False, True, True, True, False, False, False])
    np.testing.assert_array_equal(full.compressed(), data)
    np.testing.assert_array_equal(T.reduce_missing_entries(np.arange(11), steps), data)
    np.testing.assert_array_equal(T.timestamps_to_steps(np.array([0.0, 33.3, 100.0, 133.4])), [1, 2, 1])


def test_tracker_items(T, R):
    p, a = T.make_trackers(native=False)
    A1 = T.KalmanTrackerPoint1D(order=3).build_trans_mat()
    np.testing.assert_array_equal(A1, [[1, 1, 0.5], [0, 1, 1], [0, 0, 1]])
    assert [it.state_size for it in p.items] == [6, 48]
    assert a.items[0].state_size == 6
    Ar, Cr = R.point_tracker_matrices()
    from scipy.linalg import block_diag
    np.testing.assert_array_equal(block_diag(*[it.build_trans_mat() for it in p.items]), Ar)
    np.testing.assert_array_equal(block_diag(*[it.build_observ_mat() for it in p.items]), Cr)
    with pytest.raises(ValueError):
        T.KalmanTracker([])
    with pytest.raises(ValueError):
        T.KalmanTracker([T.KalmanTrackerPoint1D(delta_t=1.0), T.KalmanTrackerPoint1D(delta_t=2.0)])


@pytest.mark.parametrize("masked", [False, True])
def test_filter_smooth_em_match_pykalman_restatement(T, R, masked):
    rng = np.random.default_rng(3)
    A, C = R.angle_tracker_matrices()
    n = 120
    Z = np.stack([np.sin(np.arange(n) / 9), np.cos(np.arange(n) / 9)], 1) + rng.normal(0, 0.05, (n, 2))
    if masked:
        Z[[5, 6, 40]] = np.nan
        Z[70, 1] = np.inf
    Zm = ma.masked_invalid(Z)
    x0 = np.array([Z[0, 0], 0, 0, Z[0, 1], 0, 0])
    kf = T.KalmanFilter(A, C, x0)
    rf = R.KalmanFilter(A, C, x0)
    fin = np.isfinite(Z).any(axis=1)
    kf.em(Zm[fin], n_iter=10)
    rf.em(Zm[fin], n_iter=10)
    for got, want in ((kf.transition_covariance, rf.Q), (kf.observation_covariance, rf.R),
                      (kf.initial_state_covariance, rf.P0)):
        np.testing.assert_allclose(got, want, rtol=1e-8, atol=1e-12)
    xs, Ps = kf.smooth(Zm)
    xr, Pr = rf.smooth(Zm)
    np.testing.assert_allclose(xs, xr, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(Ps, Pr, rtol=1e-8, atol=1e-12)
    xf, _ = kf.filter(Zm)
    np.testing.assert_allclose(xf, rf.filter(Zm)[0], rtol=1e-8, atol=1e-10)
    x1, P1 = kf.filter_update(xs[-1], Ps[-1], Zm[3])
    y1, Q1 = rf.filter_update(xr[-1], Pr[-1], Zm[3])
    np.testing.assert_allclose(x1, y1, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(P1, Q1, rtol=1e-8, atol=1e-12)
    # a masked observation only predicts
    x2, _ = kf.filter_update(xs[-1], Ps[-1], ma.masked_invalid(np.array([np.nan, 0.0])))
    np.testing.assert_allclose(x2, A @ xs[-1])


def test_track_features_two_chunks_match_restatement(T, R):
    """Point smoothing (EM on chunk 0, smooth_update carried across chunks),
    keypoint flips, alignment scores and the per-frame angle loop."""
    from moseq2_detectron_extract_amd import features as F
    cen, kp, ori, axl = _traj(300, seed=5, nan_frames=(17, 150), flip_every=23)
    p, a = T.make_trackers()
    Ar, Cr = R.point_tracker_matrices()
    Aa, Ca = R.angle_tracker_matrices()
    rp, ra = R.RefTracker(Ar, Cr), R.RefTracker(Aa, Ca)
    for c0, c1 in ((0, 160), (160, 300)):
        c, k, o, ax = cen[c0:c1], kp[c0:c1], ori[c0:c1], axl[c0:c1]
        gc, gk, gang, gfl = T.track_features(p, a, c, k, o, ax)
        # restatement
        Z = R.point_format(c, k[:, :, :2])
        if rp.kf is None:
            rp.initialize(R.point_init_mean(c, k[:, :, :2]), Z)
        xs = rp.smooth_update(Z)
        sc = xs[:, 0:6:3]
        sk = xs[:, 6::3].reshape(len(xs), 8, 2)
        wk = np.array(k, dtype=float)
        wk[:, :7, :2] = sk[:, :7]
        ang = F.clamp_angles_deg(-np.rad2deg(o))
        fl, _ = F.flips_from_keypoints(wk, sc, ang, np.max(ax, axis=1))
        ang[fl] = F.clamp_angles_deg(ang[fl] + 180)
        scores = F.compute_keypoint_alignment_scores(F.rotate_points_batch(np.copy(wk[:, :7, :2]), sc, ang))
        wang, wfl = R.angle_loop_ref(ra, ang, fl, scores)
        np.testing.assert_allclose(gc, sc, rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(gk, wk, rtol=1e-9, atol=1e-8)
        np.testing.assert_array_equal(gfl, wfl)
        np.testing.assert_allclose(gang, wang, rtol=0, atol=1e-7)
        np.testing.assert_allclose(p.last_mean, rp.last_mean, rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(a.last_mean, ra.last_mean, rtol=1e-9, atol=1e-9)
    # the tracker corrected the injected 180-degree flips
    assert np.all(np.isfinite(gang[np.isfinite(ori[160:300])]))


def test_track_features_nan_first_frame_propagates(T):
    """build_init_state_means takes row 0 even when it is NaN (kalman.py:177-178):
    the reference's smoothed track is then NaN throughout; kept."""
    cen, kp, ori, axl = _traj(40, seed=1, nan_frames=(0,))
    p, a = T.make_trackers()
    c, k, ang, fl = T.track_features(p, a, cen, kp, ori, axl)
    assert np.isnan(c).all()


def test_native_tracking_matches_numpy_statement(T):
    """libmdx's tracking recursion (mdx_tracking_*) against the numpy
    statement in tracking.py over a session of chunks incl. a one-frame
    chunk (filter_update path) and NaN frames: smoothed centroid / keypoints
    and angles to 1e-9, flips exactly, tracker states to 1e-9."""
    cen, kp, ori, axl = _traj(900, seed=11, nan_frames=(5, 300, 301, 650), flip_every=17)
    pn, an = T.make_trackers(native=False)
    pc, ac = T.make_trackers()
    assert not pc.is_initialized and not ac.is_initialized
    for c0, c1 in ((0, 400), (400, 401), (401, 800), (800, 900)):
        args = (cen[c0:c1], kp[c0:c1], ori[c0:c1], axl[c0:c1])
        a = T.track_features(pn, an, *args)
        b = T.track_features(pc, ac, *args)
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_allclose(y, x, rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal(b[3], a[3])
    assert pc.is_initialized and ac.is_initialized
    np.testing.assert_allclose(pc.last_mean, pn.last_mean, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(ac.last_mean, an.last_mean, rtol=1e-9, atol=1e-12)
