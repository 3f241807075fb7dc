"""Host feature post-processing against fixtures produced by the reference's
own functions (tests/golden/make_golden_features.py, real bottleneck).

Tolerance: the reference rotates keypoints with a 2x2 @ 2xK matmul (BLAS,
possibly fused multiply-adds); the restatement vectorises the same products,
so rotated coordinates agree to ~1e-12 px.  Every decision (flips, filter
flips, final angles) must match exactly.
"""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = dict(rtol=1e-12, atol=1e-9)


@pytest.fixture(scope="module")
def gf():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ref_features.npz")))


@pytest.fixture(scope="module")
def F():
    import mdx_pkg
    mdx_pkg.load()  # registers the package (its directory name is not an identifier)
    from moseq2_detectron_extract_amd import features
    return features


def test_convert_pxs_to_mm(gf, F):
    np.testing.assert_array_equal(F.convert_pxs_to_mm(gf["px2mm_in"]), gf["px2mm_out"])
    np.testing.assert_array_equal(F.convert_pxs_to_mm(gf["px2mm_in"], true_depth=655.5), gf["px2mm_out_td"])


def test_rotate_points_batch(gf, F):
    ang = F.clamp_angles_deg(-np.rad2deg(gf["orient"]))
    got = F.rotate_points_batch(np.copy(gf["kp"]), gf["cen"], ang)
    np.testing.assert_allclose(got, gf["rot_batch"], equal_nan=True, **TOL)


def test_flips_alignment_rotation(gf, F):
    ang = F.clamp_angles_deg(-np.rad2deg(gf["orient"]))
    lengths = np.max(gf["axl"], axis=1)
    flips, conf = F.flips_from_keypoints(gf["kp"], gf["cen"], ang, lengths)
    np.testing.assert_array_equal(flips, gf["flips"])
    np.testing.assert_array_equal(conf, gf["flip_conf"])
    rot7 = F.rotate_points_batch(np.copy(gf["kp"][:, :7, :2]), gf["cen"], ang)
    np.testing.assert_array_equal(F.compute_keypoint_alignment_scores(rot7), gf["align_scores"])
    np.testing.assert_allclose(F.estimate_keypoint_rotation(rot7), gf["kp_rotation"], equal_nan=True, **TOL)


def test_move_median_matches_bottleneck(gf, F):
    mm = gf["mm_in"]
    for w in (1, 2, 3, 4, 7):
        np.testing.assert_array_equal(F.move_median(mm, w, min_count=1, axis=0), gf[f"mm_w{w}_mc1"])
        np.testing.assert_array_equal(F.move_median(mm, w, axis=0), gf[f"mm_w{w}_mcdef"])
        np.testing.assert_array_equal(F.move_median(mm[:, 0], w, min_count=1), gf[f"mm_w{w}_1d"])


def test_filter_angles(gf, F):
    np.testing.assert_array_equal(F.filter_angles(gf["filt_in"]), gf["filt_out"])
    a, fl = F.iterative_filter_angles(gf["filt_in"])
    np.testing.assert_array_equal(a, gf["ifilt_out"])
    np.testing.assert_array_equal(fl, gf["ifilt_flips"])


def test_finalize_angles_no_tracking(gf, F):
    ang, flips = F.finalize_angles(gf["orient"], gf["axl"], gf["cen"], gf["kp"])
    np.testing.assert_array_equal(ang, gf["final_angles"])
    np.testing.assert_array_equal(flips, gf["final_flips"])


def test_angle_difference(gf, F):
    np.testing.assert_array_equal(F.angle_difference(gf["adiff_a1"], gf["adiff_a2"]), gf["adiff_out"])


@pytest.mark.parametrize("mh,xh,td", [(10, 100, 673.1), (0, 100, 650.0)])
def test_compute_scalars(gf, F, mh, xh, td):
    from oracle import features_ref as FR
    fr, mk = gf["sc_frames"], gf["sc_masks"]
    tf = {k: gf[f"sc_tf_{k}"] for k in ("centroid", "axis_length", "orientation")}
    area, hmean, _ = FR.frame_scalars_ref(fr, mk, mh, xh)   # the GPU kernel's checker stands in for it on CPU
    got = F.compute_scalars(None, tf, mh, xh, td, reductions=(area, hmean))
    for k, v in got.items():
        want = gf[f"sc_{mh}_{xh}_{k}"]
        assert np.asarray(v).dtype == want.dtype, (k, np.asarray(v).dtype, want.dtype)
        if k == "velocity_theta":  # arctan2: numpy 1.26 (fixture) and 2.2 (here) libm differ by an ulp
            np.testing.assert_allclose(v, want, rtol=4e-16, atol=0, err_msg=k)
        else:
            np.testing.assert_array_equal(v, want, err_msg=k)


def test_keypoints_to_dict(gf, F):
    from oracle import features_ref as FR
    kp, fr = gf["kd_kp"], gf["kd_frames"]
    _, _, z = FR.frame_scalars_ref(fr, None, 0, 0, keypoints=kp, z_frames=fr)
    got = F.keypoints_to_dict(kp, fr, gf["kd_cen"], gf["kd_ang"], true_depth=660.0, z_data=z)
    keys = list(gf["kd_keys"])
    assert list(got.keys()) == keys
    for i, k in enumerate(keys):
        np.testing.assert_allclose(got[k], gf[f"kd_{i}"], equal_nan=True, err_msg=k, **TOL)


def test_attribute_tables(F):
    assert len(F.scalar_attributes()) == 17
    assert len(F.keypoint_attributes()) == 8 * 2 * 6


def test_iterative_filter_angles_native_matches_numpy(F):
    """libmdx's host loop (mdx_iterative_filter_angles) vs the numpy checker
    (oracle/features_ref.py), bit for bit: NaN (1000-iteration runs),
    constant series, max_iters cut-offs, windows 1..5, empty and 1-element
    series."""
    from oracle import features_ref as FR
    rng = np.random.default_rng(4)
    for trial in range(120):
        n = int(rng.integers(0, 200))
        a = rng.uniform(0, 360, n)
        if n:
            a[rng.random(n) < 0.3] += 180
        if trial % 3 == 0 and n:
            a[rng.integers(0, n)] = np.nan
        if trial % 7 == 0 and n:
            a[:] = a[0]
        for w in (1, 2, 3, 5):
            mi = int(rng.integers(0, 20)) if trial % 2 else (1000 if trial % 6 else 40)
            o1, f1 = F.iterative_filter_angles(a, w, 60, mi)
            o2, f2 = FR.iterative_filter_angles_ref(a, w, 60, mi)
            np.testing.assert_array_equal(o1, o2)
            np.testing.assert_array_equal(f1, f2)


def test_flips_native_matches_numpy(F):
    """mdx_flips_from_keypoints vs the numpy checker on random frames incl.
    NaN keypoints, NaN lengths and exact ties."""
    from oracle import features_ref as FR
    rng = np.random.default_rng(9)
    n = 3000
    kp = rng.uniform(0, 400, (n, 8, 3))
    kp[rng.random((n, 8)) < 0.02, :2] = np.nan
    cen = rng.uniform(50, 350, (n, 2))
    ang = rng.uniform(0, 360, n)
    ln = rng.uniform(20, 100, n)
    ln[::97] = np.nan
    kp[::31, :, 0] = cen[::31, 0, None]  # keypoints on the centroid: distance ties
    ang[::31] = 0.0
    f1, c1 = F.flips_from_keypoints(kp, cen, ang, ln)
    f2, c2 = FR.flips_ref(kp, cen, ang, ln)
    np.testing.assert_array_equal(f1, f2)
    np.testing.assert_array_equal(c1, c2)


def test_iterative_filter_angles_wide_window(F):
    """Windows above the native loop's 8 (and 2-D input) take the numpy
    statement of the same loop: equal to the checker."""
    from oracle import features_ref as FR
    rng = np.random.default_rng(5)
    for trial in range(20):
        n = int(rng.integers(1, 150))
        a = rng.uniform(0, 360, n)
        a[rng.random(n) < 0.3] += 180
        if trial % 3 == 0:
            a[rng.integers(0, n)] = np.nan
        for w in (9, 15):
            o1, f1 = F.iterative_filter_angles(a, w, 60, 50)
            o2, f2 = FR.iterative_filter_angles_ref(a, w, 60, 50)
            np.testing.assert_array_equal(o1, o2)
            np.testing.assert_array_equal(f1, f2)
