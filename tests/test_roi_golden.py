"""Session setup (roi.py) against the reference's own get_roi / plane_ransac /
get_bground_im (tests/golden/make_golden_roi.py, run under py3.9 with real
scikit-image and scipy; the cv2 calls inside are restatements, so OpenCV's
ellipse / dilate / medianBlur are pinned only through SURVEY.md's quoted rows
and the oracle)."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ref_roi.npz")))


@pytest.fixture(scope="module")
def R():
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import roi
    return roi


def test_select_strel(g, R):
    np.testing.assert_array_equal(R.select_strel("ellipse", (10, 10)), g["strel_ellipse_10"])
    np.testing.assert_array_equal(R.select_strel("rect", (4, 3)), np.ones((3, 4), np.uint8))


@pytest.mark.parametrize("k", [0, 1])
def test_plane_ransac(g, R, k):
    np.random.seed(int(g[f"ransac_seed_{k}"]))
    plane, dist = R.plane_ransac(g[f"ransac_img_{k}"], iters=200)
    np.testing.assert_allclose(plane, g[f"ransac_plane_{k}"], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(dist, g[f"ransac_dist_{k}"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("k", [0, 1])
def test_get_roi(g, R, k):
    np.random.seed(int(g[f"ransac_seed_{k}"]))
    rois, plane, bboxes, label_im, ranks, shape_index = R.get_roi(
        g[f"ransac_img_{k}"], strel_dilate=R.select_strel("ellipse", (10, 10)), weights=(1, .1, 1),
        depth_range=(650, 750), iters=200)
    np.testing.assert_allclose(plane, g[f"roi_plane_{k}"], rtol=1e-14, atol=1e-14)
    np.testing.assert_array_equal(label_im, g[f"roi_label_{k}"])
    np.testing.assert_array_equal(ranks, g[f"roi_ranks_{k}"])
    np.testing.assert_array_equal(shape_index, g[f"roi_shape_index_{k}"])
    np.testing.assert_array_equal(np.stack([np.asarray(r, bool) for r in rois]), g[f"roi_rois_{k}"])
    np.testing.assert_array_equal(np.stack(bboxes), g[f"roi_bboxes_{k}"])
    img = g[f"ransac_img_{k}"]
    assert float(np.median(img[rois[0] > 0])) == float(g[f"roi_true_depth_{k}"])


@pytest.mark.parametrize("k", [0, 1])
def test_oracle_bground_matches_reference(g, k):
    from oracle.frameops import bground_ref
    np.testing.assert_array_equal(bground_ref(g[f"bg_frames_{k}"]), g[f"bg_out_{k}"])


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_bground_gpu_matches_reference(g, R, k):
    np.testing.assert_array_equal(R.get_bground_im(g[f"bg_frames_{k}"]), g[f"bg_out_{k}"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,med", [(1, 5), (9, 5), (10, 3), (0, 5), (108, 5)])
def test_bground_gpu_matches_oracle(R, n, med):
    from oracle.frameops import bground_ref
    rng = np.random.default_rng(n)
    fr = rng.integers(-32768, 32767, size=(n, 61, 83), dtype=np.int64).astype(np.int16)
    fr[:, 10:40, 20:60] = (700 + rng.normal(0, 30, (n, 30, 40))).astype(np.int16)
    got = R.get_bground_im(fr, med_scale=med)
    if n == 0:
        assert got.shape == (61, 83) and np.isnan(got).all()
        return
    np.testing.assert_array_equal(got, bground_ref(fr, med))


@pytest.mark.gpu
def test_find_roi_on_dat(g, R, tmp_path):
    """find_roi over a .dat session: background from every 500th frame on the
    device, then the ROI / true depth of the reference's get_roi."""
    from moseq2_detectron_extract_amd.session import RawDepthSource
    from oracle.frameops import bground_ref
    img = g["ransac_img_0"]
    rng = np.random.default_rng(2)
    n = 1001
    fr = (img[None] + rng.normal(0, 1.0, (n,) + img.shape)).round().astype("<i2")
    path = str(tmp_path / "depth.dat")
    fr.tofile(path)
    src = RawDepthSource(path, frame_dims=(img.shape[1], img.shape[0]))
    np.random.seed(3)
    first, bg, roi, td = R.find_roi(src, bg_roi_depth_range=(650, 750))
    np.testing.assert_array_equal(first, fr[:1])
    np.testing.assert_array_equal(bg, bground_ref(fr[::500]))
    np.random.seed(3)
    rois = R.get_roi(bg, strel_dilate=R.select_strel("ellipse", (10, 10)))[0]
    np.testing.assert_array_equal(roi, rois[0])
    assert td == float(np.median(bg[roi > 0]))
