"""GPU parity of the frame-op kernels against the CPU oracle (bit-exact for
the integer/byte ops and the fixed-order float64 moment arithmetic)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def session(mdx):
    from moseq2_detectron_extract_amd import synth
    return synth.SyntheticSession(24, seed=3)


@pytest.fixture(scope="module")
def raw(session):
    return session.frames(0, 24)


def test_prep_matches_golden(mdx, golden):
    from moseq2_detectron_extract_amd import proc
    tags = sorted({k[len("prep_out_"):] for k in golden if k.startswith("prep_out_")})
    for tag in tags:
        vmin = float(golden[f"prep_vmin_{tag}"]); vmax = float(golden[f"prep_vmax_{tag}"])
        out = proc.prep_raw_frames(golden[f"prep_raw_{tag}"], golden[f"prep_bg_{tag}"], golden[f"prep_roi_{tag}"],
                                   None if np.isnan(vmin) else vmin, None if np.isnan(vmax) else vmax,
                                   fix_invalid_pixels=False)
        np.testing.assert_array_equal(out, golden[f"prep_out_{tag}"], err_msg=tag)


def test_scale_matches_golden(mdx, golden):
    from moseq2_detectron_extract_amd import proc
    for k in range(5):
        vmin, vmax = golden[f"scale_vmin_{k}"].item(), golden[f"scale_vmax_{k}"].item()
        x = np.ascontiguousarray(golden[f"scale_in_{k}"])
        np.testing.assert_array_equal(proc.scale_raw_frames(x, vmin, vmax), golden[f"scale_out_{k}"])


def test_prep_full_size_and_invalid(mdx, session, raw):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    prep = proc.FramePrep(session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
    out, inv = prep(raw, return_invalid=True)
    ref, rinv = O.prep_raw_frames(raw, session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
    assert out.shape == (24, 423, 511)
    np.testing.assert_array_equal(out, ref)
    np.testing.assert_array_equal(inv, rinv)


@pytest.mark.parametrize("roi_kind", ["full", "arena"])
def test_prep_with_inpaint(mdx, roi_kind):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc, synth
    s = synth.SyntheticSession(6, seed=11, roi=roi_kind)
    raw = s.frames(0, 6)
    raw[2, 100:104, 200:203] = 0  # a larger hole to exercise the FMM order
    raw[3, 0, :40] = 0            # invalid pixels on the frame edge (OpenCV skip quirk)
    out = proc.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    ref, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100, fix_invalid_pixels=True)
    np.testing.assert_array_equal(out, ref)
    # the fused call (mdx_prep_inpaint) with the byte mask requested too, on
    # a prep whose workspace is reused for another batch size
    _, rinv = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100, fix_invalid_pixels=False)
    prep = proc.FramePrep(s.bground_im, s.roi, 0, 100, fix_invalid_pixels=True)
    for sl in (slice(0, 6), slice(1, 4), slice(0, 6)):
        got, inv = prep(raw[sl], return_invalid=True)
        np.testing.assert_array_equal(got, ref[sl])
        np.testing.assert_array_equal(inv, rinv[sl])
    assert prep.inpaint_errors() == 0


def test_clean_frames(mdx, session, raw):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    prepped, _ = O.prep_raw_frames(raw[:6], session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
    for iters in (0, 1, 3):
        got = proc.clean_frames(prepped, iters_tail=iters)
        want = O.clean_frames(prepped, iters_tail=iters)
        np.testing.assert_array_equal(got, want, err_msg=f"iters={iters}")
    # no median, rect strel
    got = proc.clean_frames(prepped, prefilter_space=None, strel_tail=np.ones((5, 5), np.uint8), iters_tail=2)
    want = O.morph(prepped, "open", np.ones((5, 5), np.uint8), 2)
    np.testing.assert_array_equal(got, want)


def test_clean_random_edges(mdx):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    rng = np.random.default_rng(5)
    x = rng.integers(0, 256, size=(3, 71, 133), dtype=np.uint8)
    np.testing.assert_array_equal(proc.clean_frames(x, iters_tail=2), O.clean_frames(x, iters_tail=2))


@pytest.mark.parametrize("mode", [1, 2, 3, 0])
def test_clean_fused_streaming_kernel(mdx, session, raw, mode):
    """The extract path's chain (median 3, opening with the 9x9 ellipse, 3
    iterations) on the fused streaming kernel (mdx_clean_set_mode 1: strip
    width by batch, 2: 256-column strips, 3: 512) and on the per-pass kernels
    (0), bit for bit vs
    the oracle: full frames, random bytes on ragged shapes (one strip, strip
    + 1 column, tiny and 1-row / 1-column frames, an image narrower than the
    25-column halo), the extreme values 0 / 255 everywhere."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    from moseq2_detectron_extract_amd._lib import call
    old = call("mdx_clean_set_mode", mode)
    try:
        prepped, _ = O.prep_raw_frames(raw[:8], session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
        np.testing.assert_array_equal(proc.clean_frames(prepped, iters_tail=3), O.clean_frames(prepped, iters_tail=3))
        rng = np.random.default_rng(17)
        for shape in [(2, 423, 511), (2, 64, 256), (2, 37, 257), (1, 9, 513), (3, 1, 40), (2, 30, 1), (2, 5, 7),
                      (1, 200, 1030)]:
            x = rng.integers(0, 256, size=shape, dtype=np.uint8)
            # sparse blobs as well as noise: long constant runs exercise the borders
            x[0] = np.where(rng.random(shape[1:]) < 0.7, 0, x[0])
            np.testing.assert_array_equal(proc.clean_frames(x, iters_tail=3), O.clean_frames(x, iters_tail=3),
                                          err_msg=str(shape))
        for v in (0, 255):
            x = np.full((2, 50, 300), v, np.uint8)
            np.testing.assert_array_equal(proc.clean_frames(x, iters_tail=3), O.clean_frames(x, iters_tail=3))
    finally:
        call("mdx_clean_set_mode", old)


def test_frame_features(mdx, session, raw):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    prepped, _ = O.prep_raw_frames(raw, session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
    cl = O.clean_frames(prepped, iters_tail=3)
    rng = np.random.default_rng(0)
    mask = (rng.random(cl.shape) < 0.97).astype(np.uint8)  # punch holes: many blobs / hole borders
    for m in (None, mask):
        got, _ = proc.get_frame_features(cl, frame_threshold=3, mask=m if m is not None else np.array([]))
        want = O.get_frame_features(cl, 3, mask=m)
        np.testing.assert_array_equal(got["centroid"], want["centroid"])
        np.testing.assert_array_equal(got["axis_length"], want["axis_length"])
        # atan2 may differ by an ulp between ocml and glibc
        np.testing.assert_allclose(got["orientation"], want["orientation"], rtol=0, atol=4e-16 * 8)


def test_frame_features_shapes(mdx):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    rng = np.random.default_rng(9)
    f = np.zeros((5, 60, 90), np.uint8)
    f[1, 10:20, 5:35] = 10                # rectangle
    f[2] = (rng.random((60, 90)) < 0.45) * 9  # noise: many blobs, holes
    f[3, 0:60, 0:90] = 50                 # full frame (touches the border)
    f[3, 20:30, 40:50] = 0                # with a hole
    f[4, 30, 40] = 7                      # single pixel -> NaN
    got = proc.frame_moments(f, None, 3.0)
    want = O.get_frame_features(f, 3)
    for k in ("centroid", "axis_length", "area"):
        np.testing.assert_array_equal(got[k].cpu().numpy(), want[k], err_msg=k)
    np.testing.assert_allclose(got["orientation"].cpu().numpy(), want["orientation"], atol=1e-14)
    assert np.isnan(want["centroid"][0]).all() and np.isnan(want["centroid"][4]).all()


def test_crop_and_rotate(mdx, session, raw):
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    prepped, _ = O.prep_raw_frames(raw, session.bground_im, session.roi, 0, 100, fix_invalid_pixels=False)
    n = prepped.shape[0]
    rng = np.random.default_rng(2)
    centers = np.column_stack([rng.uniform(-5, 520, n), rng.uniform(-5, 430, n)])
    centers[0] = [np.nan, 10]; centers[1] = [30.5, 12.25]; centers[2] = [600, 500]
    angles = rng.uniform(0, 360, n); angles[3] = np.nan; angles[4] = 0.0; angles[5] = 90.0
    masks = (prepped > 10).astype(np.uint8)
    got, gotm = proc.crop_and_rotate_frames(prepped, centers, angles, frames2=masks)
    want = O.crop_and_rotate_frames(prepped, centers, angles)
    wantm = O.crop_and_rotate_frames(masks, centers, angles)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(gotm, wantm)
    one = proc.crop_and_rotate_frame(prepped[7], centers[7], angles[7])
    np.testing.assert_array_equal(one, want[7])
    # integer crop windows, exactly as M/proc/proc.py:325-328 computes them
    # (python int() truncates toward zero); -1 where it returns zeros first
    _, _, win = proc.crop_and_rotate_frames(prepped, centers, angles, frames2=masks, return_window=True)
    for i in range(n):
        cx, cy = centers[i]
        if np.isnan(angles[i]) or np.isnan(cx) or np.isnan(cy) or cx < 0 or cy < 0:
            assert list(win[i]) == [-1] * 4, i
        else:
            assert list(win[i]) == [int(cx - 40) + 80, int(cx + 40) + 80, int(cy - 40) + 80, int(cy + 40) + 80], i


@pytest.mark.parametrize("p,seed", [(0.03, 1), (0.2, 2)])
def test_inpaint_dense_holes(mdx, p, seed):
    """Dense invalid pixels make large hole clusters (one lane marches a big
    cluster); results must equal the serial oracle bit for bit."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 100, size=(2, 90, 120), dtype=np.uint8)
    m = (rng.random(f.shape) < p).astype(np.uint8)
    m[1, 30:60, 40:90] = 1  # a big blob
    from moseq2_detectron_extract_amd._lib import call
    call("mdx_inpaint_errors", 1)
    got = proc.fill_invalid_pixels(f.copy(), m)
    want = O.inpaint_ns(f, m)
    np.testing.assert_array_equal(got, want)
    assert call("mdx_inpaint_errors", 1) == 0


def test_inpaint_sparse_and_dense_slots(mdx):
    """One call holding frames within the sparse slots' capacity (scattered
    pixels, one-pixel clusters, a small hole, invalid pixels on the first row
    and column) and frames over it (done in the shared dense slot: dense noise,
    a big blob, a fully invalid frame, one just over the capacity), then more
    calls on the same workspace with other masks and frame counts: each equals
    the serial oracle, so every call left the workspace at rest."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    from moseq2_detectron_extract_amd._lib import call
    H, W = 90, 120
    cap = call("mdx_inpaint_sparse_capacity", H, W)
    assert 256 <= cap < H * W // 10
    rng = np.random.default_rng(31)

    def masks(n):
        m = np.zeros((n, H, W), np.uint8)
        kinds = rng.permutation(n)
        for f in range(n):
            k = kinds[f] % 10
            if k == 0:
                m[f] = rng.random((H, W)) < 0.01
            elif k == 1:
                m[f] = rng.random((H, W)) < 0.2
            elif k == 2:
                m[f, 20:40, 30:80] = 1
            elif k == 3:
                m[f] = 1
            elif k == 4:  # exactly one over the capacity, scattered
                m[f].flat[rng.choice(H * W, cap + 1, replace=False)] = 1
            elif k == 5:  # exactly the capacity
                m[f].flat[rng.choice(H * W, cap, replace=False)] = 1
            elif k == 6:  # pixels on and next to every edge (the taps' border clamps)
                m[f, 0, ::7] = 1
                m[f, ::5, 0] = 1
                m[f, 1, 3::9] = 1
                m[f, 4::11, 1] = 1
                m[f, H - 1, 2::8] = 1
                m[f, 3::7, W - 1] = 1
                m[f, H - 2, 5::13] = 1
                m[f, 6::9, W - 2] = 1
                m[f, 50:53, 60:62] = 1
            elif k == 8:  # a sparse frame's cluster too large for the march window (100 pixels)
                m[f, 30:40, 50:60] = 1
                m[f].flat[rng.choice(H * W, 50, replace=False)] = 1
            elif k == 9:  # few pixels, window too large: a dotted diagonal (every 2 px) and a ring
                for t in range(0, 70, 2):
                    m[f, 5 + t, 10 + t] = 1
                m[f, 60, 20:100:3] = 1
            # k == 7: nothing to fill
        return m

    class Owner:
        _ws = None
        _errors = None

    owner = Owner()
    call("mdx_inpaint_errors", 1)
    for n in (10, 10, 3, 20):
        f = rng.integers(0, 100, size=(n, H, W), dtype=np.uint8)
        m = masks(n)
        got = proc.fill_invalid_pixels(f.copy(), m, _workspace_owner=owner)
        np.testing.assert_array_equal(got, O.inpaint_ns(f, m), err_msg=f"n={n}")
    assert call("mdx_inpaint_errors", 1) == 0
    assert int(owner._errors.item()) == 0


@pytest.mark.parametrize("shape", [(2, 1030, 1030), (3, 7, 1000), (2, 600, 9), (4, 1, 1), (2, 3, 3)])
def test_inpaint_frame_shapes(mdx, shape):
    """Frames whose bit image does not fit the setup workgroup's LDS (all done
    in the dense slot), long thin and tiny frames: equal to the serial
    oracle."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    from moseq2_detectron_extract_amd._lib import call
    rng = np.random.default_rng(sum(shape))
    f = rng.integers(0, 200, size=shape, dtype=np.uint8)
    m = (rng.random(shape) < 0.01).astype(np.uint8)
    if shape[1] * shape[2] < 100000:
        m[0].flat[::3] = 1
    call("mdx_inpaint_errors", 1)
    got = proc.fill_invalid_pixels(f.copy(), m)
    np.testing.assert_array_equal(got, O.inpaint_ns(f, m))
    assert call("mdx_inpaint_errors", 1) == 0


def test_inpaint_workspace_not_set_up_is_counted(mdx):
    """A workspace that was not set up for the frame shape: the frames are
    left as they are and each one is counted (device and caller counters)."""
    import ctypes
    import torch
    from moseq2_detectron_extract_amd._lib import call
    H, W, n = 40, 50, 3
    f = torch.randint(0, 100, (n, H, W), dtype=torch.uint8, device="cuda")
    m = (torch.rand((n, H, W), device="cuda") < 0.05).to(torch.uint8)
    ws = torch.zeros(call("mdx_inpaint_workspace_bytes", n, H, W), dtype=torch.uint8, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    before = f.clone()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    call("mdx_inpaint_errors", 1)
    call("mdx_inpaint_ns_counted", p(f), p(m), n, H, W, 3, p(ws), p(err), s)
    torch.cuda.synchronize()
    assert torch.equal(f, before)
    assert int(err.item()) == n and call("mdx_inpaint_errors", 1) == n
    # set up for another shape: the same
    call("mdx_inpaint_workspace_init", p(ws), ws.numel(), H + 1, W, s)
    call("mdx_inpaint_ns_counted", p(f), p(m), n, H, W, 3, p(ws), p(err), s)
    torch.cuda.synchronize()
    assert torch.equal(f, before) and int(err.item()) == 2 * n
    call("mdx_inpaint_errors", 1)


def test_inpaint_long_chain_converges(mdx):
    """One hole cluster shaped as a long serpentine chain (runs of single
    invalid pixels 3 px apart, rows 6 px apart joined at alternating ends):
    the min-label propagation needs many iterations to carry the first
    pixel's label to the far end.  Every label must converge to its root
    (mdx_inpaint_errors stays 0) and the result equals the serial oracle."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    from moseq2_detectron_extract_amd._lib import call
    H, W = 211, 255
    rng = np.random.default_rng(5)
    f = rng.integers(0, 100, size=(2, H, W), dtype=np.uint8)
    m = np.zeros((2, H, W), np.uint8)
    rows = list(range(4, H - 4, 6))
    for r, y in enumerate(rows):
        m[0, y, 4:W - 4:3] = 1
        if r + 1 < len(rows):  # connector down to the next row at alternating ends
            x = W - 5 if r % 2 == 0 else 4
            m[0, y:y + 7:3, x] = 1
    # a second frame: the same chain reversed in raster order (labels must
    # travel the other way)
    m[1] = m[0][::-1, ::-1]
    call("mdx_inpaint_errors", 1)
    got = proc.fill_invalid_pixels(f.copy(), m)
    assert call("mdx_inpaint_errors", 1) == 0
    np.testing.assert_array_equal(got, O.inpaint_ns(f, m))


def test_frame_scalars_matches_oracle(mdx):
    """Area / mean height of frames*masks and the keypoint z lookup, bit-exact
    against the numpy restatement (NaN / inf / out-of-range keypoints included)."""
    from oracle import features_ref as FR
    from moseq2_detectron_extract_amd import features as F
    rng = np.random.default_rng(21)
    fr = rng.integers(0, 140, size=(7, 61, 83), dtype=np.uint8)   # W not a multiple of 16: ragged tail path
    mk = (rng.random(fr.shape) < 0.5).astype(np.uint8)
    mk[2] = 0
    kp = np.concatenate([rng.uniform(-20, 100, (7, 8, 2)), rng.random((7, 8, 1))], -1)
    kp[1, 3, :2] = [np.nan, 4.0]; kp[4, 0, :2] = [np.inf, -np.inf]; kp[5, 5, :2] = [1e300, -1e300]
    zf = rng.integers(0, 255, size=fr.shape, dtype=np.uint8)
    for lo, hi in ((10, 100), (0, 100), (-1, 256)):
        a, h, z = F.frame_scalars(fr, mk, lo, hi, keypoints=kp, z_frames=zf)
        ra, rh, rz = FR.frame_scalars_ref(fr, mk, lo, hi, keypoints=kp, z_frames=zf)
        np.testing.assert_array_equal(a.cpu().numpy(), ra)
        np.testing.assert_array_equal(h.cpu().numpy(), rh)
        np.testing.assert_array_equal(z.cpu().numpy(), rz)


def test_compute_scalars_and_keypoints_on_device_match_reference(mdx):
    """compute_scalars / keypoints_to_dict with their reductions on the GPU
    against the reference's own outputs (tests/golden/ref_features.npz)."""
    import os
    import torch
    from moseq2_detectron_extract_amd import features as F
    gf = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_features.npz")))
    fr, mk = gf["sc_frames"], gf["sc_masks"]
    tf = {k: gf[f"sc_tf_{k}"] for k in ("centroid", "axis_length", "orientation")}
    for mh, xh, td in [(10, 100, 673.1), (0, 100, 650.0)]:
        got = F.compute_scalars(torch.from_numpy(fr * mk).cuda(), tf, mh, xh, td)
        for k, v in got.items():
            np.testing.assert_allclose(v, gf[f"sc_{mh}_{xh}_{k}"], rtol=4e-16, atol=0, err_msg=k)
    kd = F.keypoints_to_dict(gf["kd_kp"], torch.from_numpy(gf["kd_frames"]).cuda(), gf["kd_cen"], gf["kd_ang"],
                             true_depth=660.0)
    for i, k in enumerate(list(gf["kd_keys"])):
        np.testing.assert_allclose(kd[k], gf[f"kd_{i}"], rtol=1e-12, atol=1e-9, equal_nan=True, err_msg=k)


@pytest.mark.parametrize("shape,thr", [((3, 64, 600), 3.0), ((3, 530, 80), 2.5), ((2, 423, 511), -1.0),
                                       ((2, 423, 511), 254.5), ((2, 40, 50), 7.0)])
def test_frame_moments_sizes_and_thresholds(mdx, shape, thr):
    """Both contour-sum paths (sides <= 512: int32 per-edge products; larger
    frames: int64) and the integer form of the threshold (fractional,
    negative, near 255) against the oracle, bit for bit."""
    from oracle import frameops as O
    from moseq2_detectron_extract_amd import proc
    rng = np.random.default_rng(sum(shape))
    n, h, w = shape
    f = np.zeros(shape, np.uint8)
    for i in range(n):
        y0, x0 = rng.integers(0, h // 3), rng.integers(0, w // 3)
        f[i, y0:y0 + h // 2, x0:x0 + w // 2] = rng.integers(0, 256, (h // 2, w // 2))
    f[0, : h // 4, : w // 4] = 255
    got = proc.frame_moments(f, None, thr)
    want = O.get_frame_features(f, thr)
    for k in ("centroid", "axis_length", "area"):
        np.testing.assert_array_equal(got[k].cpu().numpy(), want[k], err_msg=k)
    np.testing.assert_allclose(got["orientation"].cpu().numpy(), want["orientation"], atol=1e-14)
