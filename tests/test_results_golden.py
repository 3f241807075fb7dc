"""Result writers (results.py) against the reference's own
write_extracted_chunk_to_h5 (real h5py) and ResultWriterStep's keypoints TSV
(tests/golden/make_golden_results.py): identical dataset contents and
identical TSV bytes."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ref_results.npz")))


@pytest.fixture(scope="module")
def RS():
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import results
    return results


def _chunks(g):
    out = []
    for i in range(2):
        p = f"c{i}_"
        out.append({
            "frame_idxs": g[p + "frame_idxs"], "offset": int(g[p + "offset"]),
            "depth_frames": g[p + "depth_frames"], "mask_frames": g[p + "mask_frames"],
            "scalars": {k[len(p + "scalars/"):]: g[k] for k in g if k.startswith(p + "scalars/")},
            "keypoints": {k[len(p + "keypoints/"):]: g[k] for k in g if k.startswith(p + "keypoints/")},
            "features": {"flips": g[p + "flips"],
                         "features": {"centroid": g[p + "centroid"], "orientation": g[p + "orientation"]}},
        })
    return out


def test_h5_layout_and_chunk_writes(g, RS, tmp_path):
    n = int(g["nframes"])
    cfg = {"nframes": n, "crop_size": (80, 80), "frame_dtype": "uint8", "timestamps": np.arange(n) * 33.3,
           "flip_classifier": "keypoints", "true_depth": 673.5, "roi": np.ones((4, 5), bool),
           "first_frame": np.zeros((4, 5), np.int16), "bground_im": np.full((4, 5), 670.0)}
    status = {"uuid": "abc", "parameters": {"chunk_size": 1000, "bg_roi_depth_range": (650, 750), "x": None,
                                            "nested": {"a": 1.5}},
              "metadata": {"SubjectName": "m1", "Tags": ["a", "b"], "Empty": None}}
    path = str(tmp_path / "r.npz")
    h = RS.MemoryH5(path)
    RS.create_extract_h5(h, cfg, status)
    for c in _chunks(g):
        RS.write_extracted_chunk_to_h5(h, c)
    want = {k[3:]: g[k] for k in g if k.startswith("h5/")}
    for k, v in want.items():
        assert h[k].dtype == v.dtype, k
        np.testing.assert_array_equal(h[k][()], v, err_msg=k)
    assert set(RS.scalar_attributes()) <= {k.split("/", 1)[1] for k in want if k.startswith("scalars/")}
    assert h["frames_mask"].attrs["description"].startswith("Boolean mask")
    h.close()
    saved = np.load(path)
    np.testing.assert_array_equal(saved["frames"], want["frames"])
    assert float(saved["metadata/extraction/true_depth"]) == 673.5
    assert list(saved["metadata/extraction/parameters/bg_roi_depth_range"]) == [650, 750]


def test_overlapping_chunk_raises_like_reference(g, RS):
    h = RS.MemoryH5()
    n = int(g["nframes"])
    for k in ("frames", "frames_mask"):
        h.create_dataset(k, (n, 80, 80), "uint8" if k == "frames" else "bool")
    h.create_dataset("metadata/extraction/flips", (n,), "bool")
    c = _chunks(g)[0]
    c = dict(c, offset=2, scalars={}, keypoints={})
    with pytest.raises(ValueError):
        RS.write_extracted_chunk_to_h5(h, c)


def test_keypoints_tsv_bytes(g, RS, tmp_path):
    w = RS.KeypointsTSVWriter(str(tmp_path))
    for c in _chunks(g):
        w.write(c)
    with open(w.path, "rb") as fh:
        got = fh.read()
    assert got == bytes(g["tsv"])


def test_status_yaml_roundtrip(tmp_path, RS):
    """Status file (M/extract.py:47-62,129-131; write_yaml M/io/util.py:99-109;
    check_completion_status M/proc/util.py:63-77)."""
    p = RS.status_filename(str(tmp_path))
    assert p.endswith("results_00.yaml")
    assert not RS.check_completion_status(p)  # missing file
    st = {"complete": False, "skip": False, "uuid": "u", "metadata": {"DepthResolution": [512, 424]},
          "parameters": {"crop_size": (80, 80), "chunk_size": np.int64(1000), "min_height": 0.0}}
    RS.write_status(p, st)
    assert not RS.check_completion_status(p)
    st["complete"] = True
    RS.write_status(p, st)
    assert RS.check_completion_status(p)
    import yaml
    with open(p) as fh:
        d = yaml.safe_load(fh)
    assert d["parameters"]["crop_size"] == [80, 80] and d["parameters"]["chunk_size"] == 1000
    assert d["metadata"]["DepthResolution"] == [512, 424]


def test_save_npz_parallel_pieces_round_trip(tmp_path, monkeypatch):
    """MemoryH5's writer (results.save_npz): members deflated in parallel
    pieces form one valid deflate stream per member; np.load and zipfile's
    CRC check read it back exactly, with and without zip64 records."""
    import zipfile
    from moseq2_detectron_extract_amd import results as RS
    rng = np.random.default_rng(0)
    fr = np.zeros((700, 80, 80), np.uint8)  # 4.5 MB: several pieces with a small piece size
    fr[:, 20:60, 10:70] = rng.integers(0, 60, (700, 40, 60))
    arrs = {"frames": fr, "frames_mask": fr > 20, "scalars/x": rng.random(700).astype("float32"),
            "metadata/uuid": np.array("abc-def"), "empty": np.zeros((0, 3)), "k": np.array(3.5),
            "f": np.asfortranarray(rng.random((5, 7)))}
    monkeypatch.setattr(RS, "_PIECE", 1 << 20)
    for lim in (0xFFFFFFFF, 1):
        monkeypatch.setattr(RS, "_ZIP64_AT", lim)
        p = str(tmp_path / f"r{lim}.npz")
        RS.save_npz(p, arrs)
        assert zipfile.ZipFile(p).testzip() is None
        z = np.load(p)
        assert sorted(z.files) == sorted(arrs)
        for k, v in arrs.items():
            assert z[k].dtype == v.dtype and z[k].shape == v.shape and np.array_equal(z[k], v), k


@pytest.mark.parametrize("order", ["in-order", "reversed", "partial"])
def test_streamed_npz_members(RS, tmp_path, monkeypatch, order):
    """The crop stacks deflated chunk by chunk while the session runs
    (MemoryH5.rows_written: every piece as soon as its rows are in, wherever
    it lies) load back equal to the arrays, with chunks arriving in frame
    order, in reverse and with rows never written (zeros, compressed at
    close); small pieces so every member spans several."""
    monkeypatch.setattr(RS, "_PIECE", 4096)
    n, c = 50, 7
    rng = np.random.default_rng(3)
    path = str(tmp_path / "s.npz")
    h = RS.MemoryH5(path)
    h.create_dataset("frames", (n, 80, 80), "uint8")
    h.create_dataset("frames_mask", (n, 80, 80), "bool")
    h.create_dataset("scalars/x", (n,), "float32")
    starts = list(range(0, n, c))
    if order == "reversed":
        starts = starts[::-1]
    if order == "partial":
        starts = starts[:-2]
    for a in starts:
        rows = np.arange(a, min(a + c, n))
        h["frames"][rows] = rng.integers(0, 255, (len(rows), 80, 80))
        h["frames_mask"][rows] = rng.random((len(rows), 80, 80)) > 0.5
        h["scalars/x"][rows] = rng.random(len(rows))
        h.rows_written(rows)
    st = h._streams["frames"]
    if order in ("in-order", "reversed"):  # every whole piece compressed before close
        assert st.npieces > 3 and len(st.done) == st.npieces
    else:
        assert 0 < len(st.done) < st.npieces
    want = {k: v.data.copy() for k, v in h.datasets.items()}
    h.close()
    got = np.load(path)
    for k, v in want.items():
        assert got[k].dtype == v.dtype
        np.testing.assert_array_equal(got[k], v, err_msg=k)


def test_native_tsv_rows_match_python_repr(RS):
    """libmdx's TSV formatter (mdx_format_tsv_rows, host code) against the
    Python formatter (repr of each float, '' for NaN, True / False, ints) on
    values across the whole double range, the positional / exponent
    thresholds (1e-4, 1e16), signed zeros, infinities and subnormals."""
    rng = np.random.default_rng(7)
    n = 20000
    a = rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e16, 9999999999999998.0, 1e15, 1e-4, 9.999999999999999e-05,
                        1e-5, 0.1, 5.0, -123456789.125, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
                        123456789012345678.0, 0.30000000000000004])
    cols = [np.arange(n + special.size, dtype=np.int64) - 5, rng.random(n + special.size) > 0.5,
            np.concatenate([a, special]), np.concatenate([special, a])]
    native = RS._tsv_rows_native(cols)
    cells = [RS._tsv_cells(c) for c in cols]
    want = "".join("\t".join(r) + "\n" for r in zip(*cells)).encode()
    assert native == want


def test_chunk_writer_abort_leaves_no_results(mdx, tmp_path):
    """A failed extraction stops the writer thread without finishing the
    results file and without raising over the extraction's own exception
    (extract.extract_session -> _ChunkWriter.abort): here the writer thread
    itself fails on a malformed chunk, and abort() neither raises nor writes
    results_00.npz; close() on a healthy writer does."""
    import numpy as np
    from moseq2_detectron_extract_amd.extract import _ChunkWriter
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig

    class Src:
        path = str(tmp_path / "depth.dat")
        last_frame_idx = 4

        def read(self, idx):
            return np.zeros((len(idx), 424, 512), np.int16)

    args = (Src(), np.full((424, 512), 670.0), np.ones((424, 512), bool), 670.0, ExtractConfig(), None, None)
    w = _ChunkWriter(str(tmp_path / "bad"), *args)
    w.write({"frame_idxs": np.arange(2), "offset": 0, "scalars": {"no_such_scalar": np.zeros(2)}, "keypoints": {},
             "depth_frames": np.zeros((2, 80, 80), np.uint8), "mask_frames": np.zeros((2, 80, 80), np.uint8),
             "features": {"flips": np.zeros(2, bool), "features": {}}})
    w.abort()
    assert not (tmp_path / "bad" / "results_00.npz").exists()
    ok = _ChunkWriter(str(tmp_path / "good"), *args)
    ok.close()
    assert (tmp_path / "good" / "results_00.npz").exists()
