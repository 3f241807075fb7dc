"""Frame source (session.py) against the reference's own readers
(tests/golden/make_golden_io.py): bit-exact frames for every selection, from a
plain .dat and from a .tar.gz member, and identical chunk boundaries."""
import os
import tarfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gio():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "ref_io.npz")))


@pytest.fixture(scope="module")
def S():
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import session
    return session


@pytest.fixture(scope="module")
def files(gio, tmp_path_factory):
    d = tmp_path_factory.mktemp("sess")
    dat = str(d / "depth.dat")
    gio["raw"].astype("<i2").tofile(dat)
    tgz = str(d / "session.tar.gz")
    with tarfile.open(tgz, "w:gz") as tf:
        tf.add(dat, arcname="session/depth.dat")
    return dat, tgz


@pytest.mark.parametrize("key", ["all", "empty", "int", "runs", "tail"])
def test_read_frames_raw(gio, S, files, key):
    dat, tgz = files
    sel = gio[f"sel_{key}"]
    sel = None if sel.ndim == 0 and sel == -1 else (int(sel) if sel.ndim == 0 else list(sel))
    np.testing.assert_array_equal(S.read_frames_raw(dat, sel, frame_dims=(16, 12)), gio[f"read_{key}"])
    with tarfile.open(tgz, "r:gz") as tf:
        m = tf.getmember("session/depth.dat")
        np.testing.assert_array_equal(S.read_frames_raw(m, sel, frame_dims=(16, 12), tar_object=tf),
                                      gio[f"readtar_{key}"])


def test_read_frames_raw_large_runs(S, tmp_path, monkeypatch):
    """Runs read straight into the destination rows as parallel preads
    (session._direct_read, pieces cut at _READ_PIECE bytes, here smaller
    than a frame run) equal the staged read; a file that ends early raises."""
    monkeypatch.setattr(S, "_READ_PIECE", 4096 + 24)  # pieces that cut frames mid-row
    rng = np.random.default_rng(3)
    raw = rng.integers(-2000, 2000, (40, 12, 16)).astype("<i2")
    dat = str(tmp_path / "depth.dat")
    raw.tofile(dat)
    for sel in (list(range(40)), list(range(5, 37)), [3, 4, 5, 9, 10, 2, 30, 31, 32, 33, 0],
                list(range(39, -1, -1))):
        got = S.read_frames_raw(dat, sel, frame_dims=(16, 12))
        np.testing.assert_array_equal(got, raw[sel])
        out = np.full((len(sel), 12, 16), -1, np.int16)
        assert S.read_frames_raw(dat, sel, frame_dims=(16, 12), out=out) is out
        np.testing.assert_array_equal(out, raw[sel])
    with pytest.raises(ValueError):
        S.read_frames_raw(dat, list(range(38, 42)), frame_dims=(16, 12))


def test_chunk_boundaries(gio, S):
    from moseq2_detectron_extract_amd.shard import gen_batch_sequence
    for k in range(5):
        nf, t0, t1, chunk, ovl = gio[f"chunks_{k}_args"]
        first = t0 if 0 < t0 < nf else 0
        last = nf - t1 if nf - t1 > first else nf
        seq = gen_batch_sequence(int(last - first), int(chunk), int(ovl), int(first))
        np.testing.assert_array_equal([len(s) for s in seq], gio[f"chunks_{k}_lens"])
        flat = np.concatenate([np.asarray(s) for s in seq]) if seq else np.zeros(0, int)
        np.testing.assert_array_equal(flat, gio[f"chunks_{k}_flat"])


def test_source_iterates_chunks_on_host(gio, S, files):
    dat, tgz = files
    for path in (dat, tgz):
        src = S.RawDepthSource(path, frame_dims=(16, 12), member="session/depth.dat", frame_trim=(3, 2))
        got = list(src.iterate(chunk_size=7, device=False))
        want_idx = [list(s) for s in src.batches(7)]
        assert [g[0] for g in got] == want_idx
        for idx, fr in got:
            np.testing.assert_array_equal(fr, gio["raw"][idx])
        src.close()


@pytest.mark.gpu
def test_source_streams_to_hbm_with_filter(gio, S, files):
    """Pinned reader thread + copy stream: device chunks equal the host reads,
    and an attached device filter runs on them."""
    import torch
    dat, _ = files
    src = S.RawDepthSource(dat, frame_dims=(16, 12))
    src.attach_filter(lambda t: t * 2)
    got = list(src.iterate(chunk_size=6, device=True, prefetch=2))
    assert len(got) == len(src.batches(6))
    for idx, fr in got:
        assert fr.is_cuda and fr.dtype == torch.int16
        np.testing.assert_array_equal(fr.cpu().numpy(), gio["raw"][idx] * 2)
