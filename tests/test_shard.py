"""Frame sharding and the rank-0 result gather, world_size 2 on
CPU with the gloo backend."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_gen_batch_sequence_matches_reference_semantics(mdx):
    from moseq2_detectron_extract_amd.shard import gen_batch_sequence
    seq = gen_batch_sequence(2500, 1000)
    assert [len(s) for s in seq] == [1000, 1000, 500]
    assert seq[1][0] == 1000 and seq[2][-1] == 2499
    ov = gen_batch_sequence(10, 4, overlap=1)
    assert [list(s) for s in ov] == [[0, 1, 2, 3], [3, 4, 5, 6], [6, 7, 8, 9]]


@pytest.mark.parametrize("nframes,chunk,world", [(10000, 1000, 8), (1_000_000, 1000, 8), (2500, 1000, 4),
                                                  (999, 1000, 2), (7, 3, 3)])
def test_shards_partition_frames(mdx, nframes, chunk, world):
    from moseq2_detectron_extract_amd.shard import shard_chunks, shard_range
    covered = []
    for r in range(world):
        ch = shard_chunks(nframes, chunk, world, r)
        for a, b in ch:
            assert a % chunk == 0 and b - a <= chunk
        covered += ch
        if ch:
            s, e = shard_range(nframes, chunk, world, r)
            assert (s, e) == (ch[0][0], ch[-1][1])
    covered.sort()
    assert covered[0][0] == 0 and covered[-1][1] == nframes
    for (a0, b0), (a1, _) in zip(covered, covered[1:]):
        assert b0 == a1
    sizes = [sum(b - a for a, b in shard_chunks(nframes, chunk, world, r)) for r in range(world)]
    assert max(sizes) - min(sizes) <= chunk


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.shard import gather_ragged_to_rank0, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard_range(2500, 1000, world, rank)
    # stand-in per-frame results: (frame index, 2x2 "crop")
    res = torch.stack([torch.full((2, 2), float(i)) for i in range(s, e)]) if e > s else torch.zeros((0, 2, 2))
    out = gather_ragged_to_rank0(res)
    if rank == 0:
        allr = torch.cat(out)
        q.put(allr[:, 0, 0].numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_gather_results_world2_gloo(mdx):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == list(range(2500))


def _chunk_feats(n_chunks, chunk, seed=11):
    """Per-chunk host feature records as GPUExtractor.features_pass returns them."""
    rng = np.random.default_rng(seed)
    n = n_chunks * chunk
    t = np.arange(n)
    cen = np.stack([200 + 30 * np.sin(t / 20), 180 + 20 * np.cos(t / 30)], 1) + rng.normal(0, 1, (n, 2))
    ang = (t * 2.0) % 360
    kp = np.zeros((n, 8, 3))
    for k in range(8):
        d = (3.5 - k) * 6
        kp[:, k, 0] = cen[:, 0] + d * np.cos(np.deg2rad(ang))
        kp[:, k, 1] = cen[:, 1] - d * np.sin(np.deg2rad(ang))
        kp[:, k, 2] = 0.8
    kp[:, :, :2] += rng.normal(0, 1, (n, 8, 2))
    ori = -np.deg2rad(ang + np.where(t % 17 == 0, 180, 0))
    axl = np.stack([np.full(n, 40.0), np.full(n, 14.0)], 1)
    cen[7] = np.nan
    kp[9] = np.nan
    return [{"centroid": cen[i:i + chunk], "orientation": ori[i:i + chunk], "axis_length": axl[i:i + chunk],
             "keypoints": kp[i:i + chunk]} for i in range(0, n, chunk)]


def _track_worker(rank, world, port, q, n_chunks, chunk):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.extract import shard_chunk_range
    from moseq2_detectron_extract_amd.shard import tracking_exchange
    from moseq2_detectron_extract_amd.tracking import make_trackers
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    feats = _chunk_feats(n_chunks, chunk)
    c0, c1 = shard_chunk_range(len(feats), world, rank)
    p, a = make_trackers() if rank == 0 else (None, None)
    res = tracking_exchange(feats[c0:c1], p, a)
    q.put((rank, [[np.asarray(x).tolist() for x in r] for r in res]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_chunks", [(2, 3), (3, 2)])
def test_tracking_exchange_equals_sequential(mdx, world, n_chunks):
    """Rank 0 tracks every rank's chunks in session order: the scattered
    results equal one process running the tracking branch chunk by chunk
    (bit-exact), including a rank that owns no chunk (world 3, 2 chunks)."""
    from moseq2_detectron_extract_amd.tracking import make_trackers, track_features
    chunk = 40
    feats = _chunk_feats(n_chunks, chunk)
    p, a = make_trackers()
    want = [track_features(p, a, f["centroid"], f["keypoints"], f["orientation"], f["axis_length"]) for f in feats]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_track_worker, args=(r, world, port, q, n_chunks, chunk)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    flat = [r for k in sorted(got) for r in got[k]]
    assert len(flat) == len(want)
    for g, w in zip(flat, want):
        for gx, wx in zip(g, w):
            np.testing.assert_array_equal(np.asarray(gx, dtype=np.asarray(wx).dtype), wx)


def _sel_session(n_chunks, chunk, D=4, seed=4):
    """Per-chunk (nkeep, centres (n,D,2)) of a multi-animal scenario."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_instances import _scenario
    frames = _scenario(seed, n=n_chunks * chunk, max_det=D)
    nk = np.array([len(d) for d in frames])
    cen = np.full((len(frames), D, 2), np.nan)
    for f, d in enumerate(frames):
        for s, (_, c) in enumerate(d):
            cen[f, s] = c
    return [(nk[i:i + chunk], cen[i:i + chunk]) for i in range(0, len(frames), chunk)]


def _select_worker(rank, world, port, q, n_chunks, chunk):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.extract import shard_chunk_range
    from moseq2_detectron_extract_amd.instances import InstanceTracker
    from moseq2_detectron_extract_amd.shard import instance_exchange, pass_tail_forward
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sess = _sel_session(n_chunks, chunk)
    c0, c1 = shard_chunk_range(len(sess), world, rank)
    mine = sess[c0:c1]
    off, ch = instance_exchange([{"centers": c} for _, c in mine], [k for k, _ in mine],
                                InstanceTracker(1) if rank == 0 else None)
    # tail chain: a stand-in tail keyed by this shard's last session frame
    tail = None
    if mine:
        last = off + sum(len(k) for k, _ in mine) - 1
        tail = {last: (torch.full((2, 3, 5), rank, dtype=torch.uint8), np.full((2, 4, 3), float(last), np.float32),
                       np.array([1, 0]))}
    got = pass_tail_forward(tail)
    got = {g: (int(p[0, 0, 0]), float(k[0, 0, 0]), list(r)) for g, (p, k, r) in got.items()}
    q.put((rank, (off, c1 - c0, [{f: v for f, v in c.items()} for c in ch], got)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_chunks", [(2, 3), (3, 2)])
def test_instance_exchange_equals_sequential(mdx, world, n_chunks):
    """Rank 0 runs the instance tracker over every rank's frames in session
    order: the scattered picks equal one process's select_chunk chunk by chunk
    (incl. a rank without chunks), and each rank receives the preceding
    shard's tail (forwarded through a rank without frames)."""
    from moseq2_detectron_extract_amd.instances import InstanceTracker, select_chunk
    chunk = 60
    sess = _sel_session(n_chunks, chunk)
    tr = InstanceTracker(1)
    want, f0 = [], 0
    for nk, cen in sess:
        want.append(select_chunk(tr, nk, cen, f0))
        f0 += len(nk)
    assert sum(len(w) for w in want) > 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_select_worker, args=(r, world, port, q, n_chunks, chunk)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    flat = [c for r in sorted(got) for c in got[r][2]]
    assert flat == want
    last_tail = None
    for r in sorted(got):
        off, nch, _, tail = got[r]
        if r == 0:
            assert tail == {}
        else:
            assert tail == (last_tail or {})
        if nch:
            g = off + nch * chunk - 1
            last_tail = {g: (r, float(g), [1, 0])}


# ---------------------------------------------------------------- host pipeline
def test_host_pipeline_order_and_errors(mdx):
    """extract.host_pipeline (the overlapped chunk loop's worker hand-off):
    results in order; a consumer error part-way through a session of more
    than 3 chunks is raised without hanging (the queue holds 2), and so is a
    producer error and a setup error."""
    from moseq2_detectron_extract_amd.extract import host_pipeline
    assert host_pipeline(iter(range(7)), lambda i: i * i) == [i * i for i in range(7)]
    produced = []

    def gen(n):
        for i in range(n):
            produced.append(i)
            yield i

    def bad(i):
        if i == 2:
            raise RuntimeError("finish_chunk failed")
        return i

    with pytest.raises(RuntimeError, match="finish_chunk failed"):
        host_pipeline(gen(10), bad)
    assert len(produced) < 10  # production stopped early

    def bad_gen():
        yield 0
        yield 1
        raise ValueError("frame source failed")

    with pytest.raises(ValueError, match="frame source failed"):
        host_pipeline(bad_gen(), lambda i: i)

    def bad_setup():
        raise OSError("no stream")

    with pytest.raises(OSError, match="no stream"):
        host_pipeline(gen(6), lambda i: i, setup=bad_setup)


# ------------------------------------------------- one results file per session
class _FakeSrc:
    """What _ChunkWriter reads from the frame source."""

    def __init__(self, d, n):
        self.path = os.path.join(d, "depth.dat")
        self.last_frame_idx = n

    def read(self, idx):
        return np.full((len(idx), 424, 512), 7, np.int16)


def _fake_chunks(n, chunk, seed=3):
    """Writer data dicts of a synthetic session (float32 / float64 columns,
    NaNs, the reference's scalar and keypoint names)."""
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.features import keypoint_attributes, scalar_attributes
    rng = np.random.default_rng(seed)
    out = []
    for a in range(0, n, chunk):
        idx = np.arange(a, min(n, a + chunk))
        k = len(idx)
        cen = rng.normal(200, 30, (k, 2))
        cen[rng.random(k) < 0.1] = np.nan
        out.append({"frame_idxs": idx, "offset": 0,
                    "scalars": {s: rng.normal(0, 1, k).astype(np.float32) for s in scalar_attributes()},
                    "keypoints": {s: rng.normal(0, 50, k) for s in keypoint_attributes()},
                    "depth_frames": rng.integers(0, 255, (k, 80, 80), dtype=np.uint8),
                    "mask_frames": (rng.random((k, 80, 80)) < 0.3).astype(np.uint8),
                    "features": {"flips": rng.random(k) < 0.5,
                                 "features": {"centroid": cen, "orientation": rng.uniform(0, 360, k)}}})
    return out


def _writer_args(d, n):
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig
    cfg = ExtractConfig(chunk_size=50, model_streams=2)
    status = {"uuid": "0f0f", "parameters": dict(vars(cfg)), "metadata": {"SerialNumber": "x"}}
    roi = np.zeros((424, 512), np.uint8)
    roi[100:300, 100:400] = 1
    return (_FakeSrc(d, n), np.full((424, 512), 670.0), roi, 673.1, cfg, None, status)


def _gather_writer_worker(rank, world, port, q, out_dir, n, chunk):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.extract import _ChunkWriter, _GatherWriter, shard_chunk_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    chunks = _fake_chunks(n, chunk)
    c0, c1 = shard_chunk_range(len(chunks), world, rank)
    nrounds = len(range(*shard_chunk_range(len(chunks), world, 0)))
    local = _ChunkWriter(out_dir, *_writer_args(out_dir, n), parts=world) if rank == 0 else None
    w = _GatherWriter(local, nrounds)
    for d in chunks[c0:c1]:
        w.write(d)
    w.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, "ok"))


@pytest.mark.parametrize("world,n,chunk", [(2, 230, 50), (3, 100, 50)])
def test_sharded_writer_one_file_equals_one_process(mdx, tmp_path, world, n, chunk):
    """The ranks' chunks gathered round by round to rank 0 (gloo) make ONE
    results_00 file and keypoints_00.tsv equal to one process's, byte for
    byte: uneven shards (padding rounds) and a rank without chunks; rows
    arrive out of session order, and the crop stacks' deflate pieces are cut
    at absolute offsets, so the file does not depend on arrival order."""
    from moseq2_detectron_extract_amd.extract import _ChunkWriter
    from moseq2_detectron_extract_amd import results as RS
    one = tmp_path / "one"
    one.mkdir()
    w = _ChunkWriter(str(one), *_writer_args(str(one), n))
    for d in _fake_chunks(n, chunk):
        w.write(d)
    w.close()
    sh = tmp_path / "sharded"
    sh.mkdir()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_writer_worker, args=(r, world, port, q, str(sh), n, chunk))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert set(got.values()) == {"ok"}
    assert sorted(os.listdir(sh)) == sorted(os.listdir(one))  # no part files left behind
    assert (sh / "keypoints_00.tsv").read_bytes() == (one / "keypoints_00.tsv").read_bytes()
    assert (sh / "results_00.npz").read_bytes() == (one / "results_00.npz").read_bytes()
    z = np.load(str(one / "results_00.npz"))
    assert z["frames"].shape == (n, 80, 80) and z["frames"].any()


def _gather_writer_failing_worker(rank, world, port, q, out_dir, n, chunk, fail_rank, fail_at):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import time
    from datetime import timedelta
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd.extract import _ChunkWriter, _GatherWriter, shard_chunk_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=120))
    chunks = _fake_chunks(n, chunk)
    c0, c1 = shard_chunk_range(len(chunks), world, rank)
    nrounds = len(range(*shard_chunk_range(len(chunks), world, 0)))
    local = _ChunkWriter(out_dir, *_writer_args(out_dir, n), parts=world) if rank == 0 else None
    w = _GatherWriter(local, nrounds)
    t0 = time.time()
    res = "ok"
    try:
        for i, d in enumerate(chunks[c0:c1]):
            if rank == fail_rank and i == fail_at:
                raise ValueError("chunk failed")  # as extract_session: abort() on the way out
            w.write(d)
        w.close()
    except ValueError:
        w.abort()
        res = "failed"
    except RuntimeError as e:
        assert "another rank failed" in str(e), e
        w.abort()
        res = f"raised in round {w.done + 1}"
    q.put((rank, res, round(time.time() - t0, 1)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_at", [(2, 1, 1), (2, 0, 2), (3, 2, 0)])
def test_sharded_writer_rank_failure_ends_every_rank(mdx, tmp_path, world, fail_rank, fail_at):
    """A rank that fails in the middle of a sharded session's result rounds
    (as extract_session does on a chunk's exception: writer.abort()) makes
    every other rank raise in that same round, within seconds, instead of
    waiting in the gather for the process group's timeout; no part file is
    left behind."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n, chunk = 300, 50
    procs = [ctx.Process(target=_gather_writer_failing_worker,
                         args=(r, world, port, q, str(tmp_path), n, chunk, fail_rank, fail_at)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (res, t) for r, res, t in (q.get(timeout=90) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[fail_rank][0] == "failed"
    others = {got[r][0] for r in range(world) if r != fail_rank}
    assert others == {f"raised in round {fail_at + 1}"}, got
    assert max(t for _, t in got.values()) < 60, got
    assert not [f for f in os.listdir(tmp_path) if ".part" in f]


def test_deflate_stream_independent_of_arrival(mdx, tmp_path, monkeypatch):
    """The streamed crop member's bytes are the same whatever groups of rows
    arrive in which order (pieces cut at absolute _PIECE offsets), and equal
    to the member save_npz writes for the whole array at once."""
    from moseq2_detectron_extract_amd import results as RS
    monkeypatch.setattr(RS, "_PIECE", 4096)
    rng = np.random.default_rng(0)
    arr = rng.integers(0, 4, (300, 80, 80), dtype=np.uint8)
    outs = []
    for order in ([range(0, 300)], [range(200, 300), range(0, 120), range(120, 200)],
                  [range(i, min(300, i + 7)) for i in range(0, 300, 7)][::-1]):
        h = RS.MemoryH5(str(tmp_path / "a.npz"))
        ds = h.create_dataset("frames", (300, 80, 80), "uint8")
        for rows in order:
            ds[np.asarray(rows)] = arr[np.asarray(rows)]
            h.rows_written(np.asarray(rows))
        h.close()
        outs.append((tmp_path / "a.npz").read_bytes())
    assert outs[0] == outs[1] == outs[2]
    RS.save_npz(str(tmp_path / "b.npz"), {"frames": arr}, level=4)
    np.testing.assert_array_equal(np.load(str(tmp_path / "a.npz"))["frames"], arr)
