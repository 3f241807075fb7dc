"""Frame sharding across the GPUs of one node.

One process per GPU.  A session's frames are split into contiguous,
chunk-aligned ranges (chunk = --chunk-size, M/cli.py:363; chunking as in
gen_batch_sequence, M/io/util.py:24-35), so every rank runs the device hot
path on whole chunks with no data-path communication.  Collectives:

* ``tracking_exchange`` -- the one real exchange step.  With tracking on (the
  reference's default) the Kalman trackers are sequential over the whole
  session (M/proc/proc.py:737-800), so each rank sends its per-frame feature
  records (232 B/frame) to rank 0, rank 0 runs the tracking branch over all
  chunks in session order, and scatters the final centroid / angle / flip /
  keypoints (224 B/frame) back before the ranks crop.
* ``gather_to_rank0`` -- optional hand-off of per-frame results to one writer.

Both are RCCL (gather / scatter over xGMI) for GPU tensors and gloo for CPU
tensors (tests).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def gen_batch_sequence(nframes: int, chunk_size: int, overlap: int = 0, offset: int = 0) -> List[np.ndarray]:
    """Chunk index ranges, semantics of M/io/util.py:24-35."""
    seq = range(offset, nframes)
    out = []
    for i in range(offset, len(seq) - overlap, chunk_size - overlap):
        out.append(np.asarray(seq[i:i + chunk_size]))
    return out


def shard_chunks(nframes: int, chunk_size: int, world: int, rank: int) -> List[Tuple[int, int]]:
    """Chunk-aligned contiguous frame ranges [start, stop) owned by `rank`.
    Chunks are dealt in contiguous blocks (rank r gets chunks
    [r*q + min(r, rem), ...)), so shards differ by at most one chunk and rank
    order is session order (what tracking_exchange relies on)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    nchunks = (nframes + chunk_size - 1) // chunk_size
    q, rem = divmod(nchunks, world)
    c0 = rank * q + min(rank, rem)
    c1 = c0 + q + (1 if rank < rem else 0)
    return [(c * chunk_size, min((c + 1) * chunk_size, nframes)) for c in range(c0, c1)]


def shard_range(nframes: int, chunk_size: int, world: int, rank: int) -> Tuple[int, int]:
    ch = shard_chunks(nframes, chunk_size, world, rank)
    if not ch:
        return (0, 0)
    return ch[0][0], ch[-1][1]


def gather_to_rank0(tensor, group=None, dst: int = 0):
    """Gather equally-shaped per-rank result tensors to rank 0 (RCCL over xGMI
    for GPU tensors, gloo for CPU tensors).  Returns the list on rank 0, None
    elsewhere."""
    import torch.distributed as dist
    import torch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bufs = [torch.empty_like(tensor) for _ in range(world)] if rank == dst else None
    dist.gather(tensor.contiguous(), bufs, dst=dst, group=group)
    return bufs


def gather_ragged_to_rank0(tensor, group=None, dst: int = 0):
    """Gather per-rank tensors whose first dimension differs (last shard may
    be short): pad to the max length, gather, trim."""
    import torch
    import torch.distributed as dist
    n = torch.tensor([tensor.shape[0]], dtype=torch.int64, device=tensor.device)
    world = dist.get_world_size(group)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((m,) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    pad[:tensor.shape[0]] = tensor
    bufs = gather_to_rank0(pad, group, dst)
    if bufs is None:
        return None
    return [b[:int(s.item())] for b, s in zip(bufs, sizes)]


def _sizes(n: int, device, group=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([n], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [int(x.item()) for x in out]


def scatter_ragged_from_rank0(parts, n_local: int, sizes, width: int, dtype, device, group=None, src: int = 0):
    """Inverse of gather_ragged_to_rank0: rank `src` holds one (sizes[r],
    width) tensor per rank; every rank receives its own (n_local, width)."""
    import torch
    import torch.distributed as dist
    m = max(sizes) if sizes else 0
    out = torch.empty((m, width), dtype=dtype, device=device)
    lst = None
    if dist.get_rank(group) == src:
        lst = []
        for p in parts:
            buf = torch.zeros((m, width), dtype=dtype, device=device)
            buf[:p.shape[0]] = p
            lst.append(buf)
    dist.scatter(out, lst, src=src, group=group)
    return out[:n_local]


def tracking_exchange(host_chunks: List[Dict[str, np.ndarray]], point_tracker=None, angle_tracker=None,
                      group=None, device=None):
    """§8(e) exchange step for the tracking branch.  `host_chunks` are this
    rank's per-chunk host features (GPUExtractor.features_pass), in session
    order.  Rank 0 (whose trackers are used) tracks every rank's chunks in
    rank order, i.e. session order, exactly as one process would.  Returns
    this rank's [(centroid, keypoints, angles, flips)] per chunk."""
    import torch
    import torch.distributed as dist
    from . import tracking as TR
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    rank = dist.get_rank(group)
    K = host_chunks[0]["keypoints"].shape[1] if host_chunks else 8
    win, wout = 5 + 3 * K, 4 + 3 * K

    def rec(h):
        n = h["centroid"].shape[0]
        return np.concatenate([h["centroid"].reshape(n, 2), h["orientation"].reshape(n, 1),
                               h["axis_length"].reshape(n, 2), h["keypoints"].reshape(n, 3 * K)], axis=1)

    recs = np.concatenate([rec(h) for h in host_chunks]) if host_chunks else np.zeros((0, win))
    lens = np.array([h["centroid"].shape[0] for h in host_chunks], dtype=np.int64)
    sizes = _sizes(len(recs), device, group)
    t_rec = torch.from_numpy(np.ascontiguousarray(recs, dtype=np.float64)).to(device)
    t_len = torch.from_numpy(lens).to(device)
    all_rec = gather_ragged_to_rank0(t_rec, group)
    all_len = gather_ragged_to_rank0(t_len, group)
    parts = None
    if rank == 0:
        if point_tracker is None or angle_tracker is None:
            raise ValueError("rank 0 needs the trackers")
        parts = []
        for r_rec, r_len in zip(all_rec, all_len):
            r_rec = r_rec.cpu().numpy()
            outs, o = [], 0
            for ln in r_len.cpu().numpy().tolist():
                x = r_rec[o:o + ln]
                o += ln
                cen, kp, ang, fl = TR.track_features(point_tracker, angle_tracker, x[:, 0:2],
                                                     x[:, 5:].reshape(ln, K, 3), x[:, 2], x[:, 3:5])
                outs.append(np.concatenate([cen, ang.reshape(ln, 1), fl.reshape(ln, 1).astype(np.float64),
                                            kp.reshape(ln, 3 * K)], axis=1))
            parts.append(torch.from_numpy(np.concatenate(outs) if outs else np.zeros((0, wout))).to(device))
    mine = scatter_ragged_from_rank0(parts, len(recs), sizes, wout, torch.float64, device, group).cpu().numpy()
    res, o = [], 0
    for ln in lens.tolist():
        x = mine[o:o + ln]
        o += ln
        res.append((x[:, 0:2].copy(), x[:, 4:].reshape(ln, K, 3).copy(), x[:, 2].copy(), x[:, 3] != 0))
    return res


def instance_exchange(host_chunks: List[Dict[str, np.ndarray]], nkeeps: List[np.ndarray], tracker=None,
                      group=None, device=None):
    """§8(e) exchange step for the instance selection (A15): the norfair
    tracker is sequential over the whole session, tracking on or off.  Every
    rank sends its per-frame (nkeep, kept-detection centres) to rank 0, whose
    tracker (instances.InstanceTracker) runs over every rank's chunks in
    session order exactly as one process would; each rank gets back its
    frames' picks.  Returns (this rank's session frame offset, per chunk
    {chunk frame: [(session frame, kept slot), ...]} for the frames that
    change) -- what GPUExtractor.apply_selection consumes."""
    import torch
    import torch.distributed as dist
    from . import instances as INS
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    rank = dist.get_rank(group)
    D = host_chunks[0]["centers"].shape[1] if host_chunks else 1
    lens = np.array([len(k) for k in nkeeps], dtype=np.int64)
    recs = (np.concatenate([np.concatenate([np.asarray(k, np.float64).reshape(-1, 1), h["centers"].reshape(len(k), 2 * D)],
                                           axis=1) for k, h in zip(nkeeps, host_chunks)])
            if host_chunks else np.zeros((0, 1 + 2 * D)))
    sizes = _sizes(len(recs), device, group)
    offset = int(sum(sizes[:rank]))
    # per frame back: [npicked (-1 = unchanged), (session frame, slot) x expected]
    E_ = tracker.expected_instances if tracker is not None else 1
    E_t = torch.tensor([E_], dtype=torch.int64, device=device)
    dist.broadcast(E_t, 0, group=group)
    E_ = int(E_t.item())
    wout = 1 + 2 * E_
    all_rec = gather_ragged_to_rank0(torch.from_numpy(np.ascontiguousarray(recs)).to(device), group)
    parts = None
    if rank == 0:
        if tracker is None:
            raise ValueError("rank 0 needs the instance tracker")
        parts, f0 = [], 0
        for r_rec in all_rec:
            x = r_rec.cpu().numpy()
            n = len(x)
            out = np.full((n, wout), -1.0)
            ch = INS.select_chunk(tracker, x[:, 0].astype(np.int64), x[:, 1:].reshape(n, D, 2), f0)
            for f, sel in ch.items():
                out[f, 0] = len(sel)
                for e, (g, s) in enumerate(sel[:E_]):
                    out[f, 1 + 2 * e:3 + 2 * e] = (g, s)
            f0 += n
            parts.append(torch.from_numpy(out).to(device))
    mine = scatter_ragged_from_rank0(parts, len(recs), sizes, wout, torch.float64, device, group).cpu().numpy()
    res, o = [], 0
    for ln in lens.tolist():
        x = mine[o:o + ln]
        o += ln
        ch = {}
        for f in np.nonzero(x[:, 0] >= 0)[0].tolist():
            k = int(x[f, 0])
            ch[f] = [(int(x[f, 1 + 2 * e]), int(x[f, 2 + 2 * e])) for e in range(k)]
        res.append(ch)
    return offset, res


def _tail_dtypes():
    """Tail payload dtype by header code: 0 uint8 mask planes, 1 float32
    compact records (GPUExtractor.chunk_tail_compact)."""
    import torch
    return (torch.uint8, torch.float32)


def pass_tail_forward(tail: Optional[Dict], group=None, device=None):
    """Chain rank r-1 -> rank r of the last frames' kept detections (mask
    planes or compact logit records, keypoints, keep rows;
    instances.POINTWISE_HIT_COUNTER_MAX frames):
    a pick at the start of rank r's shard can be a detection of the previous
    shard's last frames.  `tail` is {session frame: (planes (D,h,w) uint8,
    keypoints (D,K,3), keep row (D,))}, a callable mapping the received tail
    to the one to send, or None for a rank without frames (it forwards what
    it received).  Returns the previous shard's tail ({} on
    rank 0)."""
    import torch
    import torch.distributed as dist
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    got: Dict = {}
    if rank > 0:
        hdr = torch.zeros(6, dtype=torch.int64, device=device)
        dist.recv(hdr, rank - 1, group=group)
        nf, D, h, w, K, code = (int(v) for v in hdr.tolist())
        if nf:
            planes = torch.empty((nf, D, h, w), dtype=_tail_dtypes()[code], device=device)
            meta = torch.empty((nf, 1 + D + D * K * 3), dtype=torch.float64, device=device)
            dist.recv(planes, rank - 1, group=group)
            dist.recv(meta, rank - 1, group=group)
            m = meta.cpu().numpy()
            for i in range(nf):
                got[int(m[i, 0])] = (planes[i], m[i, 1 + D:].reshape(D, K, 3).astype(np.float32),
                                     m[i, 1:1 + D].astype(np.int64))
    send = got if tail is None else (tail(got) if callable(tail) else tail)
    if rank < world - 1:
        keys = sorted(send)
        code = 0
        if keys:
            p0, k0, _ = send[keys[0]]
            D, h, w = (int(v) for v in p0.shape)
            K = int(np.asarray(k0).shape[1])
            code = _tail_dtypes().index(p0.dtype)
        else:
            D = h = w = K = 0
        hdr = torch.tensor([len(keys), D, h, w, K, code], dtype=torch.int64, device=device)
        dist.send(hdr, rank + 1, group=group)
        if keys:
            planes = torch.stack([send[g][0].to(device) for g in keys]).contiguous()
            meta = np.concatenate([np.array([[g] for g in keys], np.float64),
                                   np.stack([np.asarray(send[g][2], np.float64) for g in keys]),
                                   np.stack([np.asarray(send[g][1], np.float64).reshape(-1) for g in keys])], axis=1)
            dist.send(planes, rank + 1, group=group)
            dist.send(torch.from_numpy(np.ascontiguousarray(meta)).to(device), rank + 1, group=group)
    return got


# ----------------------------------------------------------------------------
# the result gather of a sharded session (one results file, written by rank 0)
# ----------------------------------------------------------------------------
def _result_columns(d: Dict) -> List[Tuple[str, np.ndarray]]:
    """The writer's fields of a finished chunk (_ChunkWriter.write), as
    per-frame columns in a fixed order (scalar / keypoint dict order kept:
    it is the TSV's column order)."""
    off = int(d.get("offset", 0))
    f = d["features"]
    cols = [("frame_idxs", np.asarray(d["frame_idxs"])), ("depth_frames", np.asarray(d["depth_frames"])[off:]),
            ("mask_frames", np.asarray(d["mask_frames"])[off:]), ("flips", np.asarray(f["flips"])[off:]),
            ("centroid", np.asarray(f["features"]["centroid"])[off:]),
            ("orientation", np.asarray(f["features"]["orientation"])[off:])]
    cols += [("scalars/" + k, np.asarray(v)[off:]) for k, v in d["scalars"].items()]
    cols += [("keypoints/" + k, np.asarray(v)[off:]) for k, v in d["keypoints"].items()]
    return cols


def pack_chunk_results(d: Dict):
    """A finished chunk's writer fields -> (schema JSON bytes, rows uint8
    (n, rowbytes)): every per-frame value's bytes side by side, so one byte
    tensor per chunk crosses the process group."""
    import json
    cols = _result_columns(d)
    n = len(cols[0][1])
    schema, parts = [], []
    for name, a in cols:
        a = np.ascontiguousarray(a)
        if len(a) != n:
            raise ValueError(f"pack_chunk_results: column {name} has {len(a)} rows, expected {n}")
        schema.append([name, a.dtype.str, list(a.shape[1:])])
        parts.append(a.reshape(n, -1).view(np.uint8) if a.size else np.zeros((n, 0), np.uint8))
    rows = np.concatenate(parts, axis=1) if parts else np.zeros((n, 0), np.uint8)
    return json.dumps(schema).encode(), np.ascontiguousarray(rows)


def unpack_chunk_results(schema: bytes, rows: np.ndarray) -> Dict:
    """Inverse of pack_chunk_results: the data dict _ChunkWriter.write
    consumes (offset 0)."""
    import json
    sch = json.loads(schema.decode())
    n = rows.shape[0]
    out, o = {}, 0
    for name, dt, shp in sch:
        dt = np.dtype(dt)
        w = dt.itemsize * int(np.prod(shp, dtype=np.int64))
        out[name] = np.ascontiguousarray(rows[:, o:o + w]).view(dt).reshape((n,) + tuple(shp))
        o += w
    d = {"frame_idxs": out["frame_idxs"], "offset": 0, "depth_frames": out["depth_frames"],
         "mask_frames": out["mask_frames"],
         "features": {"flips": out["flips"], "features": {"centroid": out["centroid"],
                                                          "orientation": out["orientation"]}},
         "scalars": {k[8:]: v for k, v in out.items() if k.startswith("scalars/")},
         "keypoints": {k[10:]: v for k, v in out.items() if k.startswith("keypoints/")}}
    return d


def gather_chunk_results(d: Optional[Dict], group=None, device=None, dst: int = 0):
    """One round of the sharded session's result gather: every rank passes
    its next finished chunk (None when it has no chunk left); rank `dst`
    gets [chunk dict or None per rank] in rank order, the others None.  The
    bytes travel as flat uint8 tensors through dist.gather (RCCL over xGMI
    with the nccl backend, gloo on the CPU)."""
    import torch
    import torch.distributed as dist
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    if d is None:
        sch, rows = b"", np.zeros((0, 0), np.uint8)
    else:
        sch, rows = pack_chunk_results(d)
    t_sch = torch.from_numpy(np.frombuffer(sch, np.uint8).copy()).to(device)
    t_rows = torch.from_numpy(rows.reshape(-1)).to(device)
    t_n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=device)
    all_n = gather_ragged_to_rank0(t_n, group, dst)
    all_sch = gather_ragged_to_rank0(t_sch, group, dst)
    all_rows = gather_ragged_to_rank0(t_rows, group, dst)
    if all_rows is None:
        return None
    res = []
    for n, s, r in zip(all_n, all_sch, all_rows):
        if s.numel() == 0:
            res.append(None)
            continue
        n = int(n.item())
        b = r.cpu().numpy()
        res.append(unpack_chunk_results(s.cpu().numpy().tobytes(), b.reshape(n, -1) if n else b.reshape(0, 0)))
    return res
