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

from typing import Dict, List, Sequence, Tuple

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
