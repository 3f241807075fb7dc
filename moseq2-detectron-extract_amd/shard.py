"""Frame sharding across the GPUs of one node.

One process per GPU.  A session's frames are split into contiguous,
chunk-aligned ranges (chunk = --chunk-size, M/cli.py:363; chunking as in
gen_batch_sequence, M/io/util.py:24-35), so every rank runs the hot path on
whole chunks with no data-path communication.  The only collective is the
final hand-off of per-frame results to rank 0 (the writer), an RCCL gather over
xGMI (``gather_to_rank0``); with the ``gloo`` backend the same code runs on CPU
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
    [r*q + min(r, rem), ...)), so shards differ by at most one chunk and every
    rank's range is contiguous (Kalman/tracking state stays rank-local)."""
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
