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
