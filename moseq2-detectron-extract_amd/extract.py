"""Session-level driver of the hot path (the loop of M/extract.py:22-139
without its control plane): frame source -> GPUExtractor.process_chunk per
chunk -> results in the writer's layout (M/io/result.py:106-130), optionally
restricted to this rank's chunk-aligned shard.

The h5 writer itself is not rebuilt (h5py is absent from this image); the
results are returned as arrays keyed like the h5 datasets and can be saved as
``.npz``.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .pipeline import ExtractConfig, GPUExtractor
from .session import RawDepthSource


def shard_chunk_range(nchunks: int, world: int, rank: int):
    """[c0, c1): the chunks rank `rank` owns (shard.shard_chunks' dealing)."""
    q, rem = divmod(nchunks, world)
    c0 = rank * q + min(rank, rem)
    return c0, c0 + q + (1 if rank < rem else 0)


def extract_session(path: str, bground_im: np.ndarray, roi: np.ndarray, predictor,
                    config: ExtractConfig = ExtractConfig(), true_depth: float = 673.1,
                    frame_trim=(0, 0), world: int = 1, rank: int = 0, out_npz: Optional[str] = None) -> Dict:
    """Extract every chunk of the session (or of this rank's shard).  Returns
    {'frames': uint8 (n,80,80), 'frames_mask': uint8 (n,80,80),
    'scalars/<name>': (n,), 'keypoints/<name>': (n,), 'flips': bool (n,),
    'frame_idxs': (n,)} in frame order."""
    src = RawDepthSource(path, frame_trim=frame_trim)
    ex = GPUExtractor(bground_im, roi, predictor, config)
    batches = src.batches(config.chunk_size, config.chunk_overlap)
    if world > 1:  # contiguous block of whole chunks per rank, as shard.shard_chunks deals them
        c0, c1 = shard_chunk_range(len(batches), world, rank)
        batches = batches[c0:c1]
    parts = []
    for idx, raw in src.iterate(device=True, batches=batches):
        parts.append(ex.process_chunk(raw, np.asarray(idx), offset=0, true_depth=true_depth))
    src.close()
    out: Dict[str, np.ndarray] = {}
    if not parts:
        return out
    out["frame_idxs"] = np.concatenate([p["frame_idxs"] for p in parts])
    out["frames"] = np.concatenate([p["depth_frames"] for p in parts])
    out["frames_mask"] = np.concatenate([p["mask_frames"] for p in parts])
    out["flips"] = np.concatenate([p["features"]["flips"] for p in parts])
    for k in parts[0]["scalars"]:
        out[f"scalars/{k}"] = np.concatenate([np.asarray(p["scalars"][k]) for p in parts])
    for k in parts[0]["keypoints"]:
        out[f"keypoints/{k}"] = np.concatenate([np.asarray(p["keypoints"][k]) for p in parts])
    if out_npz:
        np.savez_compressed(out_npz, **out)
    return out
