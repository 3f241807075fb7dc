"""Frame source of the extraction path: raw Kinect depth
files (``.dat``, little-endian int16, optionally inside a ``.tar.gz``) read in
chunks and streamed to HBM.

=============================  =============================================
this module                    reference (M/ = moseq2_detectron_extract/)
=============================  =============================================
get_raw_info                   M/io/video.py:28-56
collapse_consecutive_values    M/io/video.py:130-148
read_frames_raw                M/io/video.py:67-127
gen_batch_sequence             M/io/util.py:24-35 (shard.gen_batch_sequence)
RawDepthSource.iterate         Session.iterate / SessionFramesIterator
                               M/io/session.py:307-315, :352-466
attach_filter                  SessionFramesIterator.attach_filter :389-414
=============================  =============================================

MI355X side: ``RawDepthSource.iterate(..., device=True)`` reads chunk i+1
into a pinned host buffer on a reader thread and copies it to HBM on its own
HIP stream while the caller processes chunk i, so disk, PCIe and compute
overlap; filters (e.g. ``proc.FramePrep``) then run on the device tensor.
"""
from __future__ import annotations

import os
import queue
import tarfile
import threading
from itertools import groupby
from operator import itemgetter
from typing import Callable, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .shard import gen_batch_sequence


def get_raw_info(filename: Union[str, tarfile.TarInfo], bit_depth: int = 16, frame_dims: Tuple[int, int] = (512, 424)):
    """bytes / nframes / dims / bytes_per_frame of a raw depth file (M/io/video.py:28-56)."""
    bytes_per_frame = int((frame_dims[0] * frame_dims[1] * bit_depth) / 8)
    size = os.stat(filename).st_size if isinstance(filename, str) else filename.size
    return {"bytes": size, "nframes": int(size / bytes_per_frame), "dims": frame_dims,
            "bytes_per_frame": bytes_per_frame}


def collapse_consecutive_values(values: Iterable) -> List[Tuple[int, int]]:
    """[0,1,2,10,11] -> [(0, 3), (10, 2)] (M/io/video.py:130-148)."""
    out = []
    for _, group in groupby(enumerate(values), lambda ix: ix[0] - ix[1]):
        g = list(map(itemgetter(1), group))
        out.append((g[0], len(g)))
    return out


def read_frames_raw(filename: Union[str, tarfile.TarInfo], frames=None, frame_dims: Tuple[int, int] = (512, 424),
                    bit_depth: int = 16, dtype="<i2", tar_object: Optional[tarfile.TarFile] = None,
                    out: Optional[np.ndarray] = None) -> np.ndarray:
    """Frames (n, H, W) from a raw file, in the order of `frames` (None or []
    = all), reading each run of consecutive indices with one seek + read
    (M/io/video.py:67-127).  `out` (e.g. a pinned buffer view) receives the
    frames when given."""
    info = get_raw_info(filename, frame_dims=frame_dims, bit_depth=bit_depth)
    if isinstance(frames, (int, np.integer)):
        frames = [int(frames)]
    elif frames is not None:
        frames = [int(i) for i in frames]
    if frames is None or len(frames) == 0:
        frames = list(range(0, info["nframes"]))
    blocks = []
    for start, nfr in collapse_consecutive_values(sorted(frames)):
        blocks.append({"seek_point": int(np.maximum(0, start * info["bytes_per_frame"])),
                       "read_bytes": int(nfr * info["bytes_per_frame"]),
                       "read_points": int(nfr * frame_dims[0] * frame_dims[1]),
                       "dims": (nfr, frame_dims[1], frame_dims[0]),
                       "idxs": [frames.index(start + i) for i in range(nfr)]})
    if out is None:
        out = np.empty((len(frames), frame_dims[1], frame_dims[0]), dtype=np.dtype(dtype))
    if isinstance(tar_object, tarfile.TarFile):
        fh = tar_object.extractfile(filename)
        if fh is None:
            raise FileNotFoundError(f"Could not open tar member: {getattr(filename, 'name', filename)}")
        for blk in blocks:
            fh.seek(blk["seek_point"])
            out[blk["idxs"], ...] = np.frombuffer(fh.read(blk["read_bytes"]), dtype=np.dtype(dtype)).reshape(blk["dims"])
        fh.close()
    elif isinstance(filename, str):
        with open(filename, "rb") as fh:
            for blk in blocks:
                fh.seek(blk["seek_point"])
                chunk = np.fromfile(file=fh, dtype=np.dtype(dtype), count=blk["read_points"]).reshape(blk["dims"])
                out[blk["idxs"], ...] = chunk
    else:
        raise ValueError("Could not read!")
    return out


class RawDepthSource:
    """A depth session's frame source: a ``.dat`` path, or a ``.tar.gz`` and
    its depth member.  ``iterate`` mirrors SessionFramesIterator: chunks of
    ``chunk_size`` frames (``gen_batch_sequence``), filters applied in order."""

    def __init__(self, path: str, frame_dims: Tuple[int, int] = (512, 424), member: str = "depth.dat",
                 frame_trim: Tuple[int, int] = (0, 0)):
        self.path = path
        self.frame_dims = tuple(frame_dims)
        self.tar = None
        if path.endswith((".tar.gz", ".tgz", ".tar")):
            self.tar = tarfile.open(path, "r:*")
            self.depth_file = self.tar.getmember(member)
        else:
            self.depth_file = path
        info = get_raw_info(self.depth_file, frame_dims=self.frame_dims)
        # frame trim as Session.__init__ applies it (M/io/session.py:86-99)
        n = info["nframes"]
        self.first_frame_idx = int(frame_trim[0]) if 0 < frame_trim[0] < n else 0
        self.last_frame_idx = n - int(frame_trim[1]) if n - int(frame_trim[1]) > self.first_frame_idx else n
        self.nframes = self.last_frame_idx - self.first_frame_idx
        self.filters: List[Callable] = []

    def attach_filter(self, filterer: Callable) -> None:
        """Filters run in attachment order on every chunk (M/io/session.py:389-414)."""
        self.filters.append(filterer)

    def read(self, frame_idxs: Sequence[int], out: Optional[np.ndarray] = None) -> np.ndarray:
        return read_frames_raw(self.depth_file, list(frame_idxs), frame_dims=self.frame_dims, tar_object=self.tar,
                               out=out)

    def batches(self, chunk_size: int = 1000, chunk_overlap: int = 0):
        # exactly SessionFramesIterator.generate_samples (M/io/session.py:424):
        # the trimmed count with the first index as offset (with a leading
        # trim the reference's own sequence starts 2 x trim in and ends early;
        # kept, so chunk boundaries match the reference's)
        return gen_batch_sequence(self.nframes, chunk_size, chunk_overlap, self.first_frame_idx)

    def iterate(self, chunk_size: int = 1000, chunk_overlap: int = 0, device: bool = True, prefetch: int = 2,
                batches: Optional[List] = None):
        """Yield (frame_idxs, frames) per chunk, filters applied.  With
        device=True the frames are an int16 HIP tensor: a reader thread fills
        pinned host buffers and copies them to HBM on a copy stream `prefetch`
        chunks ahead of the consumer."""
        seq = batches if batches is not None else self.batches(chunk_size, chunk_overlap)
        if not device:
            for idx in seq:
                data = self.read(idx)
                for f in self.filters:
                    data = f(data)
                yield list(idx), data
            return
        yield from self._iterate_device(seq, prefetch)

    def _iterate_device(self, seq, prefetch):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("RawDepthSource.iterate(device=True) needs the GPU")
        W, H = self.frame_dims
        cap = max((len(s) for s in seq), default=0)
        nbuf = prefetch + 1
        pinned = [torch.empty((cap, H, W), dtype=torch.int16).pin_memory() for _ in range(nbuf)]
        free = queue.Queue()
        for i in range(nbuf):
            free.put(i)
        ready = queue.Queue(maxsize=prefetch)
        copy_stream = torch.cuda.Stream()
        dev = torch.cuda.current_device()
        err = []

        def reader():
            try:
                torch.cuda.set_device(dev)
                for idx in seq:
                    b = free.get()
                    n = len(idx)
                    self.read(idx, out=pinned[b][:n].numpy())
                    with torch.cuda.stream(copy_stream):
                        d = torch.empty((n, H, W), dtype=torch.int16, device="cuda")
                        d.copy_(pinned[b][:n], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(copy_stream)
                    ready.put((list(idx), d, ev, b))
            except BaseException as e:  # surfaced in the consumer
                err.append(e)
            finally:
                ready.put(None)

        t = threading.Thread(target=reader, daemon=True)
        t.start()
        while True:
            item = ready.get()
            if item is None:
                break
            idx, d, ev, b = item
            cur = torch.cuda.current_stream()
            cur.wait_event(ev)
            d.record_stream(cur)
            ev.synchronize()  # the pinned buffer may be refilled once its copy is done
            free.put(b)
            for f in self.filters:
                d = f(d)
            yield idx, d
        t.join()
        if err:
            raise err[0]

    def close(self):
        if self.tar is not None:
            self.tar.close()
