"""Frame source of the extraction path: raw Kinect depth
files (``.dat``, little-endian int16, optionally inside a ``.tar.gz``) read in
chunks and streamed to HBM.

=============================  =============================================
this module                    reference (M/ = moseq2_detectron_extract/)
=============================  =============================================
get_raw_info                   M/io/video.py:28-56
frame_runs                     M/io/video.py:130-148 (collapse_consecutive_values)
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
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .shard import gen_batch_sequence


def get_raw_info(filename: Union[str, tarfile.TarInfo], bit_depth: int = 16, frame_dims: Tuple[int, int] = (512, 424)):
    """Size and frame count of a headerless raw depth file or tar member
    (M/io/video.py:28-56): {bytes, nframes, dims, bytes_per_frame}."""
    frame_bytes = frame_dims[0] * frame_dims[1] * bit_depth // 8
    total = filename.size if isinstance(filename, tarfile.TarInfo) else os.path.getsize(filename)
    return {"bytes": total, "nframes": total // frame_bytes, "dims": frame_dims, "bytes_per_frame": frame_bytes}


def frame_runs(frame_idxs: np.ndarray) -> List[Tuple[int, int, np.ndarray]]:
    """Runs of consecutive frame numbers in the sorted request: (first frame,
    length, positions in the request that receive the run's frames).  One
    file read serves a run (the reference's collapse_consecutive_values,
    M/io/video.py:130-148, plus the read-back positions in O(n log n))."""
    idx = np.asarray(frame_idxs, np.int64).ravel()
    if idx.size == 0:
        return []
    order = np.argsort(idx, kind="stable")
    srt = idx[order]
    cuts = np.flatnonzero(np.diff(srt) != 1) + 1
    return [(int(srt[p[0]]), len(p), order[p]) for p in np.split(np.arange(srt.size), cuts)]


def read_frames_raw(filename: Union[str, tarfile.TarInfo], frames=None, frame_dims: Tuple[int, int] = (512, 424),
                    bit_depth: int = 16, dtype="<i2", tar_object: Optional[tarfile.TarFile] = None,
                    out: Optional[np.ndarray] = None) -> np.ndarray:
    """Frames (n, H, W) of a raw depth file (or a member of `tar_object`) in
    the order of `frames` (an index, a sequence, or None / [] for every
    frame), one seek + read per run of consecutive frames (M/io/video.py:
    67-127).  `out` (e.g. a pinned host buffer view) receives them when
    given."""
    info = get_raw_info(filename, frame_dims=frame_dims, bit_depth=bit_depth)
    if frames is None or (not np.isscalar(frames) and len(frames) == 0):
        want = np.arange(info["nframes"], dtype=np.int64)
    else:
        want = np.atleast_1d(np.asarray(frames, np.int64))
    W, H = frame_dims
    dt = np.dtype(dtype)
    if out is None:
        out = np.empty((want.size, H, W), dtype=dt)
    runs = frame_runs(want)
    if isinstance(tar_object, tarfile.TarFile):
        fh = tar_object.extractfile(filename)
        if fh is None:
            raise FileNotFoundError(f"Could not open tar member: {getattr(filename, 'name', filename)}")

        def fetch(first, count):
            fh.seek(first * info["bytes_per_frame"])
            return np.frombuffer(fh.read(count * info["bytes_per_frame"]), dtype=dt)
    elif isinstance(filename, str):
        fh = open(filename, "rb")

        def fetch(first, count):
            fh.seek(first * info["bytes_per_frame"])
            return np.fromfile(fh, dtype=dt, count=count * H * W)
    else:
        raise ValueError("Could not read!")
    try:
        for first, count, dest in runs:
            first = max(first, 0)
            if isinstance(filename, str) and _direct_read(fh, out, first, count, dest, info["bytes_per_frame"], dt):
                continue
            out[dest] = fetch(first, count).reshape(count, H, W)
    finally:
        fh.close()
    return out


_READ_PIECE = 16 << 20  # bytes per pread of a large run (pieces read by parallel threads)


def _direct_read(fh, out: np.ndarray, first: int, count: int, dest: np.ndarray, bpf: int, dt) -> bool:
    """A run of frames whose destination rows are consecutive in a
    C-contiguous `out` of the file's byte order is read straight into those
    rows (no staging copy; into a pinned buffer that is the H2D source), a
    large run as parallel preads (the GIL is released while they read).
    False when the run does not qualify (the caller stages it)."""
    if not (out.flags.c_contiguous and out.dtype == dt and dt.isnative and count > 0
            and int(dest[0]) + count - 1 == int(dest[-1]) and (count == 1 or bool(np.all(np.diff(dest) == 1)))):
        return False
    row0 = int(dest[0])
    buf = memoryview(out[row0:row0 + count].reshape(-1).view(np.uint8))
    fd, base, total = fh.fileno(), first * bpf, count * bpf
    cuts = list(range(0, total, _READ_PIECE))

    def one(a):
        n = min(_READ_PIECE, total - a)
        got = 0
        while got < n:
            r = os.preadv(fd, [buf[a + got:a + n]], base + a + got)
            if r <= 0:
                raise ValueError(f"raw depth file ends before frame {first + count - 1}")
            got += r
    if len(cuts) == 1:
        one(0)
    else:
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(min(4, len(cuts))) as pool:
            list(pool.map(one, cuts))
    return True


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
        tl = getattr(self, "timeline", None)  # extract._Timeline when the extract loop is traced
        pinned = [None] * nbuf  # allocated by the reader on first use: the first read starts after one
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
                for k, idx in enumerate(seq):
                    b = free.get()
                    n = len(idx)
                    t0 = tl.now() if tl else 0
                    if pinned[b] is None:
                        pinned[b] = torch.empty((cap, H, W), dtype=torch.int16).pin_memory()
                    self.read(idx, out=pinned[b][:n].numpy())
                    if tl:
                        tl.add("read chunk", k, t0)
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
