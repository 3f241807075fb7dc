"""Session-level driver of the hot path (the loop of M/extract.py:22-139
without its control plane): frame source -> GPUExtractor.process_chunk per
chunk -> results in the writer's layout (M/io/result.py:106-130), optionally
restricted to this rank's chunk-aligned shard.

With tracking on and more than one rank the chunk loop runs in two device
passes around the exchange step (shard.tracking_exchange): pass 1 keeps each
chunk's prepped / mask / cleaned frames resident in HBM (3 x 216 KB per frame:
a 1M-frame session over 8 GPUs holds ~81 GB per GPU, well inside 288 GB) and
ships its feature records to rank 0; pass 2 crops at the tracked values.

The h5 writer itself is not rebuilt (h5py is absent from this image); the
results are returned as arrays keyed like the h5 datasets and can be saved as
``.npz``.
"""
from __future__ import annotations

import os
import uuid
from typing import Dict, Optional

import numpy as np

from .pipeline import ExtractConfig, GPUExtractor
from .results import (KeypointsTSVWriter, MemoryH5, check_completion_status, create_extract_h5, open_results,
                      status_filename, write_extracted_chunk_to_h5, write_status)
from .session import RawDepthSource
from .shard import instance_exchange, pass_tail_forward, tracking_exchange


def shard_chunk_range(nchunks: int, world: int, rank: int):
    """[c0, c1): the chunks rank `rank` owns (shard.shard_chunks' dealing)."""
    q, rem = divmod(nchunks, world)
    c0 = rank * q + min(rank, rem)
    return c0, c0 + q + (1 if rank < rem else 0)


def extract_session(path: str, bground_im: np.ndarray, roi: np.ndarray, predictor,
                    config: ExtractConfig = ExtractConfig(), true_depth: float = 673.1,
                    frame_trim=(0, 0), world: int = 1, rank: int = 0, out_npz: Optional[str] = None,
                    exchange: Optional[bool] = None, output_dir: Optional[str] = None,
                    first_frame: Optional[np.ndarray] = None, status: Optional[dict] = None,
                    skip_completed: bool = True) -> Dict:
    """Extract every chunk of the session (or of this rank's shard).  Returns
    {'frames': uint8 (n,80,80), 'frames_mask': uint8 (n,80,80),
    'scalars/<name>': (n,), 'keypoints/<name>': (n,), 'flips': bool (n,),
    'frame_idxs': (n,)} in frame order."""
    status_path = None
    if output_dir:  # status file first, as M/extract.py:47-62 (skip a completed session)
        out_dir = output_dir if world == 1 else os.path.join(output_dir, f"rank{rank}")
        os.makedirs(out_dir, exist_ok=True)
        status_path = status_filename(out_dir)
        done = skip_completed and check_completion_status(status_path)
        if world > 1:  # every rank must agree, or a skipping rank would leave the others in the exchange
            done = _all_ranks(done)
        if done:
            return {}
        status = status or {"complete": False, "skip": False, "uuid": str(uuid.uuid4()),
                            "metadata": _load_metadata(path), "parameters": dict(vars(config))}
        status["complete"] = False
        write_status(status_path, status)
    src = RawDepthSource(path, frame_trim=frame_trim)
    ex = GPUExtractor(bground_im, roi, predictor, config)
    batches = src.batches(config.chunk_size, config.chunk_overlap)
    if world > 1:  # contiguous block of whole chunks per rank, as shard.shard_chunks deals them
        c0, c1 = shard_chunk_range(len(batches), world, rank)
        batches = batches[c0:c1]
    # the results file and keypoints TSV are written chunk by chunk as chunks
    # finish (ResultWriterStep, its own process in the reference)
    writer = _ChunkWriter(output_dir if world == 1 else os.path.join(output_dir, f"rank{rank}"), src, bground_im,
                          roi, true_depth, config, first_frame, status) if output_dir else None

    def finished(d):
        if writer is not None:
            writer.write(d)
        return _lighten(d)

    parts = []
    if exchange is None:  # two passes around the exchange step (needs torch.distributed initialised)
        exchange = world > 1 and (config.use_tracking or config.select_instances)
    ok = False
    try:
        if exchange:
            states = []
            for idx, raw in src.iterate(device=True, batches=batches):
                st, host = ex.features_pass(raw)
                states.append((np.asarray(idx), st, host))
            if config.select_instances:  # the instance tracker is sequential over the session too
                _select_exchange(ex, states)
            if config.use_tracking:
                tracked = tracking_exchange([h for _, _, h in states], ex.point_tracker, ex.angle_tracker)
            else:  # per-chunk angle filtering: no sequential state across chunks
                tracked = [ex.host_angles(h) for _, _, h in states]
            for (idx, st, host), (cen, kp, ang, fl) in zip(states, tracked):
                parts.append(finished(ex.finish_chunk(st, cen, kp, ang, fl, host["axis_length"], idx, 0,
                                                      true_depth)))
            states.clear()
        elif config.overlap_host:
            parts = _run_overlapped(src, batches, ex, true_depth, finished)
        else:
            for idx, raw in src.iterate(device=True, batches=batches):
                parts.append(finished(ex.process_chunk(raw, np.asarray(idx), 0, true_depth)))
        ok = True
    finally:
        src.close()
        if writer is not None:
            if ok:
                writer.close()
            else:  # the extraction's own exception propagates; the results file is left unfinished
                writer.abort()
    if output_dir:
        status["complete"] = True  # M/extract.py:129-131
        write_status(status_path, status)
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


def _all_ranks(flag: bool) -> bool:
    """True only if `flag` holds on every rank (MIN all-reduce; RCCL for the
    nccl backend, gloo on the CPU)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def _load_metadata(path: str) -> dict:
    """Session metadata.json next to the depth file (Session.load_metadata)."""
    import json
    f = os.path.join(os.path.dirname(os.path.abspath(path)), "metadata.json")
    if os.path.exists(f):
        with open(f, "r", encoding="utf-8") as fh:
            return json.load(fh)
    return {}


class _ChunkWriter:
    """ResultWriterStep (M/pipeline/write_results_step.py:24-73): results_00.h5
    (or .npz without h5py) + keypoints_00.tsv, the datasets created up front
    (create_extract_h5) and filled chunk by chunk.  As in the reference (its
    own process there), the writes run beside the extraction: write() hands a
    chunk's host results to a writer thread (in order, at most two queued),
    which fills the datasets, deflates the completed crop rows and appends
    the TSV; close() drains it and finishes the file."""

    def __init__(self, output_dir, src, bground_im, roi, true_depth, config, first_frame, status):
        os.makedirs(output_dir, exist_ok=True)
        ts_file = os.path.join(os.path.dirname(os.path.abspath(src.path)), "depth_ts.txt")
        nframes = src.last_frame_idx
        ts = np.loadtxt(ts_file)[:nframes] if os.path.exists(ts_file) else np.arange(nframes) * (1000 / 30)
        cfg = {"nframes": nframes, "crop_size": config.crop_size, "frame_dtype": "uint8", "timestamps": ts,
               "flip_classifier": "keypoints", "true_depth": true_depth, "roi": roi,
               "first_frame": first_frame if first_frame is not None else src.read([0])[0], "bground_im": bground_im}
        status = status or {"uuid": str(uuid.uuid4()), "parameters": {k: v for k, v in vars(config).items()},
                            "metadata": {}}
        self.h5 = open_results(output_dir)
        self.tsv = KeypointsTSVWriter(output_dir)
        create_extract_h5(self.h5, cfg, status)
        import queue
        import threading
        self._q: "queue.Queue" = queue.Queue(maxsize=2)
        self._err: list = []
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self) -> None:
        while True:
            d = self._q.get()
            if d is None:
                return
            if self._err:  # keep draining after an error so write() / close() never block
                continue
            try:
                write_extracted_chunk_to_h5(self.h5, d)
                self.tsv.write(d)
            except BaseException as e:  # surfaced by write() / close()
                self._err.append(e)

    def write(self, d: dict) -> None:
        if self._err:
            raise self._err[0]
        f = d["features"]
        self._q.put({"frame_idxs": d["frame_idxs"], "offset": d["offset"], "scalars": d["scalars"],
                     "keypoints": d["keypoints"], "depth_frames": d["depth_frames"], "mask_frames": d["mask_frames"],
                     "features": {"flips": f["flips"], "features": f["features"]}})

    def close(self) -> None:
        self._q.put(None)
        self._t.join()
        if self._err:
            raise self._err[0]
        self.h5.close()

    def abort(self) -> None:
        """Stop the writer thread after a failed extraction without finishing
        the results file and without raising: the extraction's exception is
        the one that propagates.  Without h5py nothing is written (the .npz
        is only saved by close()); an h5py file is closed as it stands, its
        status file still saying complete: False (M/extract.py:129-131), so
        the session is re-run."""
        self._err.append(RuntimeError("extraction failed"))  # the thread skips the queued chunks
        self._q.put(None)
        self._t.join()
        if not isinstance(self.h5, MemoryH5):
            try:
                self.h5.close()
            except Exception:
                pass


def _select_exchange(ex, states):
    """Instance selection of a sharded session: rank 0 runs the tracker over
    every rank's frames in session order (shard.instance_exchange); each rank
    gathers its picks, taking a pick at its shard's start from the preceding
    rank's last frames (shard.pass_tail_forward)."""
    import torch.distributed as dist
    tracker = ex.instance_tracker if dist.get_rank() == 0 else None
    off, changes = instance_exchange([h for _, _, h in states], [st["nkeep"] for _, st, _ in states], tracker)
    f0s, f = [], off
    for _, st, _ in states:
        f0s.append(f)
        f += len(st["nkeep"])
    # this shard's tail for the next rank, chained from the preceding shard's
    # through its own chunks: a shard shorter than POINTWISE_HIT_COUNTER_MAX
    # frames still forwards the session's last frames
    def own_tail(got):
        t = got
        for (_, st, _), f0 in zip(states, f0s):
            t = ex.chunk_tail(st, f0, t)
        return t

    prev = pass_tail_forward(own_tail)
    for (_, st, host), ch, f0 in zip(states, changes, f0s):
        tail = ex.chunk_tail(st, f0, prev)
        ex.apply_selection(st, host, ch, f0, prev)
        prev = tail


def _lighten(d: dict) -> dict:
    """Drop a finished chunk's device frames (prepped, cleaned, masks: 650 KB
    per frame) once its host results exist; the writer needs none of them."""
    d["chunk"] = None
    d["features"]["cleaned_frames"] = None
    d["features"]["masks"] = None
    return d


def _run_overlapped(src, batches, ex, true_depth, finished=None):
    """Chunk loop with the host step off the critical path: the calling thread
    runs each chunk's device pass (prep, model, clean, moments) and hands it
    to a worker thread, which runs the sequential host step (angles / Kalman
    tracking, in chunk order) and the small device tail (scalars, keypoint z,
    crops) on its own stream while the next chunk's device pass runs, then
    `finished` (the chunk writer) on the same thread."""
    import torch
    dev = torch.cuda.current_device()
    ctx = {}

    def setup():
        torch.cuda.set_device(dev)
        ctx["ws"] = torch.cuda.Stream()

    def produce():
        for idx, raw in src.iterate(device=True, batches=batches):
            st, host = ex.features_pass(raw)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            yield np.asarray(idx), st, host, ev

    def consume(item):
        idx, st, host, ev = item
        ws = ctx["ws"]
        ws.wait_event(ev)
        with torch.cuda.stream(ws):
            for t in (st["prepped"], st["d2"], st["cleaned"]):
                t.record_stream(ws)
            ex.select_instances(st, host)
            cen, kp, ang, fl = ex.host_angles(host)
            d = ex.finish_chunk(st, cen, kp, ang, fl, host["axis_length"], idx, 0, true_depth)
        return finished(d) if finished is not None else _lighten(d)

    return host_pipeline(produce(), consume, setup)


def host_pipeline(items, consume, setup=None, depth: int = 2):
    """Run consume(item) for every item of the iterator `items` on one worker
    thread, in order, while the calling thread produces the next ones (at most
    `depth` queued).  Returns the results in order.  The first error of either
    side stops production and is raised here; the worker keeps draining the
    queue after an error (it only skips the work), so neither the producer's
    put() nor the final sentinel can block on a dead consumer."""
    import queue
    import sys
    import threading
    q: "queue.Queue" = queue.Queue(maxsize=depth)
    out, err = [], []

    def worker():
        if setup is not None:
            try:
                setup()
            except BaseException as e:  # surfaced by the caller
                err.append(e)
        while True:
            item = q.get()
            if item is None:
                return
            if err:
                continue
            try:
                out.append(consume(item))
            except BaseException as e:  # surfaced by the caller
                err.append(e)

    # the worker's host step is many short numpy calls: a short GIL switch
    # interval keeps the producing thread from waiting out the default 5 ms
    old_si = sys.getswitchinterval()
    sys.setswitchinterval(1e-4)
    t = threading.Thread(target=worker, daemon=True)
    t.start()
    try:
        for item in items:
            if err:
                break
            q.put(item)
    finally:
        q.put(None)
        t.join()
        sys.setswitchinterval(old_si)
    if err:
        raise err[0]
    return out
