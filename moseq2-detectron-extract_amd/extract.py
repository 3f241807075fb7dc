"""Session-level driver of the hot path (the loop of M/extract.py:22-139
without its control plane): frame source -> GPUExtractor.process_chunk per
chunk -> results in the writer's layout (M/io/result.py:106-130), optionally
restricted to this rank's chunk-aligned shard.

Sharded sessions (world > 1).  Each rank runs its contiguous block of whole
chunks.  With tracking or instance selection on (the reference's defaults)
the chunk loop runs in two device passes around the exchange step
(shard.instance_exchange / tracking_exchange): pass 1 runs the whole hot path
per chunk and keeps only a compact host record per frame (the kept
detections' mask logits and boxes, keypoints, keep indices: ~13 KB per
frame; GPUExtractor.features_pass_compact), so device memory stays one
chunk's working set however long the shard is; pass 2 re-runs each chunk's
front (prep + inpaint + clean, a few % of the forward) from its raw frames,
re-pastes the selected masks and crops at the exchanged pose.  The ranks'
finished chunks are gathered to rank 0 round by round over the process group
(shard.gather_chunk_results: RCCL over xGMI for nccl), where one writer fills
the session's single results_00 file and keypoints TSV -- the files one
process writes, byte for byte (ResultWriterStep's single writer,
M/pipeline/write_results_step.py:31-36).

With `output_dir` the session's results file is written through
results.open_results: a real ``results_00.h5`` when h5py is importable (its
tree equals the reference writer's, tests/test_results_h5.py), else the same
tree as ``results_00.npz``.  The results are also returned as arrays keyed
like the h5 datasets.
"""
from __future__ import annotations

import os
import uuid
from typing import Dict, Optional

import numpy as np

from .pipeline import ExtractConfig, GPUExtractor
from .results import (KeypointsTSVWriter, MemoryH5, check_completion_status, create_extract_h5, join_tsv_parts,
                      open_results, status_filename, write_extracted_chunk_to_h5, write_status)
from .session import RawDepthSource
from .shard import gather_chunk_results, instance_exchange, pass_tail_forward, tracking_exchange


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
    'frame_idxs': (n,)} in frame order, this rank's frames.  With
    `output_dir` the session's results_00 file, keypoints_00.tsv and status
    file are written there once (by rank 0 of a sharded session)."""
    tl = _Timeline()
    status_path = None
    if output_dir:  # status file first, as M/extract.py:47-62 (skip a completed session)
        os.makedirs(output_dir, exist_ok=True)
        status_path = status_filename(output_dir)
        done = skip_completed and check_completion_status(status_path)
        if world > 1:  # every rank must agree, or a skipping rank would leave the others in the exchange
            done = _all_ranks(done)
        if done:
            return {}
        status = status or {"complete": False, "skip": False, "uuid": str(uuid.uuid4()),
                            "metadata": _load_metadata(path), "parameters": dict(vars(config))}
        status["complete"] = False
        if rank == 0:
            write_status(status_path, status)
    src = RawDepthSource(path, frame_trim=frame_trim)
    src.timeline = tl if tl.path else None
    ex = GPUExtractor(bground_im, roi, predictor, config)
    batches = src.batches(config.chunk_size, config.chunk_overlap)
    nrounds = len(batches)
    if world > 1:  # contiguous block of whole chunks per rank, as shard.shard_chunks deals them
        c0, c1 = shard_chunk_range(len(batches), world, rank)
        nrounds = len(range(*shard_chunk_range(len(batches), world, 0)))  # rank 0 owns the most chunks
        batches = batches[c0:c1]
    # the results file and keypoints TSV are written chunk by chunk as chunks
    # finish (ResultWriterStep, its own process in the reference): one writer,
    # on rank 0, fed by the result gather when the session is sharded
    writer = None
    if output_dir:
        local = _ChunkWriter(output_dir, src, bground_im, roi, true_depth, config, first_frame, status,
                             parts=world) if rank == 0 else None
        writer = local if world == 1 else _GatherWriter(local, nrounds)
        if local is not None and tl.path:
            local.timeline = tl
    tl.add("session setup", -1, tl.t0)

    def finished(d):
        if writer is not None:
            writer.write(d)
        return _lighten(d)

    parts = []
    if exchange is None:  # two passes around the exchange step (needs torch.distributed initialised)
        exchange = world > 1 and (config.use_tracking or config.select_instances)
    err = None
    try:
        if exchange:
            parts = _run_two_pass(src, batches, ex, config, true_depth, finished)
        elif config.overlap_host:
            parts = _run_overlapped(src, batches, ex, true_depth, finished, tl)
        else:
            for idx, raw in src.iterate(device=True, batches=batches):
                parts.append(finished(ex.process_chunk(raw, np.asarray(idx), 0, true_depth)))
    except BaseException as e:  # propagated below, after the writer and the other ranks know
        err = e
    t0 = tl.now()
    src.close()
    ex.close()
    if writer is not None:
        if err is None:
            try:
                writer.close()
            except BaseException as e:
                err = e
        else:  # the extraction's own exception propagates; the results file is left unfinished
            writer.abort()
    tl.add("writer close", -1, t0)
    if output_dir and world > 1 and not _all_ranks(err is None) and err is None:
        # every rank completes or fails together: a rank whose writes all went
        # through still fails when another rank did (its status stays incomplete)
        err = RuntimeError("extract_session: another rank of the sharded session failed")
    if err is not None:
        raise err
    if output_dir:
        if rank == 0:
            status["complete"] = True  # M/extract.py:129-131
            write_status(status_path, status)
        if world > 1:  # no rank returns before the status file says complete
            _all_ranks(True)
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
    tl.dump()
    return out


def _run_two_pass(src, batches, ex, config, true_depth, finished):
    """The sharded session's chunk loop around the exchange step.  Pass 1:
    each chunk's hot path up to the host step, kept as a compact host record
    (GPUExtractor.features_pass_compact; the chunk's device frames are
    released).  Exchanges: the instance tracker's picks (instance_exchange +
    the tail hand-off, changed frames' moments recomputed), then the Kalman
    tracking (tracking_exchange).  Pass 2: each chunk's front again from its
    raw frames, the selected masks re-pasted, crops at the exchanged pose."""
    comps = []
    trace = _mem_trace()
    for idx, raw in src.iterate(device=True, batches=batches):
        comp, host = ex.features_pass_compact(raw)
        comps.append((np.asarray(idx), comp, host))
        trace(f"pass1 chunk {len(comps)}")
    if config.select_instances:  # the instance tracker is sequential over the session too
        _select_exchange_compact(ex, comps, src)
    else:
        for _, comp, host in comps:
            ex.apply_selection_compact(comp, host, {}, 0, {}, None)
    if config.use_tracking:
        tracked = tracking_exchange([h for _, _, h in comps], ex.point_tracker, ex.angle_tracker)
    else:  # per-chunk angle filtering: no sequential state across chunks
        tracked = [ex.host_angles(h) for _, _, h in comps]
    parts = []
    for (idx, comp, host), (cen, kp, ang, fl), (idx2, raw) in zip(comps, tracked,
                                                                 src.iterate(device=True, batches=batches)):
        if not np.array_equal(np.asarray(idx2), idx):
            raise RuntimeError("second pass: the frame source returned another chunk")
        parts.append(finished(ex.finish_chunk_compact(comp, raw, cen, kp, ang, fl, host["axis_length"], idx, 0,
                                                      true_depth)))
        trace(f"pass2 chunk {len(parts)}")
    comps.clear()
    return parts


def _mem_trace():
    """MDX_MEM_TRACE=1: device memory (torch allocator) after each chunk of
    the two-pass loop, on stderr (the sharded memory test reads it)."""
    if not os.environ.get("MDX_MEM_TRACE"):
        return lambda what: None
    import sys
    import torch

    def trace(what):
        torch.cuda.synchronize()
        print(f"[mdx mem] {what}: allocated {torch.cuda.memory_allocated() / 2**20:.1f} MB, "
              f"peak {torch.cuda.max_memory_allocated() / 2**20:.1f} MB", file=sys.stderr, flush=True)
    return trace


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

    def __init__(self, output_dir, src, bground_im, roi, true_depth, config, first_frame, status, parts: int = 1):
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
        # a sharded session's TSV: one headerless part per rank, joined in
        # rank (= session) order at close
        self.tsv_parts = [KeypointsTSVWriter(output_dir, path=f"{self.tsv.path}.part{r}", header=False)
                          for r in range(parts)] if parts > 1 else None
        self._remove_parts()  # an earlier failed run's parts (any world size) must not be joined
        self._cols = None
        self.timeline = None  # extract._Timeline when the extract loop is traced
        self._nwritten = 0
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
            d, part = d
            tl, k = self.timeline, self._nwritten
            self._nwritten += 1
            try:
                t0 = tl.now() if tl else 0
                write_extracted_chunk_to_h5(self.h5, d)
                t1 = tl.add("results rows", k, t0) if tl else 0
                if self.tsv_parts is None:
                    self.tsv.write(d)
                else:
                    if self._cols is None:
                        self._cols = list(KeypointsTSVWriter.columns(d))
                    self.tsv_parts[part].write(d)
                if tl:
                    tl.add("keypoints tsv", k, t1)
            except BaseException as e:  # surfaced by write() / close()
                self._err.append(e)

    def _remove_parts(self) -> None:
        """Delete every keypoints part file of this results index."""
        if self.tsv_parts is None:
            return
        import glob
        for p in glob.glob(glob.escape(self.tsv.path) + ".part*"):
            os.remove(p)

    def write(self, d: dict, part: int = 0) -> None:
        if self._err:
            raise self._err[0]
        f = d["features"]
        self._q.put(({"frame_idxs": d["frame_idxs"], "offset": d["offset"], "scalars": d["scalars"],
                      "keypoints": d["keypoints"], "depth_frames": d["depth_frames"], "mask_frames": d["mask_frames"],
                      "features": {"flips": f["flips"], "features": f["features"]}}, part))

    def close(self) -> None:
        self._q.put(None)
        self._t.join()
        if self._err:
            raise self._err[0]
        t0 = self.timeline.now() if self.timeline else 0
        if self.tsv_parts is not None and self._cols is not None:
            # only the parts written in this run (a rank without chunks has none)
            join_tsv_parts(self.tsv.path, self._cols, [w.path for w in self.tsv_parts if not w._fresh])
        self._remove_parts()
        self.h5.close()
        if self.timeline:
            self.timeline.add("results file close", -1, t0)

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
        self._remove_parts()
        if not isinstance(self.h5, MemoryH5):
            try:
                self.h5.close()
            except Exception:
                pass


def _select_exchange_compact(ex, comps, src):
    """Instance selection of a sharded session: rank 0 runs the tracker over
    every rank's frames in session order (shard.instance_exchange); each rank
    applies its picks to its compact chunk records, taking a pick at its
    shard's start from the preceding rank's last frames
    (shard.pass_tail_forward, compact logit records)."""
    import torch.distributed as dist
    tracker = ex.instance_tracker if dist.get_rank() == 0 else None
    off, changes = instance_exchange([h for _, _, h in comps], [c["nkeep"] for _, c, _ in comps], tracker)
    f0s, f = [], off
    for _, c, _ in comps:
        f0s.append(f)
        f += len(c["nkeep"])

    # this shard's tail for the next rank, chained from the preceding shard's
    # through its own chunks: a shard shorter than POINTWISE_HIT_COUNTER_MAX
    # frames still forwards the session's last frames
    def own_tail(got):
        t = got
        for (_, c, _), f0 in zip(comps, f0s):
            t = ex.chunk_tail_compact(c, f0, t)
        return t

    prev = pass_tail_forward(own_tail)
    for (idx, c, host), ch, f0 in zip(comps, changes, f0s):
        tail = ex.chunk_tail_compact(c, f0, prev)
        ex.apply_selection_compact(c, host, ch, f0, prev, lambda fr, idx=idx: src.read(idx[np.asarray(fr)]))
        prev = tail


class _GatherWriter:
    """The writer end of a sharded session: every rank hands its finished
    chunks here in order; each call is one round of
    shard.gather_chunk_results, after which rank 0's _ChunkWriter writes the
    round's chunks (one per rank, rank order; rows land at their frame
    indices, TSV rows in per-rank part files joined at close).  `nrounds`
    is the most chunks any rank owns: close() runs the rounds this rank has
    no chunk for.  Each round starts with an error flag (a MIN all-reduce):
    a rank that fails says so in the round it would have sent next
    (abort()), and every other rank raises in that same round instead of
    waiting in the gather."""

    def __init__(self, local, nrounds: int):
        self.local, self.nrounds, self.done, self.failed = local, nrounds, 0, False

    def _round(self, d) -> None:
        if not _all_ranks(True):
            self.failed = True
            raise RuntimeError(f"sharded session: another rank failed (result round {self.done + 1})")
        got = gather_chunk_results(d)
        self.done += 1
        if self.local is not None:
            for r, x in enumerate(got):
                if x is not None:
                    self.local.write(x, part=r)

    def write(self, d: dict) -> None:
        self._round(d)

    def close(self) -> None:
        while self.done < self.nrounds:
            self._round(None)
        if self.local is not None:
            self.local.close()

    def abort(self) -> None:
        if not self.failed and self.done < self.nrounds:
            self.failed = True  # this rank's failure, told to the others in its next round
            _all_ranks(False)
        if self.local is not None:
            self.local.abort()


def _lighten(d: dict) -> dict:
    """Drop a finished chunk's device frames (prepped, cleaned, masks: 650 KB
    per frame) once its host results exist; the writer needs none of them."""
    d["chunk"] = None
    d["features"]["cleaned_frames"] = None
    d["features"]["masks"] = None
    return d


def _run_overlapped(src, batches, ex, true_depth, finished=None, tl=None):
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
        # high priority: the worker's few small kernels (instance selection,
        # scalars, crops) are not queued behind the next chunk's forwards on
        # a shared hardware queue, so the host step keeps pace with the device
        ctx["ws"] = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])

    tl = tl or _Timeline()

    def produce():
        # the stream pipeline runs across chunk boundaries (features_stream)
        chunks = src.iterate(device=True, batches=batches)
        stream = ex.features_stream(chunks) if ex.cfg.stream_chunks else \
            ((idx, *ex.features_pass(raw)) for idx, raw in chunks)
        t0 = tl.now()
        for k, (idx, st, host) in enumerate(stream):
            tl.add("device pass", k, t0)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            yield np.asarray(idx), st, host, ev
            t0 = tl.now()

    def consume(item):
        idx, st, host, ev = item
        ws = ctx["ws"]
        ws.wait_event(ev)
        k = ctx["k"] = ctx.get("k", -1) + 1
        with torch.cuda.stream(ws):
            for t in (st["prepped"], st["d2"], st["cleaned"]):
                t.record_stream(ws)
            t0 = tl.now()
            ex.select_instances(st, host)
            t1 = tl.add("instance selection", k, t0)
            cen, kp, ang, fl = ex.host_angles(host)
            t2 = tl.add("host angles", k, t1)
            d = ex.finish_chunk(st, cen, kp, ang, fl, host["axis_length"], idx, 0, true_depth)
            t3 = tl.add("finish chunk", k, t2)
        out = finished(d) if finished is not None else _lighten(d)
        tl.add("writer hand-off", k, t3)
        return out

    return host_pipeline(produce(), consume, setup)


class _Timeline:
    """MDX_EXTRACT_TRACE=<path>: wall-clock spans of the extract loop's host
    phases per chunk (device pass on the producing thread; instance
    selection, angles, finish and writer hand-off on the worker), written as
    JSON at the end; no-op otherwise."""

    def __init__(self):
        import time
        self.path = os.environ.get("MDX_EXTRACT_TRACE")
        self.clock = time.perf_counter
        self.t0 = self.clock()
        self.events = []

    def now(self):
        return self.clock()

    def add(self, name, chunk, t0):
        t1 = self.clock()
        if self.path:
            self.events.append({"phase": name, "chunk": chunk, "start_s": round(t0 - self.t0, 4),
                                "end_s": round(t1 - self.t0, 4)})
        return t1

    def dump(self):
        if self.path:
            import json
            with open(self.path, "w") as fh:
                json.dump({"events": self.events, "total_s": round(self.clock() - self.t0, 4)}, fh, indent=0)


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
