"""Device-resident extraction hot path for one GPU.

Replaces the chain ProduceFramesStep -> InferenceStep -> ProcessFeaturesStep
(M/pipeline/produce_frames_step.py:19-48, M/pipeline/inference_step.py:57-72,
M/pipeline/process_features_step.py:56-199) for one chunk of raw frames:

  prep_raw_frames (+NS inpaint)  -> scale_raw_frames (fused into the model's
  preprocess) -> Mask/Keypoint R-CNN forward (batch_size frames per launch
  sequence) -> mask-IoU NMS + instance-0 selection -> clean_frames ->
  get_frame_features (moments) -> [host: angle finalisation] ->
  crop_and_rotate_frame (depth and mask)

Everything between the int16 raw chunk and the 80x80 crops stays in HBM; the
only host traffic is the per-frame feature vector needed by the sequential
angle logic (A19, host-side in the reference too) and the results handed to
the writer.  The data-dict keys match the reference's steps so the writer and
h5 schema drop in unchanged.
"""
from __future__ import annotations

import collections
import ctypes
import threading
import weakref
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np
import torch

from . import features as F
from . import instances as INS
from . import proc
from . import tracking as TR
from ._lib import call


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def default_model_streams(hw_queues: Optional[int] = None) -> int:
    """Model streams for the hardware queues this process has (package
    HW_QUEUES, from GPU_MAX_HW_QUEUES).  Up to 8 queues: the front, tail and
    copy streams share two queues and every forward keeps one of its own, up
    to 4 forwards (at HIP's default of 4 queues a third forward lost 2 %).
    From 12 queues: 8 forwards (queues - 4), the measured plateau of the hot
    loop (4 / 6 / 8 / 12 / 16 forwards: 1491 / 1505 / 1525-1528 / 1528-1532 /
    1528 frames/s)."""
    if hw_queues is None:
        from . import HW_QUEUES as hw_queues
    q = int(hw_queues)
    return max(1, min(8, max(q - 4, min(4, q - 2))))


@dataclass
class ExtractConfig:
    """The extract CLI options on the hot path (M/cli.py:333-418 defaults)."""
    min_height: float = 0
    max_height: float = 100
    chunk_size: int = 1000
    chunk_overlap: int = 0
    batch_size: int = 32
    crop_size: Tuple[int, int] = (80, 80)
    frame_threshold: float = 3
    iters_tail: int = 3
    mask_iou_threshold: float = 0.5
    fix_invalid_pixels: bool = True
    use_tracking: bool = True        # --use-tracking/--no-use-tracking (M/cli.py:366), default on
    # forwards of consecutive batches in flight within a chunk: 8 at 12
    # hardware queues (the package default), as in the hot loop; 4 at 8 queues
    # (config-3 loop, 6000 frames, tracking off / on: 2 streams 1266 / 1293
    # frames/s, 3 streams 1293 / 1313 and 1294 / 1314, 4 streams 1315 / 1332;
    # profiles/r04_experiments.json), 2 at HIP's default of 4 queues
    # (default_model_streams)
    model_streams: int = field(default_factory=default_model_streams)
    overlap_host: bool = True        # extract loop: host angle/tracking step in a worker thread
    select_instances: bool = True    # norfair instance selection (process_features_step.py:133-160)
    expected_instances: int = 1      # --expected-instances (M/cli.py:341)
    pipelined: bool = True           # features_pass: batches staggered over streams (OverlappedExtractor)
    stream_chunks: bool = True       # extract loop: the stream pipeline runs across chunk boundaries


def mask_nms_select(out: dict, iou_thresh: float = 0.5):
    """GPU mask-IoU NMS + instance-0 selection over a forward's outputs.
    Returns (d2_mask uint8 (B,h,w), keypoints float64 (B,K,3), nkeep int32 (B,),
    keep_idx int32 (B,D))."""
    masks = out["masks"]
    B, D, h, w = masks.shape
    mbuf, plane = out.get("mask_planes", (None, None))
    if mbuf is None:
        mbuf, plane = masks.contiguous(), h * w
    K = out["keypoints"].shape[2]
    dev = masks.device
    keep_idx = torch.empty((B, D), dtype=torch.int32, device=dev)
    nkeep = torch.empty((B,), dtype=torch.int32, device=dev)
    sel = torch.empty((B, h, w), dtype=torch.uint8, device=dev)
    kp = torch.empty((B, K, 3), dtype=torch.float64, device=dev)
    call("mdx_mask_nms_select", _p(mbuf), int(plane), _p(out["scores"]), _p(out["ndet"]), _p(out["keypoints"]), B, D, K, h, w,
         float(iou_thresh), _p(keep_idx), _p(nkeep), _p(sel), _p(kp), _stream())
    return sel, kp, nkeep, keep_idx


def mask_centers(out: dict, keep_idx: torch.Tensor, nkeep: torch.Tensor):
    """Centres of the kept detections (center_of_mass of each kept mask, box
    centre when empty) for the instance tracker: float64 (B,D,2)."""
    masks = out["masks"]
    B, D, h, w = masks.shape
    mbuf, plane = out.get("mask_planes", (None, None))
    if mbuf is None:
        mbuf, plane = masks.contiguous(), h * w
    cen = torch.empty((B, D, 2), dtype=torch.float64, device=masks.device)
    call("mdx_mask_centers", _p(mbuf), int(plane), _p(keep_idx), _p(nkeep), _p(out["boxes"]), B, D, h, w, _p(cen),
         _stream())
    return cen


class GPUExtractor:
    """Chunk processor of the hot path on the current GPU."""

    def __init__(self, bground_im, roi, predictor, config: ExtractConfig = ExtractConfig()):
        self.cfg = config
        self.prep = proc.FramePrep(bground_im, roi, config.min_height, config.max_height, config.fix_invalid_pixels)
        self.lut = proc.scale_lut(config.min_height, config.max_height)
        self.predictor = predictor
        self.strel = proc.ELLIPSE9
        # ProcessFeaturesStep's Kalman trackers (process_features_step.py:40-51),
        # carried from chunk to chunk
        self.point_tracker, self.angle_tracker = TR.make_trackers() if config.use_tracking else (None, None)
        # ProcessFeaturesStep's norfair instance tracker (process_features_step.py:35-38), per session
        self.instance_tracker = INS.InstanceTracker(config.expected_instances)
        self._frames_seen = 0
        self._inpaint_errors_seen = 0  # of this extractor's own counter (FramePrep.inpaint_errors)
        self._tail_dets = {}  # session frame -> (mask planes (D,h,w), keypoints (D,K,3), keep_idx row)
        self._streams = []
        self._pipe = None     # OverlappedExtractor of the pipelined features pass
        self.keep_mask_logits = False  # set by the compact sharded passes (features_pass_compact)

    def infer(self, prepped: torch.Tensor):
        """Model forward over a prepped chunk in batch_size slices
        (InferenceStep.process); returns concatenated device outputs.  The
        slices alternate over `config.model_streams` HIP streams, so up to
        that many forwards are in flight (their small late kernels fill each
        other's gaps, as in OverlappedExtractor)."""
        outs = []
        n = prepped.shape[0]
        bs = min(self.cfg.batch_size, n)
        cur = torch.cuda.current_stream()
        ns = max(1, int(self.cfg.model_streams))
        if ns > 1 and n > bs:
            if len(self._streams) < ns:
                self._streams = [torch.cuda.Stream() for _ in range(ns)]
            ready = torch.cuda.Event()
            ready.record(cur)
        for k, i in enumerate(range(0, n, bs)):
            if ns > 1 and n > bs:
                st = self._streams[k % ns]
                st.wait_event(ready)
                with torch.cuda.stream(st):
                    prepped.record_stream(st)
                    o = self._infer_batch(prepped[i:i + bs])
                for v in o.values():
                    for t in (v if isinstance(v, (list, tuple)) else (v,)):
                        if torch.is_tensor(t):
                            t.record_stream(cur)
            else:
                o = self._infer_batch(prepped[i:i + bs])
            outs.append(o)
        if ns > 1 and n > bs:
            for st in self._streams[:ns]:
                cur.wait_stream(st)
        keys = ("boxes", "scores", "classes", "ndet", "keypoints", "d2_mask", "sel_keypoints", "nkeep", "keep_idx")
        keys += tuple(k for k in ("centers", "mask_logits") if k in outs[0])
        return {k: torch.cat([o[k] for o in outs]) for k in keys} | {"masks": [o["masks"] for o in outs]}

    def _infer_batch(self, x: torch.Tensor) -> dict:
        """One batch on the current stream: forward, mask NMS + instance 0,
        the kept detections' centres (instance selection on) and, for the
        compact sharded passes (keep_mask_logits), a copy of the mask head's
        logits (B, D, M, M) -- with the boxes, all mdx_paste_masks needs to
        re-make any detection's mask plane."""
        o = self.predictor.run(x, self.lut)
        sel, kp, nkeep, keep_idx = mask_nms_select(o, self.cfg.mask_iou_threshold)
        o.update(d2_mask=sel, sel_keypoints=kp, nkeep=nkeep, keep_idx=keep_idx)
        if self.cfg.select_instances:
            o["centers"] = mask_centers(o, keep_idx, nkeep)
        if self.keep_mask_logits:
            B, D = o["boxes"].shape[:2]
            lg = self.predictor.model.tensor("mask_logits")  # copied on this stream before the next forward
            o["mask_logits"] = lg.view(B, D, lg.shape[1], lg.shape[2])
        return o

    def select_instances(self, state: dict, host: dict):
        """ProcessFeaturesStep.__select_instances (process_features_step.py:
        133-160) over a chunk, after the GPU mask NMS: the kept detections'
        centres go through the session's norfair-semantics tracker on the host
        (instances.InstanceTracker), then apply_selection.  Part of the
        sequential host step (chunks in session order); rewrites state / host
        in place."""
        if "inf" not in state:
            return
        f0 = self._frames_seen
        changes = INS.select_chunk(self.instance_tracker, state["nkeep"], host["centers"], f0)
        tail = self.chunk_tail(state, f0, self._tail_dets)
        self.apply_selection(state, host, changes, f0, self._tail_dets)
        self._tail_dets = tail
        self._frames_seen = f0 + len(state["nkeep"])

    def chunk_tail(self, state: dict, f0: int, prev_tail: Optional[dict] = None) -> dict:
        """The session's last POINTWISE_HIT_COUNTER_MAX frames' kept detections
        up to the end of this chunk {session frame: (mask planes (D,h,w),
        keypoints (D,K,3), keep row (D,))}: the tracker's live objects are at
        most that many frames old, so these are all a later chunk's picks can
        refer to.  A chunk shorter than that window keeps the frames of
        `prev_tail` (the preceding chunk's tail, any rank) still inside it."""
        inf = state["inf"]
        masks = inf["masks"]
        bs = masks[0].shape[0]
        n = len(state["nkeep"])
        lo = f0 + n - INS.POINTWISE_HIT_COUNTER_MAX  # first session frame of the window
        a = max(0, n - INS.POINTWISE_HIT_COUNTER_MAX)
        kp = inf["keypoints"][a:].cpu().numpy()
        keep = inf["keep_idx"][a:].cpu().numpy()
        out = {g: v for g, v in (prev_tail or {}).items() if lo <= g < f0}
        out.update({f0 + f: (masks[f // bs][f % bs].clone(), kp[f - a], keep[f - a]) for f in range(a, n)})
        return out

    def apply_selection(self, state: dict, host: dict, changes: dict, f0: int, prev_tail: dict):
        """Frames whose picked instance differs from the NMS result get the
        picked detection's mask plane gathered into the d2 masks on the
        device (one mdx_gather_planes launch) and its keypoints;
        num_instances = the number picked; the chunk's moments are then
        recomputed.  `changes` = {chunk frame: [(session frame, kept slot)]},
        `prev_tail` = chunk_tail of the preceding chunk (any rank)."""
        inf = state.pop("inf", None)
        if inf is None or not changes:
            return
        nkeep = state["nkeep"].astype(np.int64)
        masks = inf["masks"]
        bs = masks[0].shape[0]
        keep = inf["keep_idx"].cpu().numpy()
        d2 = state["d2"]
        kph = host["keypoints"]
        det_kp = inf["keypoints"].cpu().numpy()
        hw = d2.shape[1] * d2.shape[2]
        src, dst = [], []
        for f, sel in sorted(changes.items()):
            nkeep[f] = len(sel)
            dst.append(f)
            if not sel:
                src.append(0)
                kph[f] = np.nan
                continue
            g, slot = sel[0]
            if g >= f0:
                j = int(keep[g - f0, slot])
                src.append(masks[(g - f0) // bs][(g - f0) % bs, j].data_ptr())
                kph[f] = det_kp[g - f0, j]
            else:  # a detection of the preceding chunk's last frames
                planes, kps, krow = prev_tail[g]
                if not planes.is_cuda or planes.device != d2.device:
                    # received over a CPU (gloo) group: the gather kernel reads device memory only
                    planes = planes.to(d2.device)
                    prev_tail[g] = (planes, kps, krow)
                j = int(krow[slot])
                src.append(planes[j].data_ptr())
                kph[f] = kps[j]
        tab = torch.from_numpy(np.asarray(src, dtype=np.uint64).view(np.int64)).to(d2.device)
        didx = torch.from_numpy(np.asarray(dst, dtype=np.int32)).to(d2.device)
        for c in range(0, len(dst), 65535):
            call("mdx_gather_planes", _p(tab[c:]), _p(didx[c:]), _p(d2), hw, min(65535, len(dst) - c), _stream())
        feats = proc.frame_moments(state["cleaned"], d2, float(self.cfg.frame_threshold))
        for k in ("centroid", "orientation", "axis_length"):
            host[k] = feats[k].cpu().numpy()
        state["nkeep"] = nkeep
        # the gathers read the chunk's mask planes, freed on return
        torch.cuda.current_stream().synchronize()

    def features(self, prepped: torch.Tensor, d2_mask: torch.Tensor):
        """clean_frames(iters_tail=3) + get_frame_features(mask=d2, thr=3)."""
        cleaned = proc.clean_frames(prepped, iters_tail=self.cfg.iters_tail, strel_tail=self.strel)
        feats = proc.frame_moments(cleaned, d2_mask, float(self.cfg.frame_threshold))
        return cleaned, feats

    def crop(self, prepped, d2_mask, centroid, angle_deg):
        return proc.crop_and_rotate_frames(prepped, centroid, angle_deg, self.cfg.crop_size, frames2=d2_mask)

    def step_device(self, raw: torch.Tensor):
        """One pass over a batch with the angle computed on the device
        (clamp_angles_deg(-rad2deg(orientation)), the non-tracking path
        before flip correction).  Used by bench.py; returns the crops."""
        return self.back(*self.front(raw))

    def front(self, raw: torch.Tensor):
        """Model-independent head of the path: prep (+inpaint) and clean."""
        prepped = self.prep(raw)
        cleaned = proc.clean_frames(prepped, iters_tail=self.cfg.iters_tail, strel_tail=self.strel)
        return prepped, cleaned

    def front_chunk(self, raw: torch.Tensor):
        """front() over a chunk in batch_size slices (the same per-frame
        results): the inpaint / clean workspaces stay one batch's size."""
        n = raw.shape[0]
        B = max(1, int(self.cfg.batch_size))
        if n <= B:
            return self.front(raw)
        y0, y1, x0, x1 = self.prep.crop(raw.shape[1], raw.shape[2])
        prepped = torch.empty((n, y1 - y0, x1 - x0), dtype=torch.uint8, device=raw.device)
        cleaned = torch.empty_like(prepped)
        for i in range(0, n, B):
            p, c = self.front(raw[i:i + B])
            prepped[i:i + B].copy_(p)
            cleaned[i:i + B].copy_(c)
        return prepped, cleaned

    def close(self) -> None:
        """Release the extractor's device state now (the pipeline, its
        streams and results, the prep workspaces) rather than when the
        cyclic garbage collector gets to the extractor <-> pipeline cycle."""
        if self._pipe is not None and self._pipe.streams is not None:
            _checkin_streams(self.predictor, self._pipe.streams)
        self._pipe = None
        self._streams = []
        self.prep._ws = None

    def tail(self, prepped: torch.Tensor, cleaned: torch.Tensor, inf: dict):
        """Moments of the selected mask, angle, crops."""
        feats = proc.frame_moments(cleaned, inf["d2_mask"], float(self.cfg.frame_threshold))
        ang = -torch.rad2deg(feats["orientation"])
        ang = torch.where(ang < 0, 360 + ang, ang) % 360
        depth, mask = self.crop(prepped, inf["d2_mask"], feats["centroid"], ang)
        return {"depth_frames": depth, "mask_frames": mask, "centroid": feats["centroid"], "angle": ang,
                "axis_length": feats["axis_length"], "keypoints": inf["sel_keypoints"], "ndet": inf["ndet"],
                "orientation": feats["orientation"]}

    def features_pass(self, raw):
        """Device part of one chunk up to the sequential host step: prep
        (+inpaint), model + mask NMS + instance 0, clean, moments.  Returns
        (device state kept for finish_chunk, host per-frame features
        {centroid, orientation (rad), axis_length, keypoints (n,K,3)})."""
        raw = raw if isinstance(raw, torch.Tensor) and raw.is_cuda else torch.from_numpy(np.ascontiguousarray(raw)).cuda()
        if self.cfg.pipelined and raw.shape[0] > self.cfg.batch_size:
            return self._features_pass_pipelined(raw)
        prepped = self.prep(raw)
        inf = self.infer(prepped)
        d2 = inf["d2_mask"]
        cleaned, feats = self.features(prepped, d2)
        host = {"centroid": feats["centroid"].cpu().numpy(), "orientation": feats["orientation"].cpu().numpy(),
                "axis_length": feats["axis_length"].cpu().numpy(), "keypoints": inf["sel_keypoints"].cpu().numpy()}
        state = {"prepped": prepped, "d2": d2, "cleaned": cleaned, "nkeep": inf["nkeep"].cpu().numpy()}
        if self.keep_mask_logits:  # features_pass_compact's inputs (no mask planes)
            state["inf"] = {k: inf[k] for k in ("keypoints", "keep_idx", "mask_logits", "boxes")}
        elif self.cfg.select_instances:  # inputs of the host instance-selection step (select_instances)
            state["inf"] = {k: inf[k] for k in ("masks", "keypoints", "keep_idx", "sel_keypoints")}
        if self.cfg.select_instances:
            host["centers"] = inf["centers"].cpu().numpy()
        return state, host

    def _features_pass_pipelined(self, raw: torch.Tensor):
        """features_pass with the chunk's batch_size slices staggered over the
        streams of an OverlappedExtractor (front: prep + inpaint + clean,
        forwards + mask selection on model_streams streams, tail: moments):
        the frame stages of one slice run beside the forwards of the next
        ones, as in the bench loop.  Same results as the serial pass (the
        kernels and their inputs are the same; the streams only reorder)."""
        B = self.cfg.batch_size
        pipe = self._pipeline(raw[:B])
        outs = []
        for i in range(0, raw.shape[0], B):
            r = pipe.submit(raw[i:i + B])
            if r is not None:
                outs.append(r)
        outs.extend(pipe.flush())  # the current stream now waits for every stage
        return self._collect(outs)

    def features_stream(self, chunks):
        """features_pass over a sequence of (key, raw) chunks with the stream
        pipeline running across chunk boundaries: the next chunk's first
        batches are submitted before the current chunk's last results are
        collected, so the streams do not drain (and refill) at every chunk.
        Yields (key, state, host) per chunk, in order, equal to
        features_pass(raw) of that chunk (same kernels and inputs; the
        streams only reorder)."""
        if not self.cfg.pipelined:
            for key, raw in chunks:
                yield (key, *self.features_pass(raw))
            return
        B = self.cfg.batch_size
        pipe = None
        pending = collections.deque()  # [key, nbatches, results, raw] per chunk, submission order

        def done():
            while pending and len(pending[0][2]) == pending[0][1]:
                key, _, outs, _ = pending.popleft()
                for o in outs:  # the caller's stream waits for exactly these batches
                    OverlappedExtractor.wait(o)
                yield (key, *self._collect(outs))

        for key, raw in chunks:
            raw = raw if isinstance(raw, torch.Tensor) and raw.is_cuda else \
                torch.from_numpy(np.ascontiguousarray(raw)).cuda()
            if pipe is None:
                pipe = self._pipeline(raw[:B])
            n = raw.shape[0]
            pending.append([key, (n + B - 1) // B, [], raw])
            for i in range(0, n, B):
                r = pipe.submit(raw[i:i + B])
                if r is not None:  # results come out in submission order: the oldest open chunk's
                    pending[0][2].append(r)
                    yield from done()
        if pipe is not None:
            for r in pipe.flush():
                pending[0][2].append(r)
                yield from done()

    def _pipeline(self, first: torch.Tensor):
        if self._pipe is None:
            sset = _checkout_streams(self.predictor, max(1, int(self.cfg.model_streams)))
            self._pipe = OverlappedExtractor(self, len(sset.models), keep=True, streams=sset)
            if not sset.primed:
                self._pipe.prime(first)
                sset.primed = True
        return self._pipe

    def _collect(self, outs):
        """One chunk's pipeline results -> (device state, host features)."""
        cat = lambda key: torch.cat([o[key] for o in outs])  # noqa: E731
        icat = lambda key: torch.cat([o["inf"][key] for o in outs])  # noqa: E731
        if self.keep_mask_logits:  # the compact pass keeps no device frames
            prepped = cleaned = d2 = None
        else:
            prepped, cleaned, d2 = cat("prepped"), cat("cleaned"), icat("d2_mask")
        host = {"centroid": cat("centroid").cpu().numpy(), "orientation": cat("orientation").cpu().numpy(),
                "axis_length": cat("axis_length").cpu().numpy(), "keypoints": icat("sel_keypoints").cpu().numpy()}
        state = {"prepped": prepped, "d2": d2, "cleaned": cleaned, "nkeep": icat("nkeep").cpu().numpy()}
        if self.keep_mask_logits:  # features_pass_compact's inputs (no mask planes)
            state["inf"] = {k: icat(k) for k in ("keypoints", "keep_idx", "mask_logits", "boxes")}
        elif self.cfg.select_instances:
            state["inf"] = {"masks": [m for o in outs for m in o["inf"]["masks"]], "keypoints": icat("keypoints"),
                            "keep_idx": icat("keep_idx"), "sel_keypoints": icat("sel_keypoints")}
        if self.cfg.select_instances:
            host["centers"] = icat("centers").cpu().numpy()
        return state, host

    def finish_chunk(self, state: dict, centroid, keypoints, angles, flips, axis_length, frame_idxs=None,
                     offset: int = 0, true_depth: float = 673.1) -> dict:
        """Device part after the host angle step: scalar reductions + keypoint
        z at the final keypoints, host scalar / keypoint tables, crops at the
        final centroid and angle; returns the writer's data dict."""
        cfg = self.cfg
        prepped, d2, cleaned = state["prepped"], state["d2"], state["cleaned"]
        n = prepped.shape[0]
        frame_idxs = np.arange(n) if frame_idxs is None else np.asarray(frame_idxs)
        area, hmean, z = F.frame_scalars(prepped, d2, cfg.min_height, cfg.max_height,
                                         keypoints=np.ascontiguousarray(keypoints, dtype=np.float64), z_frames=cleaned)
        track = {"centroid": centroid, "orientation": np.array(angles), "axis_length": axis_length, "contour": []}
        scalars = F.compute_scalars(None, track, cfg.min_height, cfg.max_height, true_depth,
                                    reductions=(area.cpu().numpy(), hmean.cpu().numpy()))
        kpd = F.keypoints_to_dict(keypoints, None, centroid, track["orientation"], true_depth=true_depth,
                                  z_data=z.cpu().numpy())
        depth, mask = self.crop(prepped, d2, torch.from_numpy(np.ascontiguousarray(centroid, dtype=np.float64)).cuda(),
                                torch.from_numpy(track["orientation"]).cuda())
        self._check_inpaint()
        return {
            "chunk": prepped, "frame_idxs": frame_idxs, "offset": offset,
            "features": {"cleaned_frames": cleaned, "masks": d2, "features": track, "flips": flips,
                         "keypoints": keypoints, "num_instances": state["nkeep"]},
            "scalars": scalars, "keypoints": kpd,
            "depth_frames": depth.cpu().numpy(), "mask_frames": mask.cpu().numpy(),
        }

    # ------------------------------------------------------------------
    # compact chunk state of the sharded two-pass session (extract.py)
    # ------------------------------------------------------------------
    def features_pass_compact(self, raw):
        """features_pass for the sharded session's first pass, keeping O(1)
        device memory across chunks: the chunk's prepped / cleaned / d2 frames
        and mask planes are released when this returns, and what the
        exchanges and the second pass need is kept on the host in compact
        form -- per frame the kept detections' mask logits (D x M x M fp32)
        and boxes (re-pasted on the device by mdx_paste_masks, bit-identical
        to the forward's planes), their keypoints, keep_idx and nkeep:
        ~13 KB per frame against ~1.5 MB of device planes.  Returns
        (compact, host features)."""
        raw = raw if isinstance(raw, torch.Tensor) and raw.is_cuda else torch.from_numpy(np.ascontiguousarray(raw)).cuda()
        self.keep_mask_logits = True
        try:
            state, host = self.features_pass(raw)
        finally:
            self.keep_mask_logits = False
        inf = state.pop("inf")
        comp = {"nkeep": state["nkeep"].astype(np.int64), "keep_idx": inf["keep_idx"].cpu().numpy(),
                "det_kp": inf["keypoints"].cpu().numpy(), "logits": inf["mask_logits"].cpu().numpy(),
                "boxes": inf["boxes"].cpu().numpy(), "device": raw.device}
        return comp, host

    def _sel_default(self, comp) -> None:
        """Instance 0 of every frame (mask_nms_select's choice): the record
        the second pass pastes as the frame's d2 mask."""
        n = len(comp["nkeep"])
        j = np.maximum(comp["keep_idx"][:, 0], 0)
        comp["sel_logits"] = comp["logits"][np.arange(n), j].copy()
        comp["sel_box"] = comp["boxes"][np.arange(n), j].copy()
        comp["sel_has"] = (comp["nkeep"] > 0).astype(np.int32)

    def chunk_tail_compact(self, comp, f0: int, prev_tail: Optional[dict] = None) -> dict:
        """chunk_tail over a compact chunk: {session frame: (record float32
        (D, 1, M*M + 4) = logits | box per detection, keypoints (D,K,3), keep
        row (D,))} of the session's last POINTWISE_HIT_COUNTER_MAX frames up
        to the end of this chunk (shard.pass_tail_forward ships these)."""
        n = len(comp["nkeep"])
        lo = f0 + n - INS.POINTWISE_HIT_COUNTER_MAX
        a = max(0, n - INS.POINTWISE_HIT_COUNTER_MAX)
        out = {g: v for g, v in (prev_tail or {}).items() if lo <= g < f0}
        D = comp["logits"].shape[1]
        for f in range(a, n):
            rec = np.concatenate([comp["logits"][f].reshape(D, -1), comp["boxes"][f]], axis=1)
            out[f0 + f] = (torch.from_numpy(np.ascontiguousarray(rec, np.float32)).view(D, 1, -1),
                           comp["det_kp"][f], comp["keep_idx"][f])
        return out

    def apply_selection_compact(self, comp, host: dict, changes: dict, f0: int, prev_tail: dict, raw_reader):
        """apply_selection over a compact chunk: the picked detection's logits
        and box become the frame's d2 record (pasted in the second pass), its
        keypoints the frame's, num_instances the number picked; the changed
        frames' moments are recomputed on the device from their raw frames
        (raw_reader(chunk frame indices) -> int16 (k,H,W); prep, inpaint and
        clean are per-frame, so equal to the chunk's) and the re-pasted mask.
        Drops the chunk's all-detection records afterwards."""
        self._sel_default(comp)
        if changes:
            nkeep, kph = comp["nkeep"], host["keypoints"]
            M2 = comp["logits"].shape[2] * comp["logits"].shape[3]
            fr = sorted(changes)
            for f in fr:
                sel = changes[f]
                nkeep[f] = len(sel)
                if not sel:
                    comp["sel_has"][f] = 0
                    kph[f] = np.nan
                    continue
                g, slot = sel[0]
                comp["sel_has"][f] = 1
                if g >= f0:
                    j = int(comp["keep_idx"][g - f0, slot])
                    comp["sel_logits"][f] = comp["logits"][g - f0, j]
                    comp["sel_box"][f] = comp["boxes"][g - f0, j]
                    kph[f] = comp["det_kp"][g - f0, j]
                else:  # a detection of the preceding chunk's last frames (any rank)
                    rec, kps, krow = prev_tail[g]
                    j = int(krow[slot])
                    r = np.asarray(rec[j].reshape(-1).cpu().numpy() if torch.is_tensor(rec) else rec[j]).reshape(-1)
                    comp["sel_logits"][f] = r[:M2].reshape(comp["sel_logits"].shape[1:])
                    comp["sel_box"][f] = r[M2:M2 + 4]
                    kph[f] = kps[j]
            raw = raw_reader(fr)
            raw = raw if torch.is_tensor(raw) else torch.from_numpy(np.ascontiguousarray(raw))
            raw = raw.to(comp["device"])
            prepped, cleaned = self.front_chunk(raw)
            d2 = self._paste_selected(comp, fr, prepped.shape[1:])
            feats = proc.frame_moments(cleaned, d2, float(self.cfg.frame_threshold))
            idx = np.asarray(fr)
            for k in ("centroid", "orientation", "axis_length"):
                host[k][idx] = feats[k].cpu().numpy()
        for k in ("logits", "boxes", "det_kp"):  # only the selected records travel to the second pass
            comp.pop(k, None)

    def _paste_selected(self, comp, frames, hw) -> torch.Tensor:
        """d2 masks (k, h, w) of `frames` (chunk indices) from their selected
        records: mdx_paste_masks with one detection per frame, the model's
        mask threshold -- the kernel and inputs of the forward's own paste."""
        dev = comp["device"]
        fr = np.asarray(frames, dtype=np.int64)
        k = len(fr)
        h, w = int(hw[0]), int(hw[1])
        d2 = torch.empty((k, h, w), dtype=torch.uint8, device=dev)
        if k == 0:
            return d2
        M = comp["sel_logits"].shape[1]
        lg = torch.from_numpy(np.ascontiguousarray(comp["sel_logits"][fr], np.float32)).to(dev)
        bx = torch.from_numpy(np.ascontiguousarray(comp["sel_box"][fr], np.float32)).to(dev)
        has = torch.from_numpy(np.ascontiguousarray(comp["sel_has"][fr], np.int32)).to(dev)
        thr = float(self.predictor.model.cfg.mask_threshold)
        for a in range(0, k, 65535):  # grid.y = frames per launch
            b = min(k, a + 65535)
            call("mdx_paste_masks", _p(lg[a:b]), _p(bx[a:b]), _p(has[a:b]), b - a, 1, M, h, w, h * w, thr,
                 _p(d2[a:b]), _stream())
        return d2

    def finish_chunk_compact(self, comp, raw, centroid, keypoints, angles, flips, axis_length, frame_idxs=None,
                             offset: int = 0, true_depth: float = 673.1) -> dict:
        """Second pass of a compact chunk: the chunk's front (prep + inpaint +
        clean) re-run from its raw frames -- deterministic, so equal to the
        first pass's -- the d2 masks re-pasted from the selected records, then
        finish_chunk."""
        raw = raw if isinstance(raw, torch.Tensor) and raw.is_cuda else \
            torch.from_numpy(np.ascontiguousarray(raw)).to(comp["device"])
        prepped, cleaned = self.front_chunk(raw)
        if "sel_logits" not in comp:
            self._sel_default(comp)
        d2 = self._paste_selected(comp, np.arange(len(comp["nkeep"])), prepped.shape[1:])
        state = {"prepped": prepped, "d2": d2, "cleaned": cleaned, "nkeep": comp["nkeep"]}
        return self.finish_chunk(state, centroid, keypoints, angles, flips, axis_length, frame_idxs, offset,
                                 true_depth)

    def _check_inpaint(self) -> None:
        """Once per chunk: frames whose inpaint cluster labelling did not
        converge are left un-inpainted by k_inp_setup and counted on the
        device in this extractor's own counter (mdx_inpaint_ns_counted);
        such frames would differ from the reference's, so a new count is
        raised here rather than written.  Another extractor of the same
        process does not touch the count."""
        n = self.prep.inpaint_errors()
        if n > self._inpaint_errors_seen:
            self._inpaint_errors_seen = n
            raise proc.MdxError(f"inpaint: {n} frame(s) whose invalid-pixel labelling did not converge "
                                "(mdx_inpaint_errors); their prepped frames would differ from the reference's")

    def host_angles(self, host: dict):
        """The sequential host step of instances_to_features
        (M/proc/proc.py:720-839): the tracking branch (Kalman smoothing +
        tracker-assisted flips; tracker state carried to the next chunk) or
        keypoint flips + iterative 180-degree filtering.  Returns (centroid,
        keypoints, angles deg, flips)."""
        if self.cfg.use_tracking:
            return TR.track_features(self.point_tracker, self.angle_tracker, host["centroid"], host["keypoints"],
                                     host["orientation"], host["axis_length"])
        angles, flips = F.finalize_angles(host["orientation"], host["axis_length"], host["centroid"],
                                          host["keypoints"])
        return host["centroid"], host["keypoints"], angles, flips

    def process_chunk(self, raw, frame_idxs=None, offset: int = 0, true_depth: float = 673.1) -> dict:
        """One chunk through ProduceFramesStep -> InferenceStep ->
        ProcessFeaturesStep, returning the data dict the reference's writer
        consumes (M/pipeline/produce_frames_step.py:33-38, inference_step.py:71,
        process_features_step.py:163-199; M/io/result.py:106-130).

        Device: prep/inpaint, model + mask NMS + instance 0, clean, moments,
        scalar reductions + keypoint z, crops.  Host (as in the reference, and
        sequential over frames and chunks): the angle / tracking step
        (host_angles), scalar and keypoint tables."""
        state, host = self.features_pass(raw)
        self.select_instances(state, host)
        cen, kp, angles, flips = self.host_angles(host)
        return self.finish_chunk(state, cen, kp, angles, flips, host["axis_length"], frame_idxs, offset, true_depth)

    def back(self, prepped: torch.Tensor, cleaned: torch.Tensor):
        """Model-dependent tail: forward + selection, moments, angle, crops."""
        return self.tail(prepped, cleaned, self.infer(prepped))


class _StreamSet:
    """The HIP streams of one OverlappedExtractor (front, model_streams model
    streams, tail).  The native model keeps a workspace per stream
    (mdx_model_reserve), so the extract loop of each session borrows a set
    from its predictor's pool (_checkout_streams) instead of making new
    streams: the workspaces, the allocator's per-stream pools and the priming
    forward are paid once per predictor, not once per session."""

    def __init__(self, model_streams: int):
        self.device = torch.cuda.current_device()
        self.front = torch.cuda.Stream()
        self.models = [torch.cuda.Stream() for _ in range(model_streams)]
        self.tail = torch.cuda.Stream()
        self.primed = False


_STREAM_POOLS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()  # predictor -> free _StreamSets
_STREAM_POOL_LOCK = threading.Lock()


def _checkout_streams(predictor, model_streams: int) -> _StreamSet:
    """A free stream set of `predictor` for `model_streams` model streams on
    the current device (a new one when every matching set is in use, e.g. by
    a session extracting in another thread)."""
    dev = torch.cuda.current_device()
    with _STREAM_POOL_LOCK:
        free = _STREAM_POOLS.setdefault(predictor, [])
        for i, sset in enumerate(free):
            if sset.device == dev and len(sset.models) == model_streams:
                return free.pop(i)
    return _StreamSet(model_streams)


def _checkin_streams(predictor, sset: _StreamSet) -> None:
    with _STREAM_POOL_LOCK:
        _STREAM_POOLS.setdefault(predictor, []).append(sset)


class OverlappedExtractor:
    """Software pipeline over consecutive batches on separate HIP streams:
    front (prep + inpaint + clean) of batch i+2, model forward + mask
    selection of batch i+1 and tail (moments, angle, crops) of batch i run
    concurrently, so the frame-side kernels (few, latency-bound workgroups)
    fill the CUs the convolutions leave idle.  With model_streams=2 the
    forwards of consecutive batches alternate between two streams and
    overlap each other too (the RPN / NMS / post-processing kernels and the
    small late layers of one forward leave most CUs idle).  Results come out
    in submission order, model_streams + 1 batches behind.

    submit(raw) -> results of the batch submitted model_streams + 1 calls
    earlier (or None);
    flush() -> list of the results still in flight."""

    def __init__(self, extractor: GPUExtractor, model_streams: int = 2, keep: bool = False,
                 streams: Optional["_StreamSet"] = None):
        self.ex = extractor
        self.keep = keep  # results also carry the batch's prepped / cleaned frames and forward outputs
        self.streams = streams
        sset = streams or _StreamSet(max(1, model_streams))
        self.s_front, self.s_models, self.s_tail = sset.front, sset.models, sset.tail
        self.n_model = 0
        self.fronted = None            # (prepped, cleaned, event) awaiting the model
        self.modeled = collections.deque()  # (prepped, cleaned, inf, event) awaiting the tail

    def _front(self, raw, raw_ready):
        caller = torch.cuda.current_stream()
        # raw was produced on the caller's stream before this submit; wait for
        # exactly that, not for the tail hand-offs queued on it since
        self.s_front.wait_event(raw_ready)
        with torch.cuda.stream(self.s_front):
            prepped, cleaned = self.ex.front(raw)
            ev = torch.cuda.Event()
            ev.record(self.s_front)
        raw.record_stream(self.s_front)
        return prepped, cleaned, ev

    def _model(self, item):
        prepped, cleaned, ev = item
        sm = self.s_models[self.n_model % len(self.s_models)]
        self.n_model += 1
        sm.wait_event(ev)
        with torch.cuda.stream(sm):
            prepped.record_stream(sm)
            inf = self.ex.infer(prepped)
            ev2 = torch.cuda.Event()
            ev2.record(sm)
        return prepped, cleaned, inf, ev2

    def _tail(self, item):
        prepped, cleaned, inf, ev = item
        caller = torch.cuda.current_stream()
        self.s_tail.wait_event(ev)
        with torch.cuda.stream(self.s_tail):
            for t in (prepped, cleaned, *[v for v in inf.values() if torch.is_tensor(v)]):
                t.record_stream(self.s_tail)
            out = self.ex.tail(prepped, cleaned, inf)
            ready = torch.cuda.Event()
            ready.record(self.s_tail)
        for v in out.values():
            v.record_stream(caller)
        if self.keep:
            for t in (prepped, cleaned, *[v for v in inf.values() if torch.is_tensor(v)], *inf["masks"]):
                t.record_stream(caller)
            out["prepped"], out["cleaned"], out["inf"] = prepped, cleaned, inf
        # the caller's stream does NOT wait here: a wait queued on it would
        # hold back every later front (and through it the next forwards)
        # until this batch's tail is done; consumers wait on out["ready"]
        # (OverlappedExtractor.wait) or call flush()
        out["ready"] = ready
        return out

    @staticmethod
    def wait(out, stream=None):
        """Make `stream` (default: current) wait until a submit() result is
        complete."""
        (stream or torch.cuda.current_stream()).wait_event(out["ready"])
        return out

    def prime(self, raw: torch.Tensor):
        """One batch through each stage on that stage's stream, one stream at
        a time, synchronised: kernel code objects are loaded, each model
        stream's workspace is reserved (mdx_model_reserve on first use) and
        the allocator's per-stream pools are populated before any two stages
        run concurrently.  Only the model streams run a forward, so only they
        get a model workspace."""
        cur = torch.cuda.current_stream()
        for st in (self.s_front, *self.s_models, self.s_tail):
            st.wait_stream(cur)
        with torch.cuda.stream(self.s_front):
            raw.record_stream(self.s_front)
            prepped, cleaned = self.ex.front(raw)
        torch.cuda.synchronize()
        inf = None
        for st in self.s_models:
            with torch.cuda.stream(st):
                prepped.record_stream(st)
                inf = self.ex.infer(prepped)
            torch.cuda.synchronize()
        with torch.cuda.stream(self.s_tail):
            for t in (prepped, cleaned, *[v for v in inf.values() if torch.is_tensor(v)]):
                t.record_stream(self.s_tail)
            self.ex.tail(prepped, cleaned, inf)
        torch.cuda.synchronize()

    def submit(self, raw: torch.Tensor):
        # issue order: tail of the oldest modeled batch (once `depth` forwards
        # are in flight), forward of the fronted batch, front of `raw`; every
        # stage's inputs were issued on an earlier call, so the stages (and up
        # to `depth` forwards) run concurrently on the device
        raw_ready = torch.cuda.Event()
        raw_ready.record(torch.cuda.current_stream())
        out = None
        if len(self.modeled) >= len(self.s_models):
            out = self._tail(self.modeled.popleft())
        if self.fronted is not None:
            self.modeled.append(self._model(self.fronted))
        self.fronted = self._front(raw, raw_ready)
        return out

    def flush(self):
        outs = []
        if self.fronted is not None:
            if len(self.modeled) >= len(self.s_models):
                outs.append(self._tail(self.modeled.popleft()))
            self.modeled.append(self._model(self.fronted))
            self.fronted = None
        while self.modeled:
            outs.append(self._tail(self.modeled.popleft()))
        torch.cuda.current_stream().wait_stream(self.s_tail)  # every result so far is complete
        return outs
