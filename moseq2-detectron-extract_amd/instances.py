"""Instance selection across frames:
ProcessFeaturesStep.__select_instances, M/pipeline/process_features_step.py:133-160,
with its norfair instance tracker (`Tracker(distance_function='euclidean',
distance_threshold=50, initialization_delay=0, hit_counter_max=3)`,
process_features_step.py:35-38) and the detections of
`__instances_to_detections` (:116-130).

norfair is unvendored and unpinned (setup.py:36) and absent from every
interpreter here; the string distance name and `hit_counter_max` exist only in
norfair >= 2.0, so this restates the published 2.x algorithm:

* `Tracker.update`: drop objects whose hit counter went negative, step every
  remaining object (hit counter -1, point hit counter -1, age +1, filter
  predict), match them to the detections greedily by the smallest euclidean
  distance below the threshold (float32 distance matrix, detection-major
  argmin), `hit()` the matched objects, start an object per unmatched
  detection, return the objects that are initialised with a hit counter >= 0;
* `TrackedObject.hit`: hit counter +2 capped at `hit_counter_max`, point hit
  counter +2 clamped to [0, pointwise_hit_counter_max=4];
* the default `OptimizedKalmanFilterFactory(R=4, Q=0.1, pos_variance=10,
  pos_vel_covariance=0, vel_variance=1)`: constant-velocity state per
  coordinate, `predict` moves the position only, `update` applies the
  prediction of the covariance and the Kalman gain together.  All
  coordinates of a 1-point detection share the same covariance, so it is kept
  as three scalars.

`InstanceTracker` is the product: the native host tracker in libmdx
(csrc/host_instances.hip, one call per chunk, no GIL).  `InstanceTrackerPy`
below states the same algorithm frame by frame in Python (the two are
checked against each other and against oracle/norfair_ref.py).

`select` then does what __select_instances does with the tracked objects: if
more than one is active, keep those with a live point, sort by age (stable)
and take up to `expected_instances` from the oldest end, each object's LAST
detection -- which can be a detection of an earlier frame (the reference's
behaviour, kept).  Parity is unpinned against norfair itself; it is checked
against `oracle/norfair_ref.py` (an object-level restatement) in
tests/test_instances.py.
"""
from __future__ import annotations

import math
import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

DIST_THRESHOLD = 50.0
HIT_COUNTER_MAX = 3
POINTWISE_HIT_COUNTER_MAX = 4
INITIALIZATION_DELAY = 0
_F32 = struct.Struct("f")
KF_R, KF_Q, KF_POS_VAR, KF_POS_VEL_COV, KF_VEL_VAR = 4.0, 0.1, 10.0, 0.0, 1.0


class _Object:
    """One norfair TrackedObject with a 1-point (2-D) detection."""
    __slots__ = ("pos", "vel", "p", "pv", "vv", "hit_counter", "point_hit", "age", "last")

    def __init__(self, point, det_id):
        self.pos = [float(point[0]), float(point[1])]
        self.vel = [0.0, 0.0]
        self.p, self.pv, self.vv = KF_POS_VAR, KF_POS_VEL_COV, KF_VEL_VAR
        self.hit_counter = 1          # = period
        self.point_hit = 1            # detected_at_least_once (scores None)
        self.age = 0
        self.last = det_id

    def step(self):
        self.hit_counter -= 1
        self.point_hit -= 1
        self.age += 1
        self.pos[0] += self.vel[0]
        self.pos[1] += self.vel[1]

    def hit(self, point, det_id):
        self.last = det_id
        self.hit_counter = min(self.hit_counter + 2, HIT_COUNTER_MAX)
        self.point_hit = min(max(self.point_hit + 2, 0), POINTWISE_HIT_COUNTER_MAX)
        # OptimizedKalmanFilter.update with H = [I 0] (every sensor matched)
        vpp = self.pv + self.vv
        added = self.p + self.pv + vpp + KF_Q + KF_R
        r_over = KF_R / added
        v_over = vpp / added
        for c in range(2):
            err = float(point[c]) - self.pos[c]
            self.pos[c] += (1.0 - r_over) * err
            self.vel[c] += v_over * err
        self.p = (1.0 - r_over) * KF_R
        self.pv = v_over * KF_R
        self.vv += KF_Q - (v_over * v_over) * added


class InstanceTrackerPy:
    """norfair Tracker as configured by ProcessFeaturesStep (one per session;
    state carried from chunk to chunk), frame by frame in Python."""

    def __init__(self, expected_instances: int = 1):
        self.expected_instances = int(expected_instances)
        self.objects: List[_Object] = []

    def update(self, points: Sequence[Tuple[float, float]], det_ids: Sequence) -> List[_Object]:
        objs = [o for o in self.objects if o.hit_counter >= 0]
        self.objects = objs
        for o in objs:
            o.step()
        nd, no = len(points), len(objs)
        unmatched = range(nd)
        if nd and no:
            # float32 distance matrix; greedy matching = repeated argmin with
            # detection-major tie-breaking, i.e. ascending (distance, det, obj)
            cand = []
            for i in range(nd):
                py, px = float(points[i][0]), float(points[i][1])
                for j, o in enumerate(objs):
                    dy, dx = py - o.pos[0], px - o.pos[1]
                    d = _F32.unpack(_F32.pack(math.sqrt(dy * dy + dx * dx)))[0]
                    if d != d:
                        raise ValueError("Received nan values from distance function")
                    cand.append((d, i, j))
            cand.sort()
            used_i, used_j = set(), set()
            for d, i, j in cand:
                if d >= DIST_THRESHOLD:
                    break
                if i in used_i or j in used_j:
                    continue
                used_i.add(i)
                used_j.add(j)
                objs[j].hit(points[i], det_ids[i])
            if used_i:
                unmatched = [i for i in range(nd) if i not in used_i]
        for i in unmatched:
            self.objects.append(_Object(points[i], det_ids[i]))
        return [o for o in self.objects if o.hit_counter >= 0]

    def select(self, points, det_ids) -> Optional[List]:
        """One frame of __select_instances after mask NMS.  Returns None when
        the frame's instances stay as they are (<= 1 tracked object), else the
        detection ids of the picked instances (possibly empty)."""
        active = self.update(points, det_ids)
        if len(active) <= 1:
            return None
        live = sorted((o for o in active if o.point_hit > 0), key=lambda o: o.age)
        out = []
        while len(out) < self.expected_instances and live:
            out.append(live.pop().last)
        return out


    def select_chunk(self, nkeep: np.ndarray, centers: np.ndarray, frame0: int):
        """See select_chunk."""
        changes = {}
        nk = np.asarray(nkeep).tolist()
        cen = np.asarray(centers, dtype=np.float64).tolist()
        for f in range(len(nk)):
            k = nk[f]
            g = frame0 + f
            sel = self.select(cen[f][:k], [(g, s) for s in range(k)])
            if sel is not None:
                if len(sel) == k and all(d == (g, s) for s, d in enumerate(sel)):
                    continue  # same instances, same order
                changes[f] = sel
        return changes


class InstanceTracker:
    """The session's instance tracker: the native host implementation
    (mdx_instance_tracker_*), state held behind a handle."""

    def __init__(self, expected_instances: int = 1):
        from ._lib import MdxError, lib
        self.expected_instances = int(expected_instances)
        self._lib = lib()
        self._h = self._lib.mdx_instance_tracker_create(self.expected_instances)
        if not self._h:
            raise MdxError("mdx_instance_tracker_create failed (expected_instances >= 1)")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.mdx_instance_tracker_destroy(h)

    def select_chunk(self, nkeep: np.ndarray, centers: np.ndarray, frame0: int):
        """See select_chunk."""
        import ctypes
        from ._lib import call
        nk = np.ascontiguousarray(nkeep, dtype=np.int32)
        n = len(nk)
        cen = np.ascontiguousarray(centers, dtype=np.float64)
        D = cen.shape[1] if n else 1
        out_n = np.empty(n, np.int32)
        ids = np.empty((n, self.expected_instances, 2), np.int64)
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        call("mdx_instance_tracker_select", ctypes.c_void_p(self._h), vp(nk), vp(cen), n, D, int(frame0), vp(out_n),
             vp(ids))
        return {f: [(int(ids[f, m, 0]), int(ids[f, m, 1])) for m in range(out_n[f])]
                for f in np.nonzero(out_n >= 0)[0].tolist()}


def select_chunk(tracker, nkeep: np.ndarray, centers: np.ndarray, frame0: int):
    """Run the tracker over a chunk's frames.  nkeep (n,), centers (n,D,2)
    float64 (kept detections in pick order).  A detection id is (session frame,
    kept slot).  Returns {chunk frame: list of picked detection ids} for the
    frames whose instances change."""
    return tracker.select_chunk(nkeep, centers, frame0)
