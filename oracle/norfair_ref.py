"""Object-level restatement of the reference's instance selection (TEST
INFRASTRUCTURE ONLY -- the checker of moseq2_detectron_extract_amd.instances).

ProcessFeaturesStep (M/pipeline/process_features_step.py:35-38 tracker setup,
:116-130 detections, :133-160 selection) drives ``norfair.Tracker``.  norfair
is unvendored, unpinned (setup.py:36) and absent from every interpreter in this
image, so PARITY IS UNPINNED against it: no fixture of the reference covers
this step.  This file restates norfair 2.x as published (``tracker.py``
Tracker.update / _update_objects_in_place / match_dets_and_objs,
TrackedObject.__init__ / tracker_step / hit / live_points, ``filter.py``
OptimizedKalmanFilter, ``distances.py`` ScipyDistance('euclidean') with its
float32 matrix) with the library's own array shapes -- (dim_z, 1) state
columns, an H matrix per hit -- so it shares no code path with the product's
scalar version.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.distance import cdist


class Detection:
    def __init__(self, points, data=None):
        points = np.asarray(points, dtype=np.float64)
        if points.shape == (2,):
            points = points[np.newaxis, :]
        self.points = points
        self.absolute_points = points.copy()
        self.scores = None
        self.data = data
        self.label = None


class OptimizedKalmanFilter:
    def __init__(self, initial, R=4.0, Q=0.1, pos_variance=10, pos_vel_covariance=0, vel_variance=1):
        self.dim_z = initial.size
        self.x = np.zeros((2 * self.dim_z, 1))
        self.x[: self.dim_z] = np.expand_dims(initial.flatten(), 0).T
        self.pos_variance = np.zeros((self.dim_z, 1)) + pos_variance
        self.pos_vel_covariance = np.zeros((self.dim_z, 1)) + pos_vel_covariance
        self.vel_variance = np.zeros((self.dim_z, 1)) + vel_variance
        self.q_Q = Q
        self.default_r = R * np.ones((self.dim_z, 1))

    def predict(self):
        self.x[: self.dim_z] += self.x[self.dim_z:]

    def update(self, z, R=None, H=None):
        diagonal = np.diagonal(H).reshape((self.dim_z, 1))
        one_minus_diagonal = 1 - diagonal
        kalman_r = self.default_r
        error = np.multiply(z - self.x[: self.dim_z], diagonal)
        vel_var_plus_pos_vel_cov = self.pos_vel_covariance + self.vel_variance
        added_variances = (self.pos_variance + self.pos_vel_covariance + vel_var_plus_pos_vel_cov + self.q_Q
                           + kalman_r)
        kalman_r_over_added_variances = np.divide(kalman_r, added_variances)
        vel_var_plus_pos_vel_cov_over_added_variances = np.divide(vel_var_plus_pos_vel_cov, added_variances)
        added_variances_or_kalman_r = np.multiply(added_variances, one_minus_diagonal) + np.multiply(kalman_r, diagonal)
        self.x[: self.dim_z] += np.multiply(diagonal, np.multiply(1 - kalman_r_over_added_variances, error))
        self.x[self.dim_z:] += np.multiply(diagonal, np.multiply(vel_var_plus_pos_vel_cov_over_added_variances, error))
        self.pos_variance = np.multiply(1 - kalman_r_over_added_variances, added_variances_or_kalman_r)
        self.pos_vel_covariance = np.multiply(vel_var_plus_pos_vel_cov_over_added_variances,
                                              added_variances_or_kalman_r)
        self.vel_variance += self.q_Q - np.multiply(
            diagonal, np.multiply(np.square(vel_var_plus_pos_vel_cov_over_added_variances), added_variances))


class TrackedObject:
    def __init__(self, det, hit_counter_max, initialization_delay, pointwise_hit_counter_max, period=1):
        self.num_points, self.dim_points = det.absolute_points.shape
        self.hit_counter_max = hit_counter_max
        self.pointwise_hit_counter_max = max(pointwise_hit_counter_max, period)
        self.initialization_delay = initialization_delay
        self.hit_counter = period
        self.last_detection = det
        self.age = 0
        self.is_initializing = self.hit_counter <= self.initialization_delay
        self.detected_at_least_once_points = np.array([True] * self.num_points)
        self.point_hit_counter = self.detected_at_least_once_points.astype(int)
        self.filter = OptimizedKalmanFilter(det.absolute_points)
        self.dim_z = self.dim_points * self.num_points

    def tracker_step(self):
        self.hit_counter -= 1
        self.point_hit_counter -= 1
        self.age += 1
        self.filter.predict()

    @property
    def estimate(self):
        return self.filter.x.T.flatten()[: self.dim_z].reshape(-1, self.dim_points)

    @property
    def live_points(self):
        return self.point_hit_counter > 0

    def hit(self, det, period=1):
        points = det.absolute_points
        self.last_detection = det
        self.hit_counter = min(self.hit_counter + 2 * period, self.hit_counter_max)
        if self.is_initializing and self.hit_counter > self.initialization_delay:
            self.is_initializing = False
        H_pos = np.identity(self.num_points * self.dim_points)
        self.point_hit_counter += 2 * period
        self.point_hit_counter[self.point_hit_counter >= self.pointwise_hit_counter_max] = \
            self.pointwise_hit_counter_max
        self.point_hit_counter[self.point_hit_counter < 0] = 0
        H = np.hstack([H_pos, np.zeros(H_pos.shape)])
        self.filter.update(np.expand_dims(points.flatten(), 0).T, None, H)


class Tracker:
    def __init__(self, distance_threshold=50, hit_counter_max=3, initialization_delay=0,
                 pointwise_hit_counter_max=4):
        self.distance_threshold = distance_threshold
        self.hit_counter_max = hit_counter_max
        self.initialization_delay = initialization_delay
        self.pointwise_hit_counter_max = pointwise_hit_counter_max
        self.tracked_objects = []

    @staticmethod
    def _distances(objects, candidates):
        dm = np.full((len(candidates), len(objects)), fill_value=np.inf, dtype=np.float32)
        if not objects or not candidates:
            return dm
        so = np.stack([o.estimate.ravel() for o in objects])
        sc = np.stack([c.points.ravel() for c in candidates])
        dm[:, :] = cdist(sc, so, metric="euclidean")
        return dm

    def _match(self, dm):
        dm = dm.copy()
        if dm.size > 0:
            det_idxs, obj_idxs = [], []
            current_min = dm.min()
            while current_min < self.distance_threshold:
                flat = dm.argmin()
                det_idx, obj_idx = flat // dm.shape[1], flat % dm.shape[1]
                det_idxs.append(det_idx)
                obj_idxs.append(obj_idx)
                dm[det_idx, :] = self.distance_threshold + 1
                dm[:, obj_idx] = self.distance_threshold + 1
                current_min = dm.min()
            return det_idxs, obj_idxs
        return [], []

    def _update_in_place(self, objects, candidates):
        if candidates is not None and len(candidates) > 0:
            dm = self._distances(objects, candidates)
            if np.isnan(dm).any():
                raise ValueError("nan distance")
            cand_idx, obj_idx = self._match(dm)
            if len(cand_idx) > 0:
                unmatched = [d for i, d in enumerate(candidates) if i not in cand_idx]
                for ci, oi in zip(cand_idx, obj_idx):
                    if dm[ci, oi] < self.distance_threshold:
                        objects[oi].hit(candidates[ci])
                    else:
                        unmatched.append(candidates[ci])
                return unmatched
            return candidates
        return []

    def update(self, detections):
        self.tracked_objects = [o for o in self.tracked_objects if o.hit_counter >= 0]
        alive = self.tracked_objects
        for o in self.tracked_objects:
            o.tracker_step()
        unmatched = self._update_in_place([o for o in alive if not o.is_initializing], detections)
        unmatched = self._update_in_place([o for o in alive if o.is_initializing], unmatched)
        for d in unmatched:
            self.tracked_objects.append(TrackedObject(d, self.hit_counter_max, self.initialization_delay,
                                                      self.pointwise_hit_counter_max))
        return [o for o in self.tracked_objects if not o.is_initializing and o.hit_counter >= 0]


def center_of_mass(mask):
    """scipy.ndimage.center_of_mass of a 2-D 0/1 mask (row, col)."""
    m = np.asarray(mask).astype(np.float64)
    norm = m.sum()
    ys, xs = np.ogrid[: m.shape[0], : m.shape[1]]
    return np.array([(m * ys).sum() / norm, (m * xs).sum() / norm])


def select_instances(frames, expected_instances=1):
    """__select_instances over a session.  frames: list of lists of
    (detection id, centre (2,)) in pick order.  Returns per frame the picked
    detection ids (the frame's own ids when it stays unchanged)."""
    tracker = Tracker()
    out = []
    for dets in frames:
        tracked = tracker.update([Detection(c, data={"id": i}) for i, c in dets])
        if len(tracked) <= 1:
            out.append([i for i, _ in dets])
            continue
        live = sorted(filter(lambda to: to.live_points.any(), tracked), key=lambda item: item.age)
        sel = []
        while len(sel) < expected_instances and len(live) > 0:
            sel.append(live.pop().last_detection.data["id"])
        out.append(sel)
    return out
