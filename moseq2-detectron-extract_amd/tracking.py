"""Tracking branch of the feature step (``--use-tracking``, the reference's
default, M/cli.py:366): Kalman smoothing of centroid + keypoints and
Kalman-assisted 180-degree flip correction of the angles.

=================================  ==========================================
this module                        reference (M/ = moseq2_detectron_extract/)
=================================  ==========================================
timestamps_to_steps                M/proc/kalman.py:10-20
expand_missing_entries             M/proc/kalman.py:23-58
reduce_missing_entries             M/proc/kalman.py:61-90
KalmanTrackerPoint1D / Point2D /   M/proc/kalman.py:101-278
KalmanTrackerAngle / NPoints2D
KalmanTracker                      M/proc/kalman.py:281-418
KalmanFilter                       pykalman.KalmanFilter (unpinned, absent
                                   here) as the reference calls it:
                                   em(n_iter=10) on transition_covariance,
                                   observation_covariance,
                                   initial_state_covariance; smooth;
                                   filter_update; sample(1, state)
make_trackers                      ProcessFeaturesStep.__init__
                                   M/pipeline/process_features_step.py:40-51
track_features                     instances_to_features tracking branch
                                   M/proc/proc.py:730-820
=================================  ==========================================

Host code, as in the reference: the recursions are sequential over frames
(and over chunks -- the trackers carry state from chunk to chunk), so with
frame sharding they run once, on rank 0, between the device feature pass and
the device crop pass (extract.py).  The filter exploits that every
observation matrix here is a 0/1 selection of state components:
``C P C^T`` is a gather and ``K C P`` a row gather, which pykalman computes as
dense products with identical results; EM's sums over time are batched.
``sample(1, state)`` returns the state itself (pykalman draws observation
noise from the global RNG there, which never reaches the returned states).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import numpy.ma as ma
from scipy.linalg import block_diag

from . import features as F
from ._lib import call


# ---------------------------------------------------------------------------
# missing-frame helpers (kalman.py:10-90)
# ---------------------------------------------------------------------------
def timestamps_to_steps(timestamps, step_size=(1 / 30 * 1000)):
    """Discrete steps between consecutive observations."""
    return np.rint(np.diff(timestamps) / step_size).astype(int)


def expand_missing_entries(data, time_steps):
    """Insert masked rows where `time_steps` skips frames."""
    time_steps = np.asarray(time_steps)
    out_shape = (int(np.sum(time_steps)) + 1, *data.shape[1:])
    full = np.zeros(out_shape, dtype=data.dtype)
    mask = np.zeros(out_shape, dtype="int")
    if len(time_steps) == 0:  # the reference's loop then stores data[1] (kalman.py:57)
        full[0] = data[1]
        return ma.masked_array(full, mask=mask)
    pos = np.concatenate(([0], np.cumsum(time_steps)))
    full[pos] = data[:len(pos)]
    for p, k in zip(pos[:-1], time_steps):
        if k != 1:
            mask[p + 1:p + k] = 1
    return ma.masked_array(full, mask=mask)


def reduce_missing_entries(data, time_steps):
    """Inverse of expand_missing_entries."""
    pos = np.concatenate(([0], np.cumsum(np.asarray(time_steps))))
    return np.asarray(data)[pos].copy()


# ---------------------------------------------------------------------------
# Kalman filter (pykalman semantics)
# ---------------------------------------------------------------------------
class KalmanFilter:
    """Linear-Gaussian state space model with fixed transition matrix A and
    observation matrix C, zero offsets, and Q, R, P0 identity until `em`
    learns them (the reference's em_vars)."""

    def __init__(self, transition_matrices, observation_matrices, initial_state_mean,
                 em_vars=("transition_covariance", "observation_covariance", "initial_state_covariance")):
        self.A = np.ascontiguousarray(transition_matrices, dtype=np.float64)
        C = np.atleast_2d(np.asarray(observation_matrices, dtype=np.float64))
        self.C = C
        ns, no = self.A.shape[0], C.shape[0]
        self.initial_state_mean = np.asarray(initial_state_mean, dtype=np.float64)
        self.transition_covariance = np.eye(ns)
        self.observation_covariance = np.eye(no)
        self.initial_state_covariance = np.eye(ns)
        self.em_vars = tuple(em_vars)
        # every tracker item observes one state component per observation row
        rows = [np.flatnonzero(r) for r in C]
        self._sel = None
        if all(len(r) == 1 for r in rows) and np.all(C[np.arange(no), [r[0] for r in rows]] == 1) \
                and np.count_nonzero(C) == no:
            self._sel = np.array([r[0] for r in rows])

    # -- one step --------------------------------------------------------
    def _predict(self, x, P):
        A = self.A
        return A @ x, A @ (P @ A.T) + self.transition_covariance

    def _correct(self, xp, Pp, z, zmask):
        if zmask:
            return xp, Pp
        R = self.observation_covariance
        if self._sel is not None:
            s = self._sel
            PCt = Pp[:, s]
            S = PCt[s] + R
            K = PCt @ np.linalg.inv(S)
            return xp + K @ (z - xp[s]), Pp - K @ Pp[s]
        C = self.C
        S = C @ (Pp @ C.T) + R
        K = Pp @ (C.T @ np.linalg.inv(S))
        return xp + K @ (z - C @ xp), Pp - K @ (C @ Pp)

    # -- whole sequences -------------------------------------------------
    @staticmethod
    def _parse(X):
        X = ma.asarray(X)
        if X.ndim == 1:
            X = X[:, None]
        data = np.asarray(ma.getdata(X), dtype=np.float64)
        rowmask = ma.getmaskarray(X).any(axis=1)
        return data, rowmask

    def _filter(self, data, rowmask, x0, P0):
        T, ns = data.shape[0], self.A.shape[0]
        xp = np.empty((T, ns)); Pp = np.empty((T, ns, ns))
        xf = np.empty((T, ns)); Pf = np.empty((T, ns, ns))
        for t in range(T):
            if t == 0:
                xp[0], Pp[0] = x0, P0
            else:
                xp[t], Pp[t] = self._predict(xf[t - 1], Pf[t - 1])
            xf[t], Pf[t] = self._correct(xp[t], Pp[t], data[t], rowmask[t])
        return xp, Pp, xf, Pf

    def _smooth(self, xp, Pp, xf, Pf):
        T, ns = xf.shape
        At = self.A.T
        xs = np.empty((T, ns)); Ps = np.empty((T, ns, ns)); J = np.empty((max(T - 1, 0), ns, ns))
        xs[-1], Ps[-1] = xf[-1], Pf[-1]
        for t in range(T - 2, -1, -1):
            Jt = Pf[t] @ (At @ np.linalg.inv(Pp[t + 1]))
            J[t] = Jt
            xs[t] = xf[t] + Jt @ (xs[t + 1] - xp[t + 1])
            Ps[t] = Pf[t] + Jt @ ((Ps[t + 1] - Pp[t + 1]) @ Jt.T)
        return xs, Ps, J

    def filter(self, X):
        data, m = self._parse(X)
        _, _, xf, Pf = self._filter(data, m, self.initial_state_mean, self.initial_state_covariance)
        return xf, Pf

    def smooth(self, X):
        data, m = self._parse(X)
        xp, Pp, xf, Pf = self._filter(data, m, self.initial_state_mean, self.initial_state_covariance)
        xs, Ps, _ = self._smooth(xp, Pp, xf, Pf)
        return xs, Ps

    def em(self, X, n_iter: int = 10):
        data, m = self._parse(X)
        A, C = self.A, self.C
        T = data.shape[0]
        x0 = self.initial_state_mean
        obs = ~m
        for _ in range(n_iter):
            xp, Pp, xf, Pf = self._filter(data, m, x0, self.initial_state_covariance)
            xs, Ps, J = self._smooth(xp, Pp, xf, Pf)
            if "observation_covariance" in self.em_vars:
                n = int(obs.sum())
                if n > 0:
                    err = data[obs] - xs[obs] @ C.T
                    CPC = (C @ Ps[obs] @ C.T) if self._sel is None else Ps[obs][:, self._sel][:, :, self._sel]
                    self.observation_covariance = (err.T @ err + CPC.sum(axis=0)) / n
                else:
                    self.observation_covariance = np.zeros_like(self.observation_covariance)
            if "transition_covariance" in self.em_vars and T > 1:
                pair = Ps[1:] @ np.transpose(J, (0, 2, 1))           # _smooth_pair
                err = xs[1:] - xs[:-1] @ A.T
                V = pair @ A.T
                tot = err.T @ err + (A @ Ps[:-1] @ A.T).sum(axis=0) + Ps[1:].sum(axis=0) \
                    - V.sum(axis=0) - np.transpose(V, (0, 2, 1)).sum(axis=0)
                self.transition_covariance = (1.0 / (T - 1)) * tot
            if "initial_state_covariance" in self.em_vars:
                z = xs[0]
                self.initial_state_covariance = Ps[0] + np.outer(z, z) - np.outer(x0, z) - np.outer(z, x0) \
                    + np.outer(x0, x0)
        return self

    def filter_update(self, filtered_state_mean, filtered_state_covariance, observation=None):
        xp, Pp = self._predict(np.asarray(filtered_state_mean, dtype=np.float64), filtered_state_covariance)
        if observation is None:
            return xp, Pp
        z = ma.asarray(observation)
        return self._correct(xp, Pp, np.asarray(ma.getdata(z), dtype=np.float64), bool(ma.getmaskarray(z).any()))

    def sample(self, n_timesteps: int, initial_state):
        if n_timesteps != 1:
            raise ValueError("only the one-step sample of the reference (proc.py:773) is restated")
        return np.asarray(initial_state, dtype=np.float64)[None, :], None


# ---------------------------------------------------------------------------
# tracker items (kalman.py:101-278)
# ---------------------------------------------------------------------------
class KalmanTrackerItem:
    def __init__(self, order: int = 3, delta_t: float = 1.0):
        self.order = order
        self.delta_t = delta_t

    @property
    def state_size(self) -> int:
        return np.atleast_2d(self.build_observ_mat()).shape[-1]

    def format_data(self, data):
        return data

    def inverse_format_data(self, data):
        return data[:, ::self.order]


class KalmanTrackerPoint1D(KalmanTrackerItem):
    def _derivatives(self):
        return [1.0, self.delta_t, self.delta_t ** 2 / 2, self.delta_t ** 3 / 6][:self.order]

    def build_trans_mat(self):
        der = self._derivatives()
        A = np.zeros((self.order, self.order))
        for r in range(self.order):
            A[r, r:] = der[:self.order - r]
        return A

    def build_observ_mat(self):
        c = np.zeros((self.order,))
        c[0] = 1
        return c

    def build_init_state_means(self, data):
        x0 = np.zeros((self.order,))
        x0[0] = data[0] if data.shape[0] > 0 else 0
        return x0


class KalmanTrackerPoint2D(KalmanTrackerPoint1D):
    def build_trans_mat(self):
        a = super().build_trans_mat()
        return block_diag(a, a)

    def build_observ_mat(self):
        c = super().build_observ_mat()
        return block_diag(c, c)

    def build_init_state_means(self, data):
        return np.hstack((super().build_init_state_means(data[:, 0]), super().build_init_state_means(data[:, 1])))


class KalmanTrackerAngle(KalmanTrackerPoint2D):
    """Angles tracked as (sin, cos) on the unit circle."""

    def __init__(self, order: int = 3, delta_t: float = 1.0, degrees: bool = True):
        super().__init__(order=order, delta_t=delta_t)
        self.degrees = degrees

    def build_init_state_means(self, data):
        return super().build_init_state_means(self.format_data(data))

    def format_data(self, data):
        if self.degrees:
            data = np.deg2rad(data)
        return np.column_stack([np.sin(data), np.cos(data)])

    def inverse_format_data(self, data):
        yx = data[:, ::self.order]
        a = np.arctan2(yx[:, 0], yx[:, 1])
        a = np.where(a < 0, 2 * np.pi + a, a)
        return np.rad2deg(a) if self.degrees else a


class KalmanTrackerNPoints2D(KalmanTrackerPoint2D):
    def __init__(self, n_points: int, order: int = 3, delta_t: float = 1):
        self.n_points = n_points
        super().__init__(order, delta_t)

    def build_trans_mat(self):
        return block_diag(*[super(KalmanTrackerNPoints2D, self).build_trans_mat()] * self.n_points)

    def build_observ_mat(self):
        return block_diag(*[super(KalmanTrackerNPoints2D, self).build_observ_mat()] * self.n_points)

    def build_init_state_means(self, data):
        return np.hstack([super(KalmanTrackerNPoints2D, self).build_init_state_means(data[:, i, :])
                          for i in range(self.n_points)])

    def format_data(self, data):
        return data.reshape(data.shape[0], -1)

    def inverse_format_data(self, data):
        return data[:, ::self.order].reshape(data.shape[0], self.n_points, -1)


class KalmanTracker:
    """One Kalman filter over the concatenated states of several items."""

    def __init__(self, items_to_track: Sequence[KalmanTrackerItem]):
        if items_to_track is None or len(items_to_track) <= 0:
            raise ValueError("You need to supply a list of `KalmanTrackerItem`s to the constructor!")
        steps = [it.delta_t for it in items_to_track]
        if not np.allclose(steps, steps[0]):
            raise ValueError(f"Timesteps across `KalmanTrackerItem` must be the same! Got: {', '.join(map(str, steps))}")
        self.items = list(items_to_track)
        self.kalman_filter: Optional[KalmanFilter] = None
        self.last_mean = None
        self.last_covar = None

    @property
    def is_initialized(self) -> bool:
        return self.kalman_filter is not None

    def initialize(self, init_data: Sequence[np.ndarray]) -> None:
        if len(init_data) != len(self.items):
            raise ValueError(f"Length of `init_data` ({len(init_data)}) does not equal length of "
                             f"`items_to_track` ({len(self.items)})")
        self.kalman_filter = KalmanFilter(block_diag(*[it.build_trans_mat() for it in self.items]),
                                          block_diag(*[it.build_observ_mat() for it in self.items]),
                                          self._build_init_state_means(init_data))
        Z = self._format_data(init_data)
        finite = np.isfinite(ma.getdata(Z)).any(axis=1)
        if np.count_nonzero(finite) > 0:
            self.kalman_filter.em(Z[finite], n_iter=10)
        self.last_mean = self.kalman_filter.initial_state_mean
        self.last_covar = self.kalman_filter.initial_state_covariance

    def _build_init_state_means(self, init_data):
        return np.hstack([it.build_init_state_means(init_data[i]) for i, it in enumerate(self.items)])

    def _format_data(self, data):
        return ma.masked_invalid(np.column_stack([it.format_data(data[i]) for i, it in enumerate(self.items)]))

    def _inverse_format_data(self, data) -> List[np.ndarray]:
        data = ma.getdata(data)
        out, off = [], 0
        for it in self.items:
            out.append(it.inverse_format_data(data[:, off:off + it.state_size]))
            off += it.state_size
        return out

    def sample(self, n_timesteps: int = 1, init_data=None):
        init = self._build_init_state_means(init_data) if init_data is not None else self.last_mean
        states, _ = self.kalman_filter.sample(n_timesteps, init)
        return self._inverse_format_data(states)

    def smooth(self, data):
        means, _ = self.kalman_filter.smooth(self._format_data(data))
        return self._inverse_format_data(means)

    def smooth_update(self, data):
        Z = self._format_data(data)
        if Z.shape[0] == 1:
            return self.filter_update(data)
        means, covs = self.kalman_filter.smooth(Z)
        self.last_mean = self.kalman_filter.initial_state_mean = means[-1]
        self.last_covar = self.kalman_filter.initial_state_covariance = covs[-1]
        return self._inverse_format_data(means)

    def filter(self, data):
        means, _ = self.kalman_filter.filter(self._format_data(data))
        return self._inverse_format_data(means)

    def filter_update(self, data):
        z = self._format_data(data)[0]
        self.last_mean, self.last_covar = self.kalman_filter.filter_update(self.last_mean, self.last_covar, z)
        return self._inverse_format_data(self.last_mean[None, :])


# ---------------------------------------------------------------------------
# the tracking branch of instances_to_features
# ---------------------------------------------------------------------------
class NativeTracking:
    """The tracking branch's two trackers in libmdx host code
    (mdx_tracking_*): the same model as the numpy KalmanTracker pair below,
    without the per-step Python overhead.  ``point`` / ``angle`` expose the
    trackers' ``is_initialized`` / ``last_mean`` like KalmanTracker does."""

    class _View:
        def __init__(self, owner, which):
            self._o, self._w = owner, which

        def _state(self):
            import ctypes
            ini = ctypes.c_int()
            buf = np.empty(1024, np.float64)
            n = call("mdx_tracking_state", self._o._h, self._w, ctypes.byref(ini),
                     buf.ctypes.data_as(ctypes.c_void_p), buf.size)
            return bool(ini.value), buf[:n].copy()

        @property
        def is_initialized(self) -> bool:
            return self._state()[0]

        @property
        def last_mean(self) -> np.ndarray:
            return self._state()[1]

    def __init__(self, n_keypoints: int = 8):
        self.n_keypoints = n_keypoints
        self._h = call("mdx_tracking_create", int(n_keypoints))
        if not self._h:
            raise ValueError("mdx_tracking_create failed")
        self.point, self.angle = NativeTracking._View(self, 0), NativeTracking._View(self, 1)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                call("mdx_tracking_destroy", h)
            except Exception:
                pass
            self._h = None

    def track(self, centroid, keypoints, orientation, axis_length):
        import ctypes
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        cen = np.ascontiguousarray(centroid, np.float64)
        kp = np.ascontiguousarray(keypoints, np.float64)
        ori = np.ascontiguousarray(orientation, np.float64)
        ax = np.ascontiguousarray(axis_length, np.float64)
        n, K = kp.shape[0], kp.shape[1]
        c_out, k_out = np.empty_like(cen), np.empty_like(kp)
        a_out, f_out = np.empty(n, np.float64), np.empty(n, np.uint8)
        call("mdx_tracking_track", self._h, n, K, P(cen), P(kp), P(ori), P(ax), P(c_out), P(k_out), P(a_out),
             P(f_out))
        return c_out, k_out, a_out, f_out.astype(bool)


def make_trackers(n_keypoints: int = 8, native: bool = True):
    """(point_tracker, angle_tracker) as ProcessFeaturesStep builds them
    (process_features_step.py:40-51): by default views of one NativeTracking
    (libmdx host code); native=False gives the numpy KalmanTracker pair."""
    if native:
        t = NativeTracking(n_keypoints)
        return t.point, t.angle
    point = KalmanTracker([KalmanTrackerPoint2D(order=3, delta_t=1.0),
                           KalmanTrackerNPoints2D(n_keypoints, order=3, delta_t=1.0)])
    angle = KalmanTracker([KalmanTrackerAngle(order=3, delta_t=1.0, degrees=True)])
    return point, angle


def _angle_loop(angle_tracker: KalmanTracker, angles: np.ndarray, flips: np.ndarray, scores: np.ndarray):
    """proc.py:769-800 on the angle filter directly (6 states, 2 observations)."""
    kf = angle_tracker.kalman_filter
    A, Q, R = kf.A, kf.transition_covariance, kf.observation_covariance
    x, P = np.asarray(angle_tracker.last_mean, dtype=np.float64), angle_tracker.last_covar
    At = A.T
    s = kf._sel                                                        # (sin, cos) components
    for i in range(angles.shape[0]):
        p = np.arctan2(x[s[0]], x[s[1]])
        p = np.rad2deg(2 * np.pi + p if p < 0 else p)                 # sample(1) -> angle
        diff = (angles[i] - p) % 360
        if diff > 180:
            diff = -(360 - diff)
        if scores[i] < 0.4:
            angles[i] = p
        elif abs(diff) > 140:
            a = angles[i] + 180
            angles[i] = (360 + a if a < 0 else a) % 360
            flips[i] = ~flips[i]
        r = np.deg2rad(angles[i])
        z = np.array([np.sin(r), np.cos(r)])
        xp, Pp = A @ x, A @ (P @ At) + Q                               # filter_update
        if np.isfinite(z).all():
            PCt = Pp[:, s]
            K = PCt @ np.linalg.inv(PCt[s] + R)
            x, P = xp + K @ (z - xp[s]), Pp - K @ Pp[s]
        else:
            x, P = xp, Pp
    angle_tracker.last_mean, angle_tracker.last_covar = x, P
    return angles, flips


def track_features(point_tracker: KalmanTracker, angle_tracker: KalmanTracker, centroid: np.ndarray,
                   keypoints: np.ndarray, orientation: np.ndarray, axis_length: np.ndarray):
    """Tracking branch of instances_to_features (M/proc/proc.py:720-820) for
    one chunk.  centroid (n,2), keypoints (n,K,3) of instance 0,
    orientation (n,) radians, axis_length (n,2).  The trackers carry their
    state into the next chunk.  Returns (centroid, keypoints, angles deg,
    flips) with the keypoints' first 7 (x, y) replaced by the smoothed ones."""
    if isinstance(point_tracker, NativeTracking._View):
        if not isinstance(angle_tracker, NativeTracking._View) or angle_tracker._o is not point_tracker._o:
            raise ValueError("native trackers come in pairs (make_trackers())")
        return point_tracker._o.track(centroid, keypoints, orientation, axis_length)
    centroid = np.array(centroid, dtype=np.float64)
    keypoints = np.array(keypoints, dtype=np.float64)
    lengths = np.max(axis_length, axis=1)
    angles = F.clamp_angles_deg(-np.rad2deg(orientation))
    if not point_tracker.is_initialized:
        point_tracker.initialize([centroid, keypoints[:, :, :2]])
    s_cen, s_kpts = point_tracker.smooth_update([centroid, keypoints[:, :, :2]])
    centroid = np.asarray(s_cen, dtype=np.float64)
    keypoints[:, :7, :2] = s_kpts[:, :7, :]
    flips, _ = F.flips_from_keypoints(keypoints, centroid, angles, lengths)
    angles[flips] = F.clamp_angles_deg(angles[flips] + 180)
    rot = F.rotate_points_batch(np.copy(keypoints[:, :7, :2]), centroid, angles)
    scores = F.compute_keypoint_alignment_scores(rot)
    if not angle_tracker.is_initialized:
        angle_tracker.initialize([angles])
    angles, flips = _angle_loop(angle_tracker, angles, np.asarray(flips, dtype=bool), scores)
    return centroid, keypoints, angles, flips
