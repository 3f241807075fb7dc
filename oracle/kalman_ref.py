"""Loop-level restatement of the tracking branch's Kalman machinery (TEST
INFRASTRUCTURE ONLY -- the checker of moseq2_detectron_extract_amd.tracking).

The reference drives ``pykalman.KalmanFilter`` (M/proc/kalman.py:6,322-418;
``pykalman`` is unpinned in setup.py:39 and absent from every interpreter in
this image, so PARITY IS UNPINNED: no fixture of the reference covers it).
This file restates pykalman 0.9.x ``standard.py`` as published, one time step
at a time, with ``scipy.linalg.pinv`` exactly where pykalman calls it:

  _filter_predict / _filter_correct / _filter     (a masked observation row
                                                    skips the correction)
  _smooth_update / _smooth / _smooth_pair          (RTS smoother)
  _em_observation_covariance / _em_transition_covariance /
  _em_initial_state_covariance                     (the three EM variables the
                                                    reference learns, kalman.py:326)
  KalmanFilter.em / smooth / filter / filter_update / sample
and the reference's tracker items (M/proc/kalman.py:101-278) and
KalmanTracker (:281-418), plus the per-frame angle loop of
instances_to_features (M/proc/proc.py:769-800).
"""
from __future__ import annotations

import numpy as np
import numpy.ma as ma
from scipy import linalg
from scipy.linalg import block_diag


# ---------------------------------------------------------------- pykalman core
def _filter_predict(A, Q, b, x, P):
    return A @ x + b, A @ (P @ A.T) + Q


def _filter_correct(C, R, d, x_pred, P_pred, z):
    if not np.any(ma.getmask(z)):
        y = C @ x_pred + d
        S = C @ (P_pred @ C.T) + R
        K = P_pred @ (C.T @ linalg.pinv(S))
        x = x_pred + K @ (np.asarray(z) - y)
        P = P_pred - K @ (C @ P_pred)
        return K, x, P
    return np.zeros((P_pred.shape[0], C.shape[0])), x_pred, P_pred


def _filter(A, C, Q, R, b, d, x0, P0, Z):
    T, ns = Z.shape[0], A.shape[0]
    xp = np.zeros((T, ns)); Pp = np.zeros((T, ns, ns))
    xf = np.zeros((T, ns)); Pf = np.zeros((T, ns, ns))
    for t in range(T):
        if t == 0:
            xp[t], Pp[t] = x0, P0
        else:
            xp[t], Pp[t] = _filter_predict(A, Q, b, xf[t - 1], Pf[t - 1])
        _, xf[t], Pf[t] = _filter_correct(C, R, d, xp[t], Pp[t], Z[t])
    return xp, Pp, xf, Pf


def _smooth(A, xf, Pf, xp, Pp):
    T, ns = xf.shape
    xs = np.zeros((T, ns)); Ps = np.zeros((T, ns, ns)); J = np.zeros((T - 1, ns, ns))
    xs[-1], Ps[-1] = xf[-1], Pf[-1]
    for t in reversed(range(T - 1)):
        J[t] = Pf[t] @ (A.T @ linalg.pinv(Pp[t + 1]))
        xs[t] = xf[t] + J[t] @ (xs[t + 1] - xp[t + 1])
        Ps[t] = Pf[t] + J[t] @ ((Ps[t + 1] - Pp[t + 1]) @ J[t].T)
    return xs, Ps, J


def _smooth_pair(Ps, J):
    T, ns, _ = Ps.shape
    pair = np.zeros((T, ns, ns))
    for t in range(1, T):
        pair[t] = Ps[t] @ J[t - 1].T
    return pair


def _em_observation_covariance(Z, d, C, xs, Ps):
    res = np.zeros((Z.shape[1], Z.shape[1]))
    n = 0
    for t in range(Z.shape[0]):
        if not np.any(ma.getmask(Z[t])):
            err = np.asarray(Z[t]) - C @ xs[t] - d
            res += np.outer(err, err) + C @ (Ps[t] @ C.T)
            n += 1
    return res / n if n > 0 else res


def _em_transition_covariance(A, b, xs, Ps, pair):
    T, ns = xs.shape
    res = np.zeros((ns, ns))
    for t in range(T - 1):
        err = xs[t + 1] - A @ xs[t] - b
        V = pair[t + 1] @ A.T
        res += np.outer(err, err) + A @ (Ps[t] @ A.T) + Ps[t + 1] - V - V.T
    return (1.0 / (T - 1)) * res


def _em_initial_state_covariance(x0, xs, Ps):
    z = xs[0]
    return Ps[0] + np.outer(z, z) - np.outer(x0, z) - np.outer(z, x0) + np.outer(x0, x0)


class KalmanFilter:
    """pykalman.KalmanFilter restricted to what the reference uses: fixed
    transition/observation matrices, zero offsets, identity covariances until
    EM learns Q, R and P0."""

    def __init__(self, A, C, x0):
        self.A, self.C = np.asarray(A, float), np.atleast_2d(np.asarray(C, float))
        ns, no = self.A.shape[0], self.C.shape[0]
        self.x0 = np.asarray(x0, float)
        self.Q, self.R, self.P0 = np.eye(ns), np.eye(no), np.eye(ns)
        self.b, self.d = np.zeros(ns), np.zeros(no)

    @staticmethod
    def _obs(X):
        X = ma.asarray(X)
        return X[:, None] if X.ndim == 1 else X

    def em(self, X, n_iter=10):
        Z = self._obs(X)
        for _ in range(n_iter):
            xp, Pp, xf, Pf = _filter(self.A, self.C, self.Q, self.R, self.b, self.d, self.x0, self.P0, Z)
            xs, Ps, J = _smooth(self.A, xf, Pf, xp, Pp)
            pair = _smooth_pair(Ps, J)
            # pykalman _em order: observation covariance, transition covariance,
            # initial state covariance (initial mean, matrices, offsets given)
            self.R = _em_observation_covariance(Z, self.d, self.C, xs, Ps)
            self.Q = _em_transition_covariance(self.A, self.b, xs, Ps, pair)
            self.P0 = _em_initial_state_covariance(self.x0, xs, Ps)
        return self

    def smooth(self, X):
        Z = self._obs(X)
        xp, Pp, xf, Pf = _filter(self.A, self.C, self.Q, self.R, self.b, self.d, self.x0, self.P0, Z)
        xs, Ps, _ = _smooth(self.A, xf, Pf, xp, Pp)
        return xs, Ps

    def filter(self, X):
        Z = self._obs(X)
        _, _, xf, Pf = _filter(self.A, self.C, self.Q, self.R, self.b, self.d, self.x0, self.P0, Z)
        return xf, Pf

    def filter_update(self, x, P, z):
        xp, Pp = _filter_predict(self.A, self.Q, self.b, x, P)
        _, xn, Pn = _filter_correct(self.C, self.R, self.d, xp, Pp, ma.asarray(z))
        return xn, Pn

    def sample1(self, x_init):
        """sample(1, x_init) states: the given state itself (the observation
        noise draw does not reach the states)."""
        return np.asarray(x_init, float)[None, :]


# ---------------------------------------------------------------- tracker items
def _point1d_A(order, dt):
    der = [1.0, dt, dt ** 2 / 2, dt ** 3 / 6][:order]
    A = np.zeros((order, order))
    for r in range(order):
        for i, j in enumerate(range(r, order)):
            A[r, j] = der[i]
    return A


def _point1d_C(order):
    c = np.zeros((order,))
    c[0] = 1
    return c


def point_tracker_matrices(n_kp=8, order=3, dt=1.0):
    """Centroid (Point2D) + n_kp keypoints (NPoints2D), process_features_step.py:42-45."""
    A1, C1 = _point1d_A(order, dt), _point1d_C(order)
    A = block_diag(*([A1] * (2 + 2 * n_kp)))
    C = block_diag(*([C1] * (2 + 2 * n_kp)))
    return A, C


def angle_tracker_matrices(order=3, dt=1.0):
    A1, C1 = _point1d_A(order, dt), _point1d_C(order)
    return block_diag(A1, A1), block_diag(C1, C1)


def point_init_mean(centroid, kpts, order=3):
    """first row of each coordinate, zero derivatives (kalman.py:175-209,262-268)."""
    vals = []
    vals += [centroid[0, 0] if len(centroid) else 0, centroid[0, 1] if len(centroid) else 0]
    for i in range(kpts.shape[1]):
        vals += [kpts[0, i, 0] if len(kpts) else 0, kpts[0, i, 1] if len(kpts) else 0]
    x0 = np.zeros(len(vals) * order)
    x0[::order] = vals
    return x0


def point_format(centroid, kpts):
    return ma.masked_invalid(np.column_stack([centroid.reshape(len(centroid), -1), kpts.reshape(len(kpts), -1)]))


def angle_format(angles_deg):
    r = np.deg2rad(angles_deg)
    return np.column_stack([np.sin(r), np.cos(r)])


def angle_from_state(state, order=3):
    yx = state[:, ::order]
    a = np.arctan2(yx[:, 0], yx[:, 1])
    a = np.where(a < 0, 2 * np.pi + a, a)
    return np.rad2deg(a)


class RefTracker:
    """KalmanTracker (kalman.py:281-418) over one KalmanFilter."""

    def __init__(self, A, C):
        self.A, self.C = A, C
        self.kf = None

    def initialize(self, x0, Z):
        self.kf = KalmanFilter(self.A, self.C, x0)
        fin = np.isfinite(ma.getdata(Z)).any(axis=1)  # rows with any finite value (kalman.py:331)
        if np.count_nonzero(fin) > 0:
            self.kf.em(Z[fin], n_iter=10)
        self.last_mean, self.last_covar = self.kf.x0, self.kf.P0

    def smooth_update(self, Z):
        if Z.shape[0] == 1:
            self.last_mean, self.last_covar = self.kf.filter_update(self.last_mean, self.last_covar, Z[0])
            return self.last_mean[None, :]
        xs, Ps = self.kf.smooth(Z)
        self.last_mean = self.kf.x0 = xs[-1]
        self.last_covar = self.kf.P0 = Ps[-1]
        return xs

    def filter_update(self, z):
        self.last_mean, self.last_covar = self.kf.filter_update(self.last_mean, self.last_covar, z)
        return self.last_mean[None, :]


def angle_loop_ref(angle_tracker: RefTracker, angles, flips, kpt_alignment_scores):
    """proc.py:764-800: per frame, peek at the tracker's state, defer to it on
    a low keypoint alignment score, flip on a >140 degree disagreement, then
    filter_update with the (possibly corrected) angle."""
    angles = np.array(angles, dtype=float)
    flips = np.array(flips, dtype=bool)
    if angle_tracker.kf is None:
        a0 = angle_format(angles)
        x0 = np.zeros(6)
        if len(angles):
            x0[0], x0[3] = a0[0, 0], a0[0, 1]
        angle_tracker.initialize(x0, ma.masked_invalid(a0))
    for i in range(angles.shape[0]):
        p = angle_from_state(angle_tracker.last_mean[None, :])[0]
        diff = (angles[i] - p) % 360
        if diff > 180:
            diff = -(360 - diff)
        if kpt_alignment_scores[i] < 0.4:
            angles[i] = p
        elif abs(diff) > 140:
            a = angles[i] + 180
            angles[i] = (360 + a if a < 0 else a) % 360
            flips[i] = ~flips[i]
        angle_tracker.filter_update(ma.masked_invalid(angle_format(angles[[i]]))[0])
    return angles, flips
