// Host-side (CPU) tracking branch of the feature step (--use-tracking, the
// reference's default, M/cli.py:366): Kalman smoothing of the centroid and
// keypoints, keypoint head/tail flips, and the per-frame Kalman-assisted
// 180-degree angle correction -- instances_to_features' tracking branch,
// M/proc/proc.py:720-800, with ProcessFeaturesStep's two trackers
// (M/pipeline/process_features_step.py:40-51, M/proc/kalman.py:101-418) and
// pykalman's filter / RTS smoother / EM (em_vars: transition, observation and
// initial-state covariances, n_iter 10) / filter_update as the reference
// calls them.  The trackers carry their state from call to call (chunks in
// session order).  Native so that a rank-0 exchange of an 8-GPU session is not
// bounded by Python: tracking.py holds the numpy statement of the same model,
// which the tests cross-check against.
//
// Structure used: every transition matrix here is block diagonal with 3x3
// (position, velocity, acceleration) blocks, and every observation row picks
// one state component, so A P A^T, C P C^T and K C P are gathers / 3-term
// sums; the covariances themselves are dense (EM learns full Q and R).
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"

// products / sums in any association (FMA allowed): the numpy statement it
// is checked against agrees to ~1e-12, and every decision exactly
#pragma clang fp contract(fast)

namespace {

constexpr double PI_ = 3.141592653589793238462643383279502884;

using Vec = std::vector<double>;

// in-place inverse of the n x n row-major matrix a (Gauss-Jordan, partial
// pivoting); false when singular
bool invert(double *a, int n, double *work) {
    double *inv = work;  // n x n
    for (int i = 0; i < n * n; ++i) inv[i] = 0.0;
    for (int i = 0; i < n; ++i) inv[i * n + i] = 1.0;
    for (int c = 0; c < n; ++c) {
        int p = c;
        double best = std::fabs(a[c * n + c]);
        for (int r = c + 1; r < n; ++r)
            if (std::fabs(a[r * n + c]) > best) {
                best = std::fabs(a[r * n + c]);
                p = r;
            }
        if (best == 0.0 || std::isnan(best)) return false;
        if (p != c)
            for (int k = 0; k < n; ++k) {
                std::swap(a[p * n + k], a[c * n + k]);
                std::swap(inv[p * n + k], inv[c * n + k]);
            }
        const double d = 1.0 / a[c * n + c];
        for (int k = 0; k < n; ++k) {
            a[c * n + k] *= d;
            inv[c * n + k] *= d;
        }
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            const double f = a[r * n + c];
            if (f == 0.0) continue;
            for (int k = 0; k < n; ++k) {
                a[r * n + k] -= f * a[c * n + k];
                inv[r * n + k] -= f * inv[c * n + k];
            }
        }
    }
    std::memcpy(a, inv, sizeof(double) * n * n);
    return true;
}

// in-place lower Cholesky factor of the SPD n x n matrix a (upper part left
// as is); false when not positive definite
bool cholesky(double *a, int n) {
    for (int j = 0; j < n; ++j) {
        double d = a[j * n + j];
        for (int k = 0; k < j; ++k) d -= a[j * n + k] * a[j * n + k];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        a[j * n + j] = d;
        const double inv = 1.0 / d;
        for (int i = j + 1; i < n; ++i) {
            double s = a[i * n + j];
            const double *ri = a + i * n, *rj = a + j * n;
            for (int k = 0; k < j; ++k) s -= ri[k] * rj[k];
            a[i * n + j] = s * inv;
        }
    }
    return true;
}

// X = S^-1 B for S = L L^T (L from cholesky), B and X n x m row-major (in place)
void chol_solve(const double *L, int n, double *B, int m) {
    for (int i = 0; i < n; ++i) {  // L Y = B
        double *bi = B + (size_t)i * m;
        for (int k = 0; k < i; ++k) {
            const double l = L[i * n + k];
            const double *bk = B + (size_t)k * m;
            for (int j = 0; j < m; ++j) bi[j] -= l * bk[j];
        }
        const double inv = 1.0 / L[i * n + i];
        for (int j = 0; j < m; ++j) bi[j] *= inv;
    }
    for (int i = n - 1; i >= 0; --i) {  // L^T X = Y
        double *bi = B + (size_t)i * m;
        for (int k = i + 1; k < n; ++k) {
            const double l = L[k * n + i];
            const double *bk = B + (size_t)k * m;
            for (int j = 0; j < m; ++j) bi[j] -= l * bk[j];
        }
        const double inv = 1.0 / L[i * n + i];
        for (int j = 0; j < m; ++j) bi[j] *= inv;
    }
}

// C (m x n) = A (m x k) B (k x n)
void matmul(const double *A, const double *B, double *C, int m, int k, int n) {
    for (int i = 0; i < m; ++i) {
        double *c = C + (size_t)i * n;
        for (int j = 0; j < n; ++j) c[j] = 0.0;
        for (int t = 0; t < k; ++t) {
            const double a = A[(size_t)i * k + t];
            if (a == 0.0) continue;
            const double *b = B + (size_t)t * n;
            for (int j = 0; j < n; ++j) c[j] += a * b[j];
        }
    }
}

// Linear-Gaussian model with a block-diagonal (3x3 blocks) transition and a
// selection observation matrix (pykalman semantics, zero offsets).
struct KF {
    int ns = 0, no = 0;
    Vec blk;              // the 3x3 (pos, vel, acc) transition block, row-major
    std::vector<int> sel; // observed state component of each observation row
    Vec Q, R, P0, x0;

    void init(int nblocks, double dt, const std::vector<int> &observed) {
        ns = 3 * nblocks;
        no = (int)observed.size();
        const double der[3] = {1.0, dt, dt * dt / 2};
        blk.assign(9, 0.0);
        for (int r = 0; r < 3; ++r)
            for (int c = r; c < 3; ++c) blk[r * 3 + c] = der[c - r];
        sel = observed;
        Q.assign((size_t)ns * ns, 0.0);
        P0.assign((size_t)ns * ns, 0.0);
        R.assign((size_t)no * no, 0.0);
        for (int i = 0; i < ns; ++i) Q[(size_t)i * ns + i] = P0[(size_t)i * ns + i] = 1.0;
        for (int i = 0; i < no; ++i) R[(size_t)i * no + i] = 1.0;
        x0.assign(ns, 0.0);
    }
    // y = A x
    void apply(const double *x, double *y) const {
        for (int b = 0; b < ns; b += 3)
            for (int r = 0; r < 3; ++r) {
                double s = 0.0;
                for (int c = 0; c < 3; ++c) s += blk[r * 3 + c] * x[b + c];
                y[b + r] = s;
            }
    }
    // out = A P A^T (+ Q when addQ)
    void sandwich(const double *P, double *out, double *tmp, bool addQ) const {
        // tmp = A P
        for (int b = 0; b < ns; b += 3)
            for (int r = 0; r < 3; ++r) {
                double *t = tmp + (size_t)(b + r) * ns;
                for (int j = 0; j < ns; ++j) t[j] = 0.0;
                for (int c = 0; c < 3; ++c) {
                    const double a = blk[r * 3 + c];
                    if (a == 0.0) continue;
                    const double *p = P + (size_t)(b + c) * ns;
                    for (int j = 0; j < ns; ++j) t[j] += a * p[j];
                }
            }
        // out = tmp A^T: out[i][b + r] = sum_c tmp[i][b + c] A[r][c]
        for (int i = 0; i < ns; ++i) {
            const double *t = tmp + (size_t)i * ns;
            double *o = out + (size_t)i * ns;
            for (int b = 0; b < ns; b += 3)
                for (int r = 0; r < 3; ++r) {
                    double s = 0.0;
                    for (int c = 0; c < 3; ++c) s += t[b + c] * blk[r * 3 + c];
                    o[b + r] = s + (addQ ? Q[(size_t)i * ns + b + r] : 0.0);
                }
        }
    }
};

struct Work {
    Vec tmp, S, Sinv, K, big;
    void size(int ns, int no) {
        tmp.resize((size_t)ns * ns);
        big.resize((size_t)ns * ns * 2);
        S.resize((size_t)no * no);
        Sinv.resize((size_t)no * no);
        K.resize((size_t)ns * no);
    }
};

// correct (xp, Pp) with observation z (missing: unchanged)
void correct(const KF &f, const double *xp, const double *Pp, const double *z, bool missing, double *x, double *P,
             Work &w) {
    const int ns = f.ns, no = f.no;
    if (missing) {
        std::memcpy(x, xp, sizeof(double) * ns);
        std::memcpy(P, Pp, sizeof(double) * ns * ns);
        return;
    }
    for (int i = 0; i < no; ++i)
        for (int j = 0; j < no; ++j) w.S[i * no + j] = Pp[(size_t)f.sel[i] * ns + f.sel[j]] + f.R[i * no + j];
    std::memcpy(w.Sinv.data(), w.S.data(), sizeof(double) * no * no);
    if (!invert(w.Sinv.data(), no, w.tmp.data())) {
        for (auto &v : w.Sinv) v = NAN;
    }
    // K = Pp[:, sel] Sinv
    for (int i = 0; i < ns; ++i)
        for (int j = 0; j < no; ++j) {
            double s = 0.0;
            for (int k = 0; k < no; ++k) s += Pp[(size_t)i * ns + f.sel[k]] * w.Sinv[k * no + j];
            w.K[(size_t)i * no + j] = s;
        }
    // x = xp + K (z - xp[sel]);  P = Pp - K Pp[sel, :]
    for (int i = 0; i < ns; ++i) {
        double s = 0.0;
        for (int k = 0; k < no; ++k) s += w.K[(size_t)i * no + k] * (z[k] - xp[f.sel[k]]);
        x[i] = xp[i] + s;
    }
    for (int i = 0; i < ns; ++i) {
        double *p = P + (size_t)i * ns;
        for (int j = 0; j < ns; ++j) p[j] = Pp[(size_t)i * ns + j];
        for (int k = 0; k < no; ++k) {
            const double kk = w.K[(size_t)i * no + k];
            if (kk == 0.0) continue;
            const double *r = Pp + (size_t)f.sel[k] * ns;
            for (int j = 0; j < ns; ++j) p[j] -= kk * r[j];
        }
    }
}

// forward filter over T observations (data T x no, missing rows flagged)
struct Pass {
    int T = 0, ns = 0;
    Vec xp, Pp, xf, Pf, xs, Ps, J;
};

void filter_pass(const KF &f, const double *data, const uint8_t *missing, int T, const double *x0, const double *P0,
                 Pass &p, Work &w) {
    const int ns = f.ns;
    const size_t NN = (size_t)ns * ns;
    p.T = T;
    p.ns = ns;
    p.xp.resize((size_t)T * ns);
    p.Pp.resize((size_t)T * NN);
    p.xf.resize((size_t)T * ns);
    p.Pf.resize((size_t)T * NN);
    for (int t = 0; t < T; ++t) {
        double *xp = &p.xp[(size_t)t * ns], *Pp = &p.Pp[(size_t)t * NN];
        if (t == 0) {
            std::memcpy(xp, x0, sizeof(double) * ns);
            std::memcpy(Pp, P0, sizeof(double) * NN);
        } else {
            f.apply(&p.xf[(size_t)(t - 1) * ns], xp);
            f.sandwich(&p.Pf[(size_t)(t - 1) * NN], Pp, w.tmp.data(), true);
        }
        correct(f, xp, Pp, data + (size_t)t * f.no, missing[t] != 0, &p.xf[(size_t)t * ns], &p.Pf[(size_t)t * NN],
                w);
    }
}

// RTS smoother: J[t] = Pf[t] A^T Pp[t+1]^-1, formed as J^T = Pp[t+1]^-1 (A
// Pf[t]) by a Cholesky solve (Pp is symmetric positive definite; Gauss-Jordan
// when the factorisation fails)
void smooth_pass(const KF &f, Pass &p, Work &w, bool want_J) {
    const int T = p.T, ns = f.ns;
    const size_t NN = (size_t)ns * ns;
    p.xs.resize((size_t)T * ns);
    p.Ps.resize((size_t)T * NN);
    if (want_J) p.J.resize((size_t)(T > 1 ? T - 1 : 0) * NN);
    if (T == 0) return;
    std::memcpy(&p.xs[(size_t)(T - 1) * ns], &p.xf[(size_t)(T - 1) * ns], sizeof(double) * ns);
    std::memcpy(&p.Ps[(size_t)(T - 1) * NN], &p.Pf[(size_t)(T - 1) * NN], sizeof(double) * NN);
    Vec L(NN), Jt(NN), JT(NN), d(NN), dv(ns), jd(NN);
    for (int t = T - 2; t >= 0; --t) {
        const double *Pf = &p.Pf[(size_t)t * NN], *Pp1 = &p.Pp[(size_t)(t + 1) * NN];
        // JT = A Pf[t]  (= (Pf A^T)^T, Pf symmetric)
        for (int b = 0; b < ns; b += 3)
            for (int r = 0; r < 3; ++r) {
                double *o = &JT[(size_t)(b + r) * ns];
                for (int j = 0; j < ns; ++j) o[j] = 0.0;
                for (int c = 0; c < 3; ++c) {
                    const double a = f.blk[r * 3 + c];
                    if (a == 0.0) continue;
                    const double *pr = Pf + (size_t)(b + c) * ns;
                    for (int j = 0; j < ns; ++j) o[j] += a * pr[j];
                }
            }
        std::memcpy(L.data(), Pp1, sizeof(double) * NN);
        if (cholesky(L.data(), ns)) {
            chol_solve(L.data(), ns, JT.data(), ns);  // JT = Pp^-1 A Pf = J^T
        } else {
            std::memcpy(L.data(), Pp1, sizeof(double) * NN);
            if (!invert(L.data(), ns, w.big.data()))
                for (auto &v : L) v = NAN;
            Vec tmp(JT);
            matmul(L.data(), tmp.data(), JT.data(), ns, ns, ns);
        }
        for (int i = 0; i < ns; ++i)
            for (int j = 0; j < ns; ++j) Jt[(size_t)i * ns + j] = JT[(size_t)j * ns + i];
        if (want_J) std::memcpy(&p.J[(size_t)t * NN], JT.data(), sizeof(double) * NN);  // stored transposed
        // xs[t] = xf[t] + J (xs[t+1] - xp[t+1])
        for (int i = 0; i < ns; ++i) dv[i] = p.xs[(size_t)(t + 1) * ns + i] - p.xp[(size_t)(t + 1) * ns + i];
        for (int i = 0; i < ns; ++i) {
            double s = 0.0;
            const double *ji = &Jt[(size_t)i * ns];
            for (int k = 0; k < ns; ++k) s += ji[k] * dv[k];
            p.xs[(size_t)t * ns + i] = p.xf[(size_t)t * ns + i] + s;
        }
        // Ps[t] = Pf[t] + J (Ps[t+1] - Pp[t+1]) J^T  (symmetric: upper half, mirrored)
        for (size_t q = 0; q < NN; ++q) d[q] = p.Ps[(size_t)(t + 1) * NN + q] - Pp1[q];
        matmul(Jt.data(), d.data(), jd.data(), ns, ns, ns);
        double *Ps = &p.Ps[(size_t)t * NN];
        matmul(jd.data(), JT.data(), Ps, ns, ns, ns);
        for (size_t q = 0; q < NN; ++q) Ps[q] += Pf[q];
    }
}

// Smoothed means only (what smooth_update returns; its last covariance is
// Pf[T-1]): xs[t] = xf[t] + Pf[t] A^T Pp[t+1]^-1 (xs[t+1] - xp[t+1]), a
// Cholesky factorisation and two triangular vector solves per step instead
// of the full gain matrix and covariance recursion
void smooth_means(const KF &f, Pass &p, Work &w) {
    const int T = p.T, ns = f.ns;
    const size_t NN = (size_t)ns * ns;
    p.xs.resize((size_t)T * ns);
    if (T == 0) return;
    std::memcpy(&p.xs[(size_t)(T - 1) * ns], &p.xf[(size_t)(T - 1) * ns], sizeof(double) * ns);
    Vec L(NN), y(ns), ay(ns);
    for (int t = T - 2; t >= 0; --t) {
        const double *Pp1 = &p.Pp[(size_t)(t + 1) * NN], *Pf = &p.Pf[(size_t)t * NN];
        for (int i = 0; i < ns; ++i) y[i] = p.xs[(size_t)(t + 1) * ns + i] - p.xp[(size_t)(t + 1) * ns + i];
        std::memcpy(L.data(), Pp1, sizeof(double) * NN);
        if (cholesky(L.data(), ns)) {
            chol_solve(L.data(), ns, y.data(), 1);
        } else {
            std::memcpy(L.data(), Pp1, sizeof(double) * NN);
            if (!invert(L.data(), ns, w.big.data()))
                for (auto &v : L) v = NAN;
            Vec v(y);
            for (int i = 0; i < ns; ++i) {
                double s = 0.0;
                for (int k = 0; k < ns; ++k) s += L[(size_t)i * ns + k] * v[k];
                y[i] = s;
            }
        }
        // ay = A^T y
        for (int b = 0; b < ns; b += 3)
            for (int c = 0; c < 3; ++c) {
                double s = 0.0;
                for (int r = 0; r < 3; ++r) s += f.blk[r * 3 + c] * y[b + r];
                ay[b + c] = s;
            }
        for (int i = 0; i < ns; ++i) {
            double s = 0.0;
            const double *pr = Pf + (size_t)i * ns;
            for (int k = 0; k < ns; ++k) s += pr[k] * ay[k];
            p.xs[(size_t)t * ns + i] = p.xf[(size_t)t * ns + i] + s;
        }
    }
}

// EM on Q, R, P0 (n_iter passes), pykalman's M-step formulas
void em(KF &f, const double *data, const uint8_t *missing, int T, int n_iter, Work &w) {
    const int ns = f.ns, no = f.no;
    const size_t NN = (size_t)ns * ns;
    Pass p;
    Vec tot(NN), tmp(NN), tmp2(NN);
    for (int it = 0; it < n_iter; ++it) {
        filter_pass(f, data, missing, T, f.x0.data(), f.P0.data(), p, w);
        smooth_pass(f, p, w, true);
        // observation covariance
        int nobs = 0;
        Vec Rn((size_t)no * no, 0.0);
        for (int t = 0; t < T; ++t) {
            if (missing[t]) continue;
            ++nobs;
            const double *z = data + (size_t)t * no, *x = &p.xs[(size_t)t * ns], *P = &p.Ps[(size_t)t * NN];
            for (int i = 0; i < no; ++i)
                for (int j = 0; j < no; ++j)
                    Rn[i * no + j] += (z[i] - x[f.sel[i]]) * (z[j] - x[f.sel[j]]) + P[(size_t)f.sel[i] * ns + f.sel[j]];
        }
        for (auto &v : Rn) v = nobs > 0 ? v / nobs : 0.0;
        // transition covariance
        if (T > 1) {
            std::fill(tot.begin(), tot.end(), 0.0);
            Vec ax(ns), e(ns);
            for (int t = 0; t + 1 < T; ++t) {
                const double *x1 = &p.xs[(size_t)(t + 1) * ns];
                f.apply(&p.xs[(size_t)t * ns], ax.data());
                for (int i = 0; i < ns; ++i) e[i] = x1[i] - ax[i];
                // A Ps[t] A^T + Ps[t+1]
                f.sandwich(&p.Ps[(size_t)t * NN], tmp.data(), w.tmp.data(), false);
                // V = Ps[t+1] J[t]^T A^T  (p.J holds J^T)
                const double *P1 = &p.Ps[(size_t)(t + 1) * NN];
                matmul(P1, &p.J[(size_t)t * NN], tmp2.data(), ns, ns, ns);  // Ps[t+1] J^T
                for (int i = 0; i < ns; ++i) {
                    for (int b = 0; b < ns; b += 3)
                        for (int r = 0; r < 3; ++r) {
                            double s = 0.0;
                            for (int c = 0; c < 3; ++c) s += tmp2[(size_t)i * ns + b + c] * f.blk[r * 3 + c];
                            w.tmp[(size_t)i * ns + b + r] = s;  // V[i][b+r]
                        }
                }
                for (int i = 0; i < ns; ++i)
                    for (int j = 0; j < ns; ++j)
                        tot[(size_t)i * ns + j] += e[i] * e[j] + tmp[(size_t)i * ns + j] + P1[(size_t)i * ns + j] -
                                                   w.tmp[(size_t)i * ns + j] - w.tmp[(size_t)j * ns + i];
            }
            for (size_t q = 0; q < NN; ++q) f.Q[q] = (1.0 / (T - 1)) * tot[q];
        }
        f.R = Rn;
        // initial state covariance
        const double *z0 = &p.xs[0], *x0 = f.x0.data();
        for (int i = 0; i < ns; ++i)
            for (int j = 0; j < ns; ++j)
                f.P0[(size_t)i * ns + j] =
                    p.Ps[(size_t)i * ns + j] + z0[i] * z0[j] - x0[i] * z0[j] - z0[i] * x0[j] + x0[i] * x0[j];
    }
}

struct Tracker {
    KF kf;
    bool ready = false;
    Vec last_mean, last_cov;
    Work w;
};

// KalmanTracker.initialize: x0 from row 0, EM over the rows holding any finite value
void tracker_init(Tracker &tr, int nblocks, const std::vector<int> &observed, const double *Z, int T) {
    KF &f = tr.kf;
    f.init(nblocks, 1.0, observed);
    tr.w.size(f.ns, f.no);
    for (int i = 0; i < f.no; ++i) f.x0[f.sel[i]] = T > 0 ? Z[i] : 0.0;
    std::vector<double> rows;
    std::vector<uint8_t> miss;
    for (int t = 0; t < T; ++t) {
        bool any = false, all = true;
        for (int i = 0; i < f.no; ++i) {
            const bool fin = std::isfinite(Z[(size_t)t * f.no + i]);
            any |= fin;
            all &= fin;
        }
        if (!any) continue;
        rows.insert(rows.end(), Z + (size_t)t * f.no, Z + (size_t)(t + 1) * f.no);
        miss.push_back(all ? 0 : 1);
    }
    if (!miss.empty()) em(f, rows.data(), miss.data(), (int)miss.size(), 10, tr.w);
    tr.last_mean = f.x0;
    tr.last_cov = f.P0;
    tr.ready = true;
}

// KalmanTracker.smooth_update over T rows: smoothed means -> out (T x ns)
void tracker_smooth_update(Tracker &tr, const double *Z, int T, Vec &out) {
    KF &f = tr.kf;
    const int ns = f.ns;
    const size_t NN = (size_t)ns * ns;
    std::vector<uint8_t> miss(T);
    for (int t = 0; t < T; ++t) {
        bool all = true;
        for (int i = 0; i < f.no; ++i) all &= std::isfinite(Z[(size_t)t * f.no + i]);
        miss[t] = all ? 0 : 1;
    }
    out.resize((size_t)T * ns);
    if (T == 1) {  // filter_update from the last state (initial state untouched)
        Vec xp(ns), Pp(NN), x(ns), P(NN);
        f.apply(tr.last_mean.data(), xp.data());
        f.sandwich(tr.last_cov.data(), Pp.data(), tr.w.tmp.data(), true);
        correct(f, xp.data(), Pp.data(), Z, miss[0] != 0, x.data(), P.data(), tr.w);
        tr.last_mean = x;
        tr.last_cov = P;
        std::memcpy(out.data(), x.data(), sizeof(double) * ns);
        return;
    }
    Pass p;
    filter_pass(f, Z, miss.data(), T, f.x0.data(), f.P0.data(), p, tr.w);
    smooth_means(f, p, tr.w);
    std::memcpy(out.data(), p.xs.data(), sizeof(double) * T * ns);
    f.x0.assign(p.xs.end() - ns, p.xs.end());
    f.P0.assign(p.Pf.end() - NN, p.Pf.end());  // Ps[T-1] = Pf[T-1]
    tr.last_mean = f.x0;
    tr.last_cov = f.P0;
}

// numpy float64 remainder (npy_divmod)
inline double np_remainder(double a, double b) {
    double m = std::fmod(a, b);
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = std::copysign(0.0, b);
    }
    return m;
}
inline double clamp_deg(double a) { return np_remainder(a < 0 ? 360 + a : a, 360.0); }

const int EXPECTED[7][7] = {{0, 1, 1, 1, 1, 1, 1},     {-1, 0, 0, 1, 1, 1, 1},   {-1, 0, 0, 1, 1, 1, 1},
                            {-1, -1, -1, 0, 1, 1, 1},  {-1, -1, -1, -1, 0, 0, 1}, {-1, -1, -1, -1, 0, 0, 1},
                            {-1, -1, -1, -1, -1, -1, 0}};

struct Tracking {
    int K;
    Tracker point, angle;
};

}  // namespace

extern "C" void *mdx_tracking_create(int n_keypoints) {
    if (n_keypoints < 7 || n_keypoints > 64) {
        mdx::set_error("mdx_tracking_create: 7..64 keypoints");
        return nullptr;
    }
    Tracking *t = new Tracking();
    t->K = n_keypoints;
    return t;
}

extern "C" int mdx_tracking_destroy(void *h) {
    delete (Tracking *)h;
    return MDX_OK;
}

extern "C" int mdx_tracking_state(void *h, int which, int *initialized, double *mean, int64_t mean_len) {
    MDX_REQUIRE(h && initialized && (which == 0 || which == 1), "mdx_tracking_state: bad arguments");
    Tracker &tr = which == 0 ? ((Tracking *)h)->point : ((Tracking *)h)->angle;
    *initialized = tr.ready ? 1 : 0;
    if (mean && tr.ready) {
        MDX_REQUIRE(mean_len >= (int64_t)tr.last_mean.size(), "mdx_tracking_state: mean buffer too small");
        std::memcpy(mean, tr.last_mean.data(), sizeof(double) * tr.last_mean.size());
    }
    return tr.ready ? (int)tr.last_mean.size() : 0;
}

extern "C" int mdx_tracking_track(void *h, int64_t n, int K, const double *centroid, const double *keypoints,
                                  const double *orientation, const double *axis_length, double *centroid_out,
                                  double *keypoints_out, double *angles_out, uint8_t *flips_out) {
    MDX_REQUIRE(h && n >= 0, "mdx_tracking_track: bad arguments");
    Tracking &tk = *(Tracking *)h;
    MDX_REQUIRE(K == tk.K, "mdx_tracking_track: tracker built for %d keypoints, got %d", tk.K, K);
    MDX_REQUIRE(n == 0 || (centroid && keypoints && orientation && axis_length && centroid_out && keypoints_out &&
                           angles_out && flips_out),
                "mdx_tracking_track: null pointer");
    if (n == 0) return MDX_OK;
    const int T = (int)n;
    // point tracker: observations [cx, cy, kp0x, kp0y, ...]; state blocks
    // (x, y) of the centroid then of every keypoint, position first
    const int no = 2 + 2 * K;
    std::vector<int> obs_sel(no);
    for (int i = 0; i < no; ++i) obs_sel[i] = 3 * i;
    Vec Z((size_t)T * no);
    for (int t = 0; t < T; ++t) {
        Z[(size_t)t * no] = centroid[2 * t];
        Z[(size_t)t * no + 1] = centroid[2 * t + 1];
        for (int k = 0; k < K; ++k) {
            Z[(size_t)t * no + 2 + 2 * k] = keypoints[((size_t)t * K + k) * 3];
            Z[(size_t)t * no + 3 + 2 * k] = keypoints[((size_t)t * K + k) * 3 + 1];
        }
    }
    if (!tk.point.ready) tracker_init(tk.point, no, obs_sel, Z.data(), T);
    Vec xs;
    tracker_smooth_update(tk.point, Z.data(), T, xs);
    const int ns = tk.point.kf.ns;
    std::memcpy(keypoints_out, keypoints, sizeof(double) * T * K * 3);
    for (int t = 0; t < T; ++t) {
        centroid_out[2 * t] = xs[(size_t)t * ns];
        centroid_out[2 * t + 1] = xs[(size_t)t * ns + 3];
        for (int k = 0; k < 7 && k < K; ++k) {  // the tail tip (8th) keeps its inference
            keypoints_out[((size_t)t * K + k) * 3] = xs[(size_t)t * ns + 6 + 6 * k];
            keypoints_out[((size_t)t * K + k) * 3 + 1] = xs[(size_t)t * ns + 9 + 6 * k];
        }
    }
    // angles, keypoint flips, alignment scores
    Vec ang(T), conf(T), score(T);
    std::vector<uint8_t> flips(T);
    for (int t = 0; t < T; ++t) {
        const double a0 = axis_length[2 * t], a1 = axis_length[2 * t + 1];
        const double len = (std::isnan(a0) || std::isnan(a1)) ? NAN : (a0 > a1 ? a0 : a1);
        ang[t] = clamp_deg(-(orientation[t] * (180.0 / PI_)));
        mdx_flips_from_keypoints(keypoints_out + (size_t)t * K * 3, 1, K, centroid_out + 2 * t, &ang[t], &len,
                                 &flips[t], &conf[t]);
        if (flips[t]) ang[t] = clamp_deg(ang[t] + 180);
        // alignment score of the first 7 keypoints rotated by -angle about the centroid
        const double th = (-ang[t]) * (PI_ / 180.0);
        const double c = std::cos(th), s = std::sin(th);
        const double ox = centroid_out[2 * t], oy = centroid_out[2 * t + 1];
        double xr[7];
        for (int k = 0; k < 7; ++k) {
            const double dx = keypoints_out[((size_t)t * K + k) * 3] - ox;
            const double dy = keypoints_out[((size_t)t * K + k) * 3 + 1] - oy;
            xr[k] = c * dx + (-s) * dy + ox;
        }
        int met = 0, total = 0;
        for (int i = 0; i < 7; ++i)
            for (int j = 0; j < 7; ++j) {
                if (!EXPECTED[i][j]) continue;
                ++total;
                const double d = xr[i] - xr[j];
                const int sg = d > 0 ? 1 : (d < 0 ? -1 : 0);  // NaN -> 0 (np.sign gives NaN, never equal)
                met += !std::isnan(d) && sg == EXPECTED[i][j];
            }
        score[t] = (double)met / total;
    }
    // angle tracker: (sin, cos) of the angle, 2 position-velocity-acceleration blocks
    if (!tk.angle.ready) {
        Vec Za((size_t)T * 2);
        for (int t = 0; t < T; ++t) {
            const double r = ang[t] * (PI_ / 180.0);
            Za[2 * t] = std::sin(r);
            Za[2 * t + 1] = std::cos(r);
        }
        tracker_init(tk.angle, 2, {0, 3}, Za.data(), T);
    }
    Tracker &at = tk.angle;
    const KF &f = at.kf;
    Vec xp(6), Pp(36), x(6), P(36);
    for (int t = 0; t < T; ++t) {
        // sample(1): the current state's angle
        double p = std::atan2(at.last_mean[0], at.last_mean[3]);
        p = (p < 0 ? 2 * PI_ + p : p) * (180.0 / PI_);
        double diff = np_remainder(ang[t] - p, 360.0);
        if (diff > 180) diff = -(360 - diff);
        if (score[t] < 0.4) {
            ang[t] = p;
        } else if (std::fabs(diff) > 140) {
            ang[t] = clamp_deg(ang[t] + 180);
            flips[t] = !flips[t];
        }
        const double r = ang[t] * (PI_ / 180.0);
        const double z[2] = {std::sin(r), std::cos(r)};
        f.apply(at.last_mean.data(), xp.data());
        f.sandwich(at.last_cov.data(), Pp.data(), at.w.tmp.data(), true);
        correct(f, xp.data(), Pp.data(), z, !(std::isfinite(z[0]) && std::isfinite(z[1])), x.data(), P.data(), at.w);
        at.last_mean = x;
        at.last_cov = P;
    }
    for (int t = 0; t < T; ++t) {
        angles_out[t] = ang[t];
        flips_out[t] = flips[t];
    }
    return MDX_OK;
}
