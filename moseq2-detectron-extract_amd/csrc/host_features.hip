// Host-side (CPU) restatement of the angle filter of the no-tracking branch,
// iterative_filter_angles (M/proc/proc.py:600-654) with bottleneck's
// move_median(window, min_count=1): native so that the extract loop's host
// step runs without holding the Python GIL.  Same double arithmetic as the
// numpy code (no FMA contraction), so results are bit-identical.
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

namespace {

// median of the non-NaN values among v[0..c) (c <= 8); NaN when none
double nan_median(const double *v, int c) {
    double s[8];
    int k = 0;
    for (int i = 0; i < c; ++i)
        if (!std::isnan(v[i])) s[k++] = v[i];
    if (k == 0) return NAN;
    for (int i = 1; i < k; ++i)  // insertion sort (k <= 8)
        for (int j = i; j > 0 && s[j - 1] > s[j]; --j) {
            const double t = s[j];
            s[j] = s[j - 1];
            s[j - 1] = t;
        }
    return (k & 1) ? s[(k - 1) / 2] : (s[k / 2 - 1] + s[k / 2]) / 2;
}

// np.isclose(a, b) with the default rtol 1e-5, atol 1e-8 (False for NaN)
inline bool isclose(double a, double b) {
    if (std::isnan(a) || std::isnan(b)) return false;
    if (std::isinf(a) || std::isinf(b)) return a == b;
    return std::fabs(a - b) <= 1e-8 + 1e-5 * std::fabs(b);
}

}  // namespace

extern "C" int mdx_iterative_filter_angles(const double *angles, int64_t n, int window, double tolerance,
                                           int max_iters, double *out, uint8_t *flips) {
    MDX_REQUIRE(n >= 0 && (n == 0 || (angles && out && flips)), "mdx_iterative_filter_angles: bad arguments");
    MDX_REQUIRE(window >= 1 && window <= 8, "mdx_iterative_filter_angles: window must be 1..8");
    if (n == 0) return MDX_OK;
    const int w = window < n ? window : (int)n;  // filter_angles: min(window, len)
    std::vector<double> last(angles, angles + n), curr(n);
    const std::vector<double> *result = &last;  // numpy's `curr` at loop exit
    int iterations = 0;
    for (;;) {
        if (iterations > max_iters) break;  // then curr is last (numpy: last = curr)
        ++iterations;
        // filter_angles(last)
        for (int64_t i = 0; i < n; ++i) {
            const int64_t b = i - w + 1 < 0 ? 0 : i - w + 1;
            const double med = nan_median(&last[b], (int)(i - b + 1));
            const double diff = last[i] - med;
            const double ad = std::fabs(diff);
            double v = last[i];
            if ((ad > (180 - tolerance)) && (ad < (180 + tolerance))) {
                const double sg = diff > 0 ? 1.0 : (diff < 0 ? -1.0 : 0.0);
                v = v + (-180 * sg);
            }
            curr[i] = v;
        }
        // np.allclose(curr, last): every pair close (a NaN anywhere: False)
        bool same = true;
        for (int64_t i = 0; i < n && same; ++i) same = isclose(curr[i], last[i]);
        if (same) {
            result = &curr;
            break;
        }
        last.swap(curr);
    }
    const std::vector<double> &r = *result;
    for (int64_t i = 0; i < n; ++i) {
        out[i] = r[i];
        flips[i] = isclose(std::fabs(r[i] - angles[i]), 180.0) ? 1 : 0;
    }
    return MDX_OK;
}

namespace {

// numpy's float64 remainder (npy_divmod): fmod, moved to the divisor's sign,
// +0.0 for an exact zero
inline double np_remainder(double a, double b) {
    double m = std::fmod(a, b);
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = std::copysign(0.0, b);
    }
    return m;
}

// clamp_angles_deg (M/proc/proc.py:688-692): where(a < 0, 360 + a, a) % 360
inline double clamp_deg(double a) { return np_remainder(a < 0 ? 360 + a : a, 360.0); }

constexpr double PI_ = 3.141592653589793238462643383279502884;

// One frame of the keypoint head/tail vote: the front (0-3) and rear (4-6)
// keypoints, rotated by -angle about the centroid, each side by which end
// of the body axis (centroid x +- length / 2) it is nearer to.
void flip_vote(const double *kp, int K, double ox, double oy, double angle_deg, double length, uint8_t *flip,
               double *conf) {
    const double a = (-angle_deg) * (PI_ / 180.0);  // np.deg2rad
    const double c = std::cos(a), s = std::sin(a);
    const double lo = ox - length / 2, hi = ox + length / 2;
    int side[7];
    for (int k = 0; k < 7; ++k) {
        const double dx = kp[3 * k] - ox, dy = kp[3 * k + 1] - oy;
        const double xr = c * dx + (-s) * dy + ox;
        side[k] = std::fabs(lo - xr) < std::fabs(hi - xr) ? -1 : 1;  // NaN -> +1, as np.where
    }
    (void)K;
    const double front = (double)(side[0] + side[1] + side[2] + side[3]) / 4;
    const double rear = (double)(side[4] + side[5] + side[6]) / 3;
    const bool f = front < rear;
    const int ef = f ? -1 : 1, er = -ef;
    int agree = 0;
    for (int k = 0; k < 4; ++k) agree += side[k] == ef;
    for (int k = 4; k < 7; ++k) agree += side[k] == er;
    *flip = f ? 1 : 0;
    *conf = agree / 7.0;
}

}  // namespace

// flips_from_keypoints (M/proc/proc.py:851-889): kp float64 [n][K][3]
// (K >= 7), centroid [n][2], angle_deg [n], length [n] -> flips, conf.
extern "C" int mdx_flips_from_keypoints(const double *kp, int64_t n, int K, const double *centroid,
                                        const double *angle_deg, const double *length, uint8_t *flips,
                                        double *conf) {
    MDX_REQUIRE(n >= 0 && K >= 7 && (n == 0 || (kp && centroid && angle_deg && length && flips && conf)),
                "mdx_flips_from_keypoints: bad arguments (K >= 7)");
    for (int64_t i = 0; i < n; ++i)
        flip_vote(kp + i * K * 3, K, centroid[2 * i], centroid[2 * i + 1], angle_deg[i], length[i], &flips[i], &conf[i]);
    return MDX_OK;
}

// The no-tracking angle step of instances_to_features (M/proc/proc.py:
// 720-724, 827-839): angle = clamp(-rad2deg(orientation)); keypoint flips
// with length = max(axis_length) add 180; iterative_filter_angles; final
// flips = keypoint flips xor filter flips.
extern "C" int mdx_finalize_angles(const double *orientation, const double *axis_length, const double *centroid,
                                   const double *kp, int64_t n, int K, double *angles_out, uint8_t *flips_out) {
    MDX_REQUIRE(n >= 0 && K >= 7 &&
                    (n == 0 || (orientation && axis_length && centroid && kp && angles_out && flips_out)),
                "mdx_finalize_angles: bad arguments (K >= 7)");
    if (n == 0) return MDX_OK;
    std::vector<double> ang(n);
    std::vector<uint8_t> kflip(n), fflip(n);
    for (int64_t i = 0; i < n; ++i) {
        const double a0 = axis_length[2 * i], a1 = axis_length[2 * i + 1];
        const double len = (std::isnan(a0) || std::isnan(a1)) ? NAN : (a0 > a1 ? a0 : a1);  // np.max
        double a = clamp_deg(-(orientation[i] * (180.0 / PI_)));  // np.rad2deg
        double conf;
        flip_vote(kp + i * K * 3, K, centroid[2 * i], centroid[2 * i + 1], a, len, &kflip[i], &conf);
        if (kflip[i]) a += 180;
        ang[i] = a;
    }
    const int rc = mdx_iterative_filter_angles(ang.data(), n, 3, 60.0, 1000, angles_out, fflip.data());
    if (rc != MDX_OK) return rc;
    for (int64_t i = 0; i < n; ++i) flips_out[i] = kflip[i] ^ fflip[i];
    return MDX_OK;
}
