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
