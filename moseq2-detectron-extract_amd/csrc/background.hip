// Session background: get_bground_im, M/proc/roi.py:293-307
//
//   for every sampled frame: cv2.medianBlur(frame, med_scale)   (int16,
//                            BORDER_REPLICATE, med_scale 3 or 5)
//   bground = np.median(frames, axis=0)                         (float64)
//
// k_bg_blur     one thread per output pixel, the (2R+1)^2 window read with
//               clamped (= replicated) indices; the median by rank counting.
// k_bg_tmedian  one thread per pixel, the temporal median by an MSB-first
//               radix select over the 16-bit keys (v ^ 0x8000): 16 passes over
//               the pixel's column of n blurred frames, both middle order
//               statistics selected in the same passes (even n averages
//               them in double, as np.median does).
// Algorithmic bytes: read 2 B/pixel/frame (+ the blurred copy written and
// re-read 16 times, L2/MALL-resident for the reference's ~1 frame in 500);
// write 8 B/pixel.  Integer work, bit-exact.
#include <cmath>

#include "common.h"

namespace mdx {

constexpr int BG_TX = 64, BG_TY = 4;

template <int R>
__global__ __launch_bounds__(BG_TX *BG_TY) void k_bg_blur(const int16_t *__restrict__ src, int H, int W,
                                                          int16_t *__restrict__ dst) {
    constexpr int D = 2 * R + 1, N = D * D, MID = N / 2;
    const int x = blockIdx.x * BG_TX + threadIdx.x;
    const int y = blockIdx.y * BG_TY + threadIdx.y;
    const int64_t plane = (int64_t)H * W;
    const int16_t *f = src + (int64_t)blockIdx.z * plane;
    if (x >= W || y >= H) return;
    int v[N];
#pragma unroll
    for (int dy = 0; dy < D; ++dy) {
        const int yy = min(max(y + dy - R, 0), H - 1);
#pragma unroll
        for (int dx = 0; dx < D; ++dx) {
            const int xx = min(max(x + dx - R, 0), W - 1);
            v[dy * D + dx] = f[(int64_t)yy * W + xx];
        }
    }
    int med = v[0];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        int lt = 0, le = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            lt += v[j] < v[i];
            le += v[j] <= v[i];
        }
        if (lt <= MID && le > MID) med = v[i];
    }
    dst[(int64_t)blockIdx.z * plane + (int64_t)y * W + x] = (int16_t)med;
}

__global__ __launch_bounds__(256) void k_bg_tmedian(const int16_t *__restrict__ frames, int64_t n, int64_t plane,
                                                    double *__restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= plane) return;
    if (n == 0) {
        out[p] = NAN;
        return;
    }
    const int16_t *col = frames + p;
    int64_t r1 = (n - 1) / 2, r2 = n / 2;  // wanted ranks (0-based)
    uint32_t p1 = 0, p2 = 0;                // selected key prefixes
    for (int bit = 15; bit >= 0; --bit) {
        const uint32_t hi = (0xFFFFu << (bit + 1)) & 0xFFFFu;
        int64_t c1 = 0, c2 = 0;
        for (int64_t f = 0; f < n; ++f) {
            const uint32_t key = (uint32_t)(uint16_t)col[f * plane] ^ 0x8000u;
            const bool zero = ((key >> bit) & 1u) == 0u;
            c1 += (zero && (key & hi) == p1);
            c2 += (zero && (key & hi) == p2);
        }
        if (r1 >= c1) {
            r1 -= c1;
            p1 |= 1u << bit;
        }
        if (r2 >= c2) {
            r2 -= c2;
            p2 |= 1u << bit;
        }
    }
    const double a = (double)(int16_t)(uint16_t)(p1 ^ 0x8000u);
    const double b = (double)(int16_t)(uint16_t)(p2 ^ 0x8000u);
    out[p] = (n & 1) ? a : (a + b) / 2.0;
}

}  // namespace mdx

using namespace mdx;

extern "C" int mdx_bground_median(const int16_t *frames, int64_t n, int H, int W, int med_scale, int16_t *work,
                                  double *out, mdx_stream_t stream) {
    MDX_REQUIRE(out && H > 0 && W > 0 && n >= 0, "mdx_bground_median: bad arguments");
    MDX_REQUIRE(med_scale == 3 || med_scale == 5, "mdx_bground_median: med_scale must be 3 or 5 (got %d)", med_scale);
    MDX_REQUIRE(n == 0 || (frames && work), "mdx_bground_median: null frames / workspace");
    MDX_REQUIRE(n <= 65535, "mdx_bground_median: at most 65535 frames (got %lld)", (long long)n);
    hipStream_t s = as_stream(stream);
    const int64_t plane = (int64_t)H * W;
    if (n > 0) {
        dim3 grid((unsigned)ceil_div(W, BG_TX), (unsigned)ceil_div(H, BG_TY), (unsigned)n);
        if (med_scale == 5)
            hipLaunchKernelGGL(k_bg_blur<2>, grid, dim3(BG_TX, BG_TY), 0, s, frames, H, W, work);
        else
            hipLaunchKernelGGL(k_bg_blur<1>, grid, dim3(BG_TX, BG_TY), 0, s, frames, H, W, work);
        MDX_CHECK_LAUNCH("mdx_bground_median(blur)");
    }
    hipLaunchKernelGGL(k_bg_tmedian, dim3((unsigned)ceil_div(plane, 256)), dim3(256), 0, s, work, n, plane, out);
    MDX_CHECK_LAUNCH("mdx_bground_median(temporal)");
    return MDX_OK;
}
