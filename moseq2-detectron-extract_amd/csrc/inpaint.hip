// fill_invalid_pixels -> cv2.inpaint(frame, invalid, 3, cv2.INPAINT_NS)
// (M/proc/proc.py:189-210; OpenCV imgproc/inpaint.cpp icvNSInpaintFMM as
// restated in oracle/frameops.c orc_inpaint_ns_one).
//
// One wavefront per frame.  The fast-marching order is inherently serial per
// frame, so the frame axis carries the parallelism (a 1000-frame chunk keeps
// ~1000 waves in flight); inside a frame the 64 lanes evaluate the (2r+1)^2
// window taps of one pixel in parallel and lane 0 folds them in the
// reference's k-major/l-minor order (float adds are not reassociated).
//
// Priority queue: OpenCV's sorted list pops by (T, insertion order).  The
// initial narrow band is pushed in raster order with T = 0 and every later
// push has T >= 0.5, so the band drains first, in raster order: it is kept as
// a FIFO array; later pushes go to a binary min-heap on (T, seq) in LDS (or in
// global workspace when a frame has more unknown pixels than LDS holds).
#include <cmath>

#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

constexpr int INP_KNOWN = 0, INP_BAND = 1, INP_INSIDE = 2;
constexpr int INP_LDS_HEAP = 3072;  // entries (12 B each)

struct HEnt {
    float T;
    int seq;
    int idx;
};

__device__ __forceinline__ bool hless(const HEnt &a, const HEnt &b) {
    return a.T < b.T || (a.T == b.T && a.seq < b.seq);
}

__device__ void heap_push(HEnt *h, int &n, HEnt e) {
    int k = n++;
    while (k > 0) {
        const int p = (k - 1) >> 1;
        if (!hless(e, h[p])) break;
        h[k] = h[p];
        k = p;
    }
    h[k] = e;
}

__device__ HEnt heap_pop(HEnt *h, int &n) {
    const HEnt top = h[0];
    const HEnt e = h[--n];
    int k = 0;
    for (;;) {
        int c = 2 * k + 1;
        if (c >= n) break;
        if (c + 1 < n && hless(h[c + 1], h[c])) ++c;
        if (!hless(h[c], e)) break;
        h[k] = h[c];
        k = c;
    }
    if (n > 0) h[k] = e;
    return top;
}

__device__ __forceinline__ float fm_solve(int i1, int j1, int i2, int j2, const uint8_t *f, const float *t, int PW) {
    double sol;
    const double a11 = t[i1 * PW + j1], a22 = t[i2 * PW + j2];
    const double m12 = a11 < a22 ? a11 : a22;
    if (f[i1 * PW + j1] != INP_INSIDE) {
        if (f[i2 * PW + j2] != INP_INSIDE) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt((double)(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else
            sol = 1 + a11;
    } else if (f[i2 * PW + j2] != INP_INSIDE)
        sol = 1 + a22;
    else
        sol = 1 + m12;
    return (float)sol;
}

__device__ __forceinline__ float min4f(float a, float b, float c, float d) {
    const float x = a < b ? a : b, y = c < d ? c : d;
    return x < y ? x : y;
}

static inline int64_t inp_frame_bytes(int H, int W) {
    const int64_t np = (int64_t)(H + 2) * (W + 2);
    const int64_t fb = (np + 15) / 16 * 16;
    return fb + 4 * np + (int64_t)sizeof(HEnt) * np + 16;
}

__global__ __launch_bounds__(64) void k_inpaint(uint8_t *__restrict__ frames, const uint8_t *__restrict__ invalid,
                                                int H, int W, int range, uint8_t *__restrict__ ws,
                                                int64_t ws_per_frame) {
    __shared__ HEnt s_heap[INP_LDS_HEAP];
    __shared__ int s_cnt[2];
    __shared__ float s_w[64], s_wv[64];
    const int lane = threadIdx.x;
    const int64_t fidx = blockIdx.x;
    uint8_t *out = frames + fidx * (int64_t)H * W;
    const uint8_t *msk = invalid + fidx * (int64_t)H * W;
    const int PH = H + 2, PW = W + 2;
    const int64_t np = (int64_t)PH * PW;
    uint8_t *base = ws + fidx * ws_per_frame;
    uint8_t *f = base;
    float *t = reinterpret_cast<float *>(base + (np + 15) / 16 * 16);
    HEnt *fifo = reinterpret_cast<HEnt *>(t + np);  // band FIFO, then global heap storage

    // any unknown pixel at all?  (inpaint is a no-op otherwise)
    int any = 0;
    for (int64_t i = lane; i < (int64_t)H * W; i += 64) any |= msk[i] != 0;
    if (!__any(any)) return;

    for (int64_t i = lane; i < np; i += 64) {
        const int y = (int)(i / PW), x = (int)(i - (int64_t)y * PW);
        const bool in = y >= 1 && y <= H && x >= 1 && x <= W && msk[(int64_t)(y - 1) * W + x - 1] != 0;
        f[i] = in ? INP_INSIDE : INP_KNOWN;
        t[i] = 1.0e6f;
    }
    __syncthreads();
    // narrow band = dilate(mask, cross) - mask on the interior, raster order
    int nband = 0, ninside = 0;
    for (int64_t i0 = 0; i0 < np; i0 += 64) {
        const int64_t i = i0 + lane;
        bool band = false;
        if (i < np) {
            const int y = (int)(i / PW), x = (int)(i - (int64_t)y * PW);
            if (y >= 1 && y < PH - 1 && x >= 1 && x < PW - 1) {
                if (f[i] == INP_INSIDE) {
                    ++ninside;
                } else {
                    band = f[i - 1] == INP_INSIDE || f[i + 1] == INP_INSIDE || f[i - PW] == INP_INSIDE ||
                           f[i + PW] == INP_INSIDE;
                }
            }
        }
        const unsigned long long bal = __ballot(band);
        if (band) {
            const int pos = nband + __popcll(bal & ((1ull << lane) - 1ull));
            fifo[pos] = HEnt{0.0f, pos, (int)i};
        }
        nband += __popcll(bal);
    }
    // ninside is per-lane: reduce
    for (int o = 32; o > 0; o >>= 1) ninside += __shfl_xor(ninside, o);
    __syncthreads();
    for (int k = lane; k < nband; k += 64) {
        const int i = fifo[k].idx;
        f[i] = INP_BAND;
        t[i] = 0.0f;
    }
    const bool lds_heap = ninside <= INP_LDS_HEAP;
    HEnt *heap = lds_heap ? s_heap : fifo + nband;
    int heap_n = 0, head = 0, seq = nband;
    __syncthreads();

    const int wsz = 2 * range + 1;
    for (;;) {
        // pop: FIFO (T = 0) first, then the heap
        int idx = -1;
        if (lane == 0) {
            if (head < nband)
                idx = fifo[head++].idx;
            else if (heap_n > 0)
                idx = heap_pop(heap, heap_n).idx;
        }
        idx = __shfl(idx, 0);
        if (idx < 0) break;
        const int ii = idx / PW, jj = idx - ii * PW;
        if (lane == 0) f[idx] = INP_KNOWN;
        __syncthreads();
        for (int q = 0; q < 4; ++q) {
            int i, j;
            if (q == 0) { i = ii - 1; j = jj; }
            else if (q == 1) { i = ii; j = jj - 1; }
            else if (q == 2) { i = ii + 1; j = jj; }
            else { i = ii; j = jj + 1; }
            if (i <= 1 || j <= 1 || i > PH - 1 || j > PW - 1) continue;
            if (f[i * PW + j] != INP_INSIDE) continue;
            const float dist = min4f(fm_solve(i - 1, j, i, j - 1, f, t, PW), fm_solve(i + 1, j, i, j - 1, f, t, PW),
                                     fm_solve(i - 1, j, i, j + 1, f, t, PW), fm_solve(i + 1, j, i, j + 1, f, t, PW));
            // window taps, one per lane (range <= 3)
            float w = 0.0f, wv = 0.0f;
            bool valid = false;
            if (lane < wsz * wsz) {
                const int k = i - range + lane / wsz, l = j - range + lane % wsz;
                const int km = k - 1 + (k == 1), kp = k - 1 - (k == PH - 2);
                const int lm = l - 1 + (l == 1), lp = l - 1 - (l == PW - 2);
                if (k > 0 && l > 0 && k < PH - 1 && l < PW - 1 && f[k * PW + l] != INP_INSIDE &&
                    (l - j) * (l - j) + (k - i) * (k - i) <= range * range) {
                    valid = true;
                    const float ry = (float)(k - i), rx = (float)(l - j);
                    const float lr = rx * rx + ry * ry;
                    const float dst = (float)(1. / (lr * sqrt((double)lr)));
                    const bool up_ok = f[(k - 1) * PW + l] != INP_INSIDE, dn_ok = f[(k + 1) * PW + l] != INP_INSIDE;
                    const bool lf_ok = f[k * PW + l - 1] != INP_INSIDE, rt_ok = f[k * PW + l + 1] != INP_INSIDE;
                    float gx, gy;
                    if (dn_ok) {
                        if (up_ok)
                            gx = (float)(abs(out[(kp + 1) * W + lm] - out[kp * W + lm]) +
                                         abs(out[kp * W + lm] - out[(km - 1) * W + lm]));
                        else
                            gx = (float)(abs(out[(kp + 1) * W + lm] - out[kp * W + lm])) * 2.0f;
                    } else {
                        if (up_ok)
                            gx = (float)(abs(out[kp * W + lm] - out[(km - 1) * W + lm])) * 2.0f;
                        else
                            gx = 0;
                    }
                    if (rt_ok) {
                        if (lf_ok)
                            gy = -(float)(abs(out[km * W + lp + 1] - out[km * W + lm]) +
                                          abs(out[km * W + lm] - out[km * W + lm - 1]));
                        else
                            gy = -(float)(abs(out[km * W + lp + 1] - out[km * W + lm])) * 2.0f;
                    } else {
                        if (lf_ok)
                            gy = -(float)(abs(out[km * W + lm] - out[km * W + lm - 1])) * 2.0f;
                        else
                            gy = 0;
                    }
                    const float dot = rx * gx + ry * gy;
                    const float lg = gx * gx + gy * gy;
                    float dir = fabsf(dot / sqrtf(lr * lg));
                    if (!(dir > 0.01f)) dir = 0.000001f;
                    w = dst * dir;
                    wv = w * (float)out[km * W + lm];
                }
            }
            s_w[lane] = valid ? w : 0.0f;
            s_wv[lane] = valid ? wv : -1.0f;  // -1 marks a skipped tap
            __syncthreads();
            if (lane == 0) {
                float Ia = 0.0f, s = 1.0e-20f;
                for (int L = 0; L < wsz * wsz; ++L) {
                    if (s_wv[L] < 0.0f) continue;
                    Ia += s_wv[L];
                    s += s_w[L];
                }
                const double v = (double)Ia / s;
                const int r = __double2int_rn(v);
                out[(i - 1) * W + (j - 1)] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
                t[i * PW + j] = dist;
                f[i * PW + j] = INP_BAND;
                heap_push(heap, heap_n, HEnt{dist, seq++, i * PW + j});
            }
            __syncthreads();
        }
    }
}

}  // namespace mdx

using namespace mdx;

extern "C" int64_t mdx_inpaint_workspace_bytes(int64_t n, int H, int W) {
    if (n <= 0 || H <= 0 || W <= 0) return 0;
    return n * inp_frame_bytes(H, W);
}

extern "C" int mdx_inpaint_ns(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                              void *workspace, mdx_stream_t stream) {
    MDX_REQUIRE(frames && invalid, "mdx_inpaint_ns: null frames/invalid");
    MDX_REQUIRE(radius >= 0 && radius <= 3, "mdx_inpaint_ns: radius must be in [0, 3] (got %d)", radius);
    MDX_REQUIRE(H > 0 && W > 0, "mdx_inpaint_ns: bad shape");
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(workspace != nullptr, "mdx_inpaint_ns: null workspace");
    MDX_REQUIRE((int64_t)(H + 2) * (W + 2) < (1ll << 31), "mdx_inpaint_ns: frame too large");
    MDX_REQUIRE(n <= 0x7fffffff, "mdx_inpaint_ns: n too large");
    hipLaunchKernelGGL(k_inpaint, dim3((unsigned)n), dim3(64), 0, as_stream(stream), frames, invalid, H, W, radius,
                       (uint8_t *)workspace, inp_frame_bytes(H, W));
    MDX_CHECK_LAUNCH("mdx_inpaint_ns");
    return MDX_OK;
}
