// Frame-op kernels of the extraction hot path (gfx950).
//
//   k_prep        prep_raw_frames numpy part      M/proc/proc.py:129-186, M/proc/roi.py:215-254
//   k_scale       scale_raw_frames (256-entry LUT) M/proc/proc.py:214-234
//   k_clean       clean_frames: medianBlur(3) + morphologyEx(OPEN, strel, iters),
//                 all passes fused per LDS tile    M/proc/proc.py:480-515
//   k_moments     get_frame_features + im_moment_features
//                 (largest contour, polygon moments) M/proc/proc.py:237-302,518-549
//   k_crop        crop_and_rotate_frame (warpAffine INTER_LINEAR fixed point)
//                                                  M/proc/proc.py:305-340
//
// All double/float arithmetic that the reference performs in a fixed order is
// written in that order with FMA contraction disabled, so results are
// bit-identical to the oracle (oracle/frameops.c).
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

// ---------------------------------------------------------------------------
// prep
// ---------------------------------------------------------------------------
constexpr int PREP_FRAMES_PER_BLOCK = 32;

// One thread per cropped pixel (256 consecutive pixels per workgroup) and up
// to 32 frames, loaded 8 at a time (the background and ROI read once per 32
// frames); grid (ceil(oh * ow / 256), ceil(n / 32)).  bits (or null): the
// inpaint workspace's bit images, zero at rest: each invalid pixel ORs its bit
// (padded row y + 1, bit x + 1 of the row's wpr words).
__global__ __launch_bounds__(256) void k_prep(const int16_t *__restrict__ raw, int64_t n, int H, int W,
                                              const double *__restrict__ bg, const uint8_t *__restrict__ roi,
                                              int y0, int x0, int oh, int ow, int flags, double vmin,
                                              double vmax, uint8_t *__restrict__ out, uint8_t *__restrict__ inv,
                                              uint32_t *__restrict__ bits, int64_t bits_fstride, int wpr) {
    const int64_t npix = (int64_t)oh * ow;
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    const int y = (int)(p / ow), x = (int)(p - (int64_t)y * ow);
    const int64_t si = (int64_t)(y + y0) * W + x + x0;
    const double b = bg ? bg[si] : 0.0;
    const uint8_t r8 = roi ? roi[si] : (uint8_t)1;
    const int64_t f0 = (int64_t)blockIdx.y * PREP_FRAMES_PER_BLOCK;
    const int nf = (int)(n - f0 < PREP_FRAMES_PER_BLOCK ? n - f0 : PREP_FRAMES_PER_BLOCK);
    const int64_t fstride = (int64_t)H * W;
    const int16_t *rp = raw + f0 * fstride + si;
    uint32_t *bp = bits ? bits + f0 * bits_fstride + (int64_t)(y + 1) * wpr + ((x + 1) >> 5) : nullptr;
    const uint32_t bit = 1u << ((x + 1) & 31);
    for (int u0 = 0; u0 < nf; u0 += 8) {
        int16_t r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = u0 + u < nf ? rp[(int64_t)(u0 + u) * fstride] : (int16_t)1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (u0 + u >= nf) break;
            const int64_t f = f0 + u0 + u;
            double v = bg ? b - (double)r[u] : (double)r[u];  // bground_im - frames (float64)
            if (roi) v = v * (double)r8;                      // frames * roi
            if ((flags & 1) && v < vmin) v = 0.0;             // frames[frames < vmin] = 0
            if ((flags & 2) && v > vmax) v = vmax;            // frames[frames > vmax] = vmax
            out[f * npix + p] = (uint8_t)(int32_t)v;          // astype(uint8) (truncation)
            const bool invalid = r[u] == 0 && r8;
            if (inv) inv[f * npix + p] = (uint8_t)invalid;
            if (bp && invalid) atomicOr(bp + (int64_t)(u0 + u) * bits_fstride, bit);
        }
    }
}

int launch_prep(const int16_t *raw, int64_t n, int H, int W, const double *bg, const uint8_t *roi, int y0, int y1,
                int x0, int x1, int flags, double vmin, double vmax, uint8_t *out, uint8_t *invalid, uint32_t *bits,
                int64_t bits_fstride, int wpr, hipStream_t s) {
    const int oh = y1 - y0, ow = x1 - x0;
    dim3 grid((unsigned)ceil_div((int64_t)oh * ow, 256), (unsigned)ceil_div(n, PREP_FRAMES_PER_BLOCK));
    hipLaunchKernelGGL(k_prep, grid, dim3(256), 0, s, raw, n, H, W, bg, roi, y0, x0, oh, ow, flags, vmin, vmax, out,
                       invalid, bits, bits_fstride, wpr);
    MDX_CHECK_LAUNCH("mdx_prep_frames");
    return MDX_OK;
}

// ---------------------------------------------------------------------------
// scale LUT
// ---------------------------------------------------------------------------
struct Lut256 {
    uint8_t v[256];
};

__global__ __launch_bounds__(256) void k_scale(const uint8_t *__restrict__ in, int64_t count, Lut256 lut,
                                               uint8_t *__restrict__ out) {
    __shared__ uint8_t s_lut[256];
    s_lut[threadIdx.x] = lut.v[threadIdx.x];
    __syncthreads();
    const int64_t nvec = count / 16;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
        uint4 v = reinterpret_cast<const uint4 *>(in)[i];
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t o = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) o |= (uint32_t)s_lut[(w[k] >> (8 * b)) & 255] << (8 * b);
            w[k] = o;
        }
        reinterpret_cast<uint4 *>(out)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (blockIdx.x == 0)
        for (int64_t i = nvec * 16 + threadIdx.x; i < count; i += 256) out[i] = s_lut[in[i]];
}

// ---------------------------------------------------------------------------
// clean_frames: median3 (replicate border) -> erode^iters -> dilate^iters, one
// launch per pass over 64x32 output tiles (the frames stay in L2/MALL between
// passes; a fused multi-pass tile would recompute a 2*iters*rad halo).  Pixels
// outside the image read as the pass's neutral element (255 for an erosion, 0
// for a dilation) -- OpenCV's morphologyDefaultBorderValue, applied per pass.
// Morphology is done separably: per LDS row, the min/max over each distinct
// strel row span, then per output pixel the combine over the strel rows.
// ---------------------------------------------------------------------------
constexpr int CT_W = 64, CT_H = 32, CT_THREADS = 256, MAX_KH = 15;

struct StrelSpans {
    int kh, kw, ay, ax, nspan;
    int8_t j1[MAX_KH], j2[MAX_KH];    // row ky: ones in [j1, j2)
    int8_t sj1[MAX_KH], sj2[MAX_KH];  // distinct spans
    int8_t rspan[MAX_KH];             // row ky -> distinct span index (-1: empty row)
};

__device__ __forceinline__ int med9(int *v) {
#define MDX_S(a, c)               \
    {                             \
        int lo = min(v[a], v[c]); \
        int hi = max(v[a], v[c]); \
        v[a] = lo;                \
        v[c] = hi;                \
    }
    MDX_S(1, 2); MDX_S(4, 5); MDX_S(7, 8); MDX_S(0, 1); MDX_S(3, 4); MDX_S(6, 7);
    MDX_S(1, 2); MDX_S(4, 5); MDX_S(7, 8); MDX_S(0, 3); MDX_S(5, 8); MDX_S(4, 7);
    MDX_S(3, 6); MDX_S(1, 4); MDX_S(2, 5); MDX_S(4, 7); MDX_S(4, 2); MDX_S(6, 4);
    MDX_S(4, 2);
#undef MDX_S
    return v[4];
}

// medianBlur(3), BORDER_REPLICATE
__global__ __launch_bounds__(CT_THREADS) void k_median3(const uint8_t *__restrict__ src, int H, int W,
                                                        uint8_t *__restrict__ out, int tiles_x) {
    constexpr int LW = CT_W + 2, LH = CT_H + 2;
    __shared__ uint8_t A[LH * LW];
    const long long frame = blockIdx.y;
    const int x0 = (blockIdx.x % tiles_x) * CT_W, y0 = (blockIdx.x / tiles_x) * CT_H;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const uint8_t *s = src + frame * H * W;
    for (int ly = ty; ly < LH; ly += 4) {
        const int gy = min(max(y0 + ly - 1, 0), H - 1);
        for (int lx = tx; lx < LW; lx += 64) {
            const int gx = min(max(x0 + lx - 1, 0), W - 1);
            A[ly * LW + lx] = s[gy * W + gx];
        }
    }
    __syncthreads();
    uint8_t *o = out + frame * H * W;
    const int gx = x0 + tx;
    if (gx >= W) return;
#pragma unroll 2
    for (int r = 0; r < CT_H / 4; ++r) {
        const int y = ty * (CT_H / 4) + r, gy = y0 + y;
        if (gy >= H) break;
        int v[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) v[dy * 3 + dx] = A[(y + dy) * LW + tx + dx];
        o[gy * W + gx] = (uint8_t)med9(v);
    }
}

// one erosion (DIL = false) or dilation (DIL = true) pass.  Pixels are held
// as u16 in LDS so that two of them are combined per v_pk_min/max_u16; each
// lane owns 4 adjacent columns (two packed dwords).  The strel tables are
// copied to LDS once (kernarg arrays indexed at run time would be re-fetched
// with a scalar load per use).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <bool DIL>
__device__ __forceinline__ uint32_t pk_op(uint32_t a, uint32_t b) {
    const u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
    return __builtin_bit_cast(uint32_t, DIL ? __builtin_elementwise_max(x, y) : __builtin_elementwise_min(x, y));
}

constexpr int MP_MAXW = CT_W + MAX_KH + 1;  // u16 pixels per LDS row (even, 8-byte aligned rows)

template <bool DIL>
__global__ __launch_bounds__(CT_THREADS) void k_morph(const uint8_t *__restrict__ src, int H, int W, StrelSpans st,
                                                      uint8_t *__restrict__ out, int tiles_x) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int8_t s_sj1[MAX_KH], s_sj2[MAX_KH], s_rspan[MAX_KH];
    const int LW = CT_W + st.kw - 1, LH = CT_H + st.kh - 1;
    const int LP = (LW + 7) & ~3;                                 // u16 pitch (>= LW + 3, multiple of 4)
    uint16_t *A = reinterpret_cast<uint16_t *>(smem);             // [LH][LP]
    uint16_t *Hs = A + LH * LP;                                   // [nspan][LH][CT_W]
    const long long frame = blockIdx.y;
    const int x0 = (blockIdx.x % tiles_x) * CT_W, y0 = (blockIdx.x / tiles_x) * CT_H;
    const uint8_t *s = src + frame * H * W;
    const uint32_t neutral = DIL ? 0u : 255u;
    if (threadIdx.x < MAX_KH) {
        s_sj1[threadIdx.x] = st.sj1[threadIdx.x];
        s_sj2[threadIdx.x] = st.sj2[threadIdx.x];
        s_rspan[threadIdx.x] = st.rspan[threadIdx.x];
    }
    {
        const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
        for (int ly = ty; ly < LH; ly += 4) {
            const int gy = y0 + ly - st.ay;
            const bool yin = gy >= 0 && gy < H;
            for (int lx = tx; lx < LP; lx += 64) {
                const int gx = x0 + lx - st.ax;
                A[ly * LP + lx] = (uint16_t)((lx < LW && yin && gx >= 0 && gx < W) ? s[gy * W + gx] : neutral);
            }
        }
    }
    __syncthreads();
    const int g = threadIdx.x & 15, rg = threadIdx.x >> 4;  // column quad, row group
    const int nsp = st.nspan, kw = st.kw;
    // horizontal: per LDS row, span min/max for the 4 columns 4g..4g+3
    for (int ly = rg; ly < LH; ly += 16) {
        const uint32_t *row = reinterpret_cast<const uint32_t *>(A + ly * LP + 4 * g);
        uint32_t d[(MAX_KH + 3) / 2 + 1];
#pragma unroll
        for (int m = 0; m < (MAX_KH + 3) / 2 + 1; ++m)
            if (m <= (kw + 3) / 2) d[m] = row[m];
        for (int k = 0; k < nsp; ++k) {
            const int j1 = s_sj1[k], j2 = s_sj2[k];
            uint32_t a0 = DIL ? 0u : 0x00FF00FFu, a1 = a0;
#pragma unroll
            for (int kx = 0; kx < MAX_KH; ++kx) {
                if (kx < j1 || kx >= j2) continue;
                // pixels (kx, kx+1) and (kx+2, kx+3) relative to column 4g
                const uint32_t lo = (kx & 1) ? __builtin_amdgcn_alignbyte(d[kx / 2 + 1], d[kx / 2], 2) : d[kx / 2];
                const uint32_t hi =
                    (kx & 1) ? __builtin_amdgcn_alignbyte(d[kx / 2 + 2], d[kx / 2 + 1], 2) : d[kx / 2 + 1];
                a0 = pk_op<DIL>(a0, lo);
                a1 = pk_op<DIL>(a1, hi);
            }
            uint2 *hp = reinterpret_cast<uint2 *>(Hs + (k * LH + ly) * CT_W + 4 * g);
            *hp = make_uint2(a0, a1);
        }
    }
    __syncthreads();
    // vertical combine: rows 2*rg, 2*rg+1 of the output tile
    const int kh = st.kh;
    uint32_t acc[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) acc[r][0] = acc[r][1] = DIL ? 0u : 0x00FF00FFu;
    const int yb = 2 * rg;
    for (int ky = 0; ky < kh; ++ky) {
        const int k = s_rspan[ky];
        if (k < 0) continue;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint2 v = *reinterpret_cast<const uint2 *>(Hs + (k * LH + yb + r + ky) * CT_W + 4 * g);
            acc[r][0] = pk_op<DIL>(acc[r][0], v.x);
            acc[r][1] = pk_op<DIL>(acc[r][1], v.y);
        }
    }
    uint8_t *o = out + frame * H * W;
    const int gx = x0 + 4 * g;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int gy = y0 + yb + r;
        if (gy >= H || gx >= W) continue;
        const uint32_t packed = (acc[r][0] & 0xFFu) | ((acc[r][0] >> 8) & 0xFF00u) | ((acc[r][1] & 0xFFu) << 16) |
                                ((acc[r][1] << 8) & 0xFF000000u);
        if (gx + 4 <= W && (W & 3) == 0) {
            *reinterpret_cast<uint32_t *>(o + gy * W + gx) = packed;
        } else {
            for (int q = 0; q < 4 && gx + q < W; ++q) o[gy * W + gx + q] = (uint8_t)(packed >> (8 * q));
        }
    }
}

// ---------------------------------------------------------------------------
// clean_frames fused: the extract path's exact chain -- medianBlur(3)
// (replicate border), erode x3 and dilate x3 with the 9x9 ellipse (OpenCV's
// neutral border per pass) -- as ONE streaming kernel (M/proc/proc.py:480-515).
//
// One workgroup per (frame, strip of SW output columns) walks the frame from
// top to bottom, one row per step, as a 7-stage line-buffer pipeline: every
// stage consumes the row its predecessor produced in the previous step and
// emits one row, so each pixel of each pass is computed once (no vertical
// halo; the horizontal halo is the 25-column strip margin) and the frame is
// read once and written once.  Stage inputs travel through double-buffered
// LDS rows (u16 per pixel, one barrier per step); each stage's vertical
// window lives in registers (a 9-row ring, the step loop unrolled by 9).
//
//   stage 0 (waves MW..): median of the 3x3 window -- columns sorted with
//     v_min3 / v_med3 / v_max3, median = med3(max3(lows), med3(mids),
//     min3(highs)) (exact); these lanes also stream the raw rows in, 9
//     steps ahead (registers -> LDS).
//   stages 1..6 (waves 0..MW-1), 4 output columns per lane as two u16 pairs:
//     the ellipse rows are spans of half-width 0 / 3 / 4 (rows 0,8 / 1,2,6,7
//     / 3,4,5), so per input row the lane computes the three span minima
//     (v_pk_min_u16, shared between its two pairs) and per output row the
//     min over the 9 ring rows.  Dilation runs as erosion of the inverted
//     image (max(a,b) = 255 - min(255-a, 255-b)): stage 3 writes 255 - v, the
//     last stage inverts back, so all six stages share one instruction stream
//     and one neutral value (255) for pixels outside the frame.
// Rows / columns outside the frame are written as the neutral value, which
// is exactly OpenCV's per-pass border handling.
// ---------------------------------------------------------------------------
template <int SW>
struct CleanStream {
    static constexpr int E(int s) { return 4 * (6 - s); }            // stage s: extra columns each side
    static constexpr int NQ(int s) { return SW / 4 + E(s) / 2; }      // quads (4 columns) of stage s
    static constexpr int MORPH_LANES = 6 * (SW / 4) + 30;              // stages 1..6
    static constexpr int MW = (MORPH_LANES + 63) / 64;                 // morph waves
    static constexpr int DW = (NQ(0) + 63) / 64;                       // median / loader waves
    static constexpr int THREADS = 64 * (MW + DW);
    static constexpr int PU = SW + 64;                                 // u16 per LDS row
    static constexpr int PB = SW + 64;                                 // raw bytes per LDS row
    static constexpr int RAWB = SW + 50;                               // raw columns per row: X0-25 .. X0+SW+24
    static constexpr int LB = (RAWB + 64 * DW - 1) / (64 * DW);        // raw bytes per loader lane per row
    // step t: the median consumes raw row t - 26 and emits row t - 27; stage
    // s >= 1 consumes row t - IN(s) and emits row t - OUT(s)
    static constexpr int IN(int s) { return 28 + 5 * (s - 1); }
    static constexpr int OUT(int s) { return IN(s) + 4; }
};

__device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b) { return pk_op<false>(a, b); }
// 3-input minimum of u16 pairs held as 0x6400 + v (v <= 255): those halves
// are the normal f16 values 1024 + v, ordered as their integers, so the f16
// minimum is the integer minimum (one instruction for two pmin)
__device__ __forceinline__ uint32_t pmin3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// one VALU instruction each (written out: the compiler shares min(a, b)
// between a min3 and a med3 of the same operands and then emits neither)
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

template <int SW>
__global__ __launch_bounds__(CleanStream<SW>::THREADS) void k_clean_stream(const uint8_t *__restrict__ src, int H,
                                                                             int W, int strips,
                                                                             uint8_t *__restrict__ out) {
    using C = CleanStream<SW>;
    __shared__ __attribute__((aligned(16))) uint16_t stg[6][2][C::PU];  // stage 0..5 outputs, by step parity
    __shared__ __attribute__((aligned(16))) uint8_t raw[9][C::PB];      // raw rows of the current 9-step block
    const long long frame = blockIdx.x / strips;
    const int X0 = (int)(blockIdx.x % strips) * SW, BX = X0 - 28;      // LDS column 0 = image column BX
    const uint8_t *s = src + frame * H * W;
    uint8_t *o = out + frame * H * W;
    const int tid = threadIdx.x, wave = tid >> 6;
    const bool med = wave >= C::MW;
    const int NSTEP = H + C::OUT(6) + 1;
    // stage rows hold each pixel v as 0x6400 + v (pmin3); the neutral value
    // is 255, dilation works on 255 - v = v ^ 0xFF
    constexpr uint32_t FH = 0x64006400u, NEUT = 0x64FF64FFu, INVX = 0x00FF00FFu;

    // ---- per-lane role ----
    int stage = 0, q = -1, x0 = 0;
    if (!med) {
        int l = tid, st = 1;
        while (st <= 6 && l >= C::NQ(st)) l -= C::NQ(st++);
        if (st <= 6) {
            stage = st;
            q = l;
            x0 = X0 - C::E(st) + 4 * l;
        }
    } else {
        const int l = tid - 64 * C::MW;
        if (l < C::NQ(0)) {
            q = l;
            x0 = X0 - C::E(0) + 4 * l;
        }
    }
    // outside-column masks of this lane's two pairs (0xFF in the outside halves)
    uint32_t cm[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int c0 = x0 + 2 * p, c1 = c0 + 1;
        cm[p] = ((c0 < 0 || c0 >= W) ? 0xFFu : 0u) | ((c1 < 0 || c1 >= W) ? 0xFF0000u : 0u);
    }
    bool cok[4];  // this lane's output columns inside the frame
#pragma unroll
    for (int c = 0; c < 4; ++c) cok[c] = x0 + c >= 0 && x0 + c < W;
    const uint32_t inv = stage == 3 || stage == 6 ? INVX : 0u;  // dilation: work on 255 - v
    const int idx = x0 - BX;                                      // u16 / byte column of this lane's quad
    const int out_off = stage >= 1 ? C::OUT(stage) : 27;

    // ---- register file shared by the two roles (one array, so the compiler
    // allocates it once): morph lanes hold their 9-row ring of span minima
    // (slot k: R[6k .. 6k+5] = span-0 pair 0/1, span-3 pair 0/1, span-4 pair
    // 0/1); median lanes hold their 3-row window of raw columns (R[0..17]) ----
    uint32_t R[54];
#pragma unroll
    for (int k = 0; k < 54; ++k) R[k] = NEUT;
#define MV(kk, c) R[(kk) * 6 + (c)]
#define R0(k, p) R[(k) * 6 + (p)]
#define R3(k, p) R[(k) * 6 + 2 + (p)]
#define R4(k, p) R[(k) * 6 + 4 + (p)]
    const int ll = tid - 64 * C::MW;
    uint32_t s3p[2] = {NEUT, NEUT};  // morph lanes: the previous input row's span-3 minima
    // raw rows stream in a 9-step block ahead: at the start of block b the
    // median lanes store block b's 9 rows (loaded at the start of block b-1)
    // into LDS and load block b+1's into registers of their own (not shared
    // with the ring: no wait on these loads anywhere but the next block's
    // store, 9 steps later).  Columns past the strip read a clamped, valid
    // byte that the store skips.
    uint32_t qv[9][C::LB];
    auto load_row = [&](int k, int r) {
        const int gy = min(max(r, 0), H - 1);
#pragma unroll
        for (int m = 0; m < C::LB; ++m) {
            const int c = ll + 64 * C::DW * m;
            const int gx = min(max(BX + 3 + c, 0), W - 1);
            qv[k][m] = (uint32_t)s[(long long)gy * W + gx];
        }
    };
    if (med) {
#pragma unroll
        for (int k = 0; k < 9; ++k) load_row(k, k - 26);  // block 0: steps 0..8 consume raw rows -26 .. -18
#pragma unroll
        for (int k = 0; k < 18; ++k) R[k] = 255u;
    }

    for (int t0 = 0; t0 < NSTEP; t0 += 9) {
        if (med) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
#pragma unroll
                for (int m = 0; m < C::LB; ++m) {
                    const int c = ll + 64 * C::DW * m;
                    if (c < C::RAWB) raw[k][3 + c] = (uint8_t)qv[k][m];
                }
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) load_row(k, t0 + 9 + k - 26);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int t = t0 + k;
            if (t >= NSTEP) continue;  // uniform (no break: the ring indices must stay compile-time)
            const int rd = (t - 1) & 1, wr = t & 1;
            if (med) {
                if (q >= 0) {
                    const uint32_t *rw = reinterpret_cast<const uint32_t *>(raw[k]);  // raw row t - 26
                    const uint32_t d0 = rw[idx / 4 - 1], d1 = rw[idx / 4], d2 = rw[idx / 4 + 1];
                    const int kk = k % 3;
                    MV(kk, 0) = d0 >> 24;
                    MV(kk, 1) = d1 & 255u;
                    MV(kk, 2) = (d1 >> 8) & 255u;
                    MV(kk, 3) = (d1 >> 16) & 255u;
                    MV(kk, 4) = d1 >> 24;
                    MV(kk, 5) = d2 & 255u;
                    uint32_t lo[6], mi[6], hi[6];
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        lo[c] = umin3(MV(0, c), MV(1, c), MV(2, c));
                        mi[c] = umed3(MV(0, c), MV(1, c), MV(2, c));
                        hi[c] = umax3(MV(0, c), MV(1, c), MV(2, c));
                    }
                    uint32_t m4[4];
#pragma unroll
                    for (int p = 0; p < 4; ++p)
                        m4[p] = umed3(umax3(lo[p], lo[p + 1], lo[p + 2]), umed3(mi[p], mi[p + 1], mi[p + 2]),
                                      umin3(hi[p], hi[p + 1], hi[p + 2]));
                    const int row = t - out_off;
                    uint32_t a = m4[0] | (m4[1] << 16) | FH, b = m4[2] | (m4[3] << 16) | FH;
                    if (row < 0 || row >= H) {
                        a = b = NEUT;
                    } else {
                        a |= cm[0];
                        b |= cm[1];
                    }
                    *reinterpret_cast<uint2 *>(&stg[0][wr][idx]) = make_uint2(a, b);
                }
            } else if (q >= 0) {
                const uint16_t *in = stg[stage - 1][rd];
                const uint2 u0 = *reinterpret_cast<const uint2 *>(in + idx - 4);
                const uint2 u1 = *reinterpret_cast<const uint2 *>(in + idx);
                const uint2 u2 = *reinterpret_cast<const uint2 *>(in + idx + 4);
                // pairs (x + s, x + s + 1) for s = -4 .. 6
                const uint32_t qm4 = u0.x, qm2 = u0.y, q0 = u1.x, q2 = u1.y, q4 = u2.x, q6 = u2.y;
                const uint32_t qm3 = __builtin_amdgcn_alignbyte(qm2, qm4, 2);
                const uint32_t qm1 = __builtin_amdgcn_alignbyte(q0, qm2, 2);
                const uint32_t q1 = __builtin_amdgcn_alignbyte(q2, q0, 2);
                const uint32_t q3 = __builtin_amdgcn_alignbyte(q4, q2, 2);
                const uint32_t q5 = __builtin_amdgcn_alignbyte(q6, q4, 2);
                const uint32_t u = pmin3(pmin3(qm1, q0, q1), q2, q3);
                const uint32_t s3a = pmin3(u, qm3, qm2), s3b = pmin3(u, q4, q5);
                // the ring keeps, per row r, the span-3 minimum of rows r-1 and r
                // (the ellipse's half-width-3 rows come in adjacent pairs)
                R3(k, 0) = pmin(s3a, s3p[0]);
                R3(k, 1) = pmin(s3b, s3p[1]);
                s3p[0] = s3a;
                s3p[1] = s3b;
                R4(k, 0) = pmin3(s3a, qm4, q4);
                R4(k, 1) = pmin3(s3b, qm2, q6);
                R0(k, 0) = q0;
                R0(k, 1) = q2;
                // ellipse rows 0..8 of the output row = ring slots k+1 .. k+9:
                // row 0 span 0, rows 1-2 (pair at slot k+3), rows 3-5 span 4,
                // rows 6-7 (pair at slot k+8), row 8 span 0
                uint32_t v[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    v[p] = pmin3(pmin3(R0((k + 1) % 9, p), R0(k, p), R3((k + 3) % 9, p)),
                                 pmin3(R3((k + 8) % 9, p), R4((k + 4) % 9, p), R4((k + 5) % 9, p)),
                                 R4((k + 6) % 9, p));
                }
                const int row = t - out_off;
                if (stage < 6) {
                    uint32_t a = (v[0] ^ inv) | cm[0], b = (v[1] ^ inv) | cm[1];
                    if (row < 0 || row >= H) a = b = NEUT;
                    *reinterpret_cast<uint2 *>(&stg[stage][wr][idx]) = make_uint2(a, b);
                } else if (row >= 0 && row < H) {
                    const uint32_t a = v[0] ^ inv, b = v[1] ^ inv;
                    uint8_t *dst = o + (long long)row * W + x0;
                    // byte stores (rows of an odd-width frame are not 4-B aligned)
                    if (cok[0]) dst[0] = (uint8_t)a;
                    if (cok[1]) dst[1] = (uint8_t)(a >> 16);
                    if (cok[2]) dst[2] = (uint8_t)b;
                    if (cok[3]) dst[3] = (uint8_t)(b >> 16);
                }
            }
            __syncthreads();
        }
    }
#undef MV
#undef R0
#undef R3
#undef R4
}

// the ellipse 9x9 (cv2.getStructuringElement(MORPH_ELLIPSE, (9, 9))) row spans
// the fused kernel hard-codes
__host__ inline bool is_ellipse9(const uint8_t *strel, int kh, int kw) {
    static const int hw[9] = {0, 3, 3, 4, 4, 4, 3, 3, 0};
    if (kh != 9 || kw != 9) return false;
    for (int r = 0; r < 9; ++r)
        for (int c = 0; c < 9; ++c)
            if ((strel[r * 9 + c] != 0) != (c >= 4 - hw[r] && c <= 4 + hw[r])) return false;
    return true;
}

// ---------------------------------------------------------------------------
// moments: one workgroup per frame.
// The blob mask (frame > thr) & mask is bit-packed into LDS with a 1-pixel
// zero frame (findContours pads the image with zeros).  Every pixel that can
// start the outer border of its 8-connected blob (fg, with W, NW, N, NE all
// background; the raster-first pixel of every blob qualifies) is traced with
// the Suzuki85 outer-border follower, accumulating the Green's-theorem sums of
// cv::contourMoments in int64 (exact, so trace order does not matter).  The
// largest |a00| wins (contourArea argmax; ties -> raster-first start, which is
// the reference's first blob in scan order).  Traces started inside a hole
// produce hole borders whose area never exceeds their blob's outer border.
// ---------------------------------------------------------------------------
constexpr int MOM_THREADS = 1024;

struct Green {
    long long a00, a10, a01, a20, a11, a02;
};

__device__ __forceinline__ void green_edge(Green &g, long long xi_1, long long yi_1, long long xi, long long yi) {
    const long long xi2 = xi * xi, yi2 = yi * yi;
    const long long dxy = xi_1 * yi - xi * yi_1;
    const long long xii_1 = xi_1 + xi, yii_1 = yi_1 + yi;
    g.a00 += dxy;
    g.a10 += dxy * xii_1;
    g.a01 += dxy * yii_1;
    g.a20 += dxy * (xi_1 * xii_1 + xi2);
    g.a11 += dxy * (xi_1 * (yii_1 + yi_1) + xi * (yii_1 + yi));
    g.a02 += dxy * (yi_1 * yii_1 + yi2);
}

// direction d: 0 E, 1 NE, 2 N, 3 NW, 4 W, 5 SW, 6 S, 7 SE (y grows down);
// (dx + 1, dy + 1) packed 2 bits per direction so a lane-varying d needs no
// table load
__device__ __forceinline__ int dir_dx(int d) { return (int)((0x901Au >> (2 * d)) & 3u) - 1; }
__device__ __forceinline__ int dir_dy(int d) { return (int)((0xA901u >> (2 * d)) & 3u) - 1; }

__device__ __forceinline__ int getbit(const uint32_t *bits, int pww, int px, int py) {
    return (bits[py * pww + (px >> 5)] >> (px & 31)) & 1;
}

// bits (x-1 .. x+1) of padded row y as a 3-bit value.  Both words are read
// unconditionally (one ds_read2_b32, no branch on the trace's critical path;
// the LDS image has a slack word after its last row)
__device__ __forceinline__ uint32_t row3(const uint32_t *bits, int pww, int x, int y) {
    const int xm = x - 1, w = xm >> 5, b = xm & 31;
    const uint32_t *r = bits + y * pww + w;
    const uint64_t v = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
    return (uint32_t)(v >> b) & 7u;
}

// 8-neighbour mask of an interior padded pixel, bit d = direction d
__device__ __forceinline__ uint32_t nbmask(const uint32_t *bits, int pww, int x, int y) {
    const uint32_t t = row3(bits, pww, x, y - 1), m = row3(bits, pww, x, y), d = row3(bits, pww, x, y + 1);
    return ((m >> 2) & 1u) | (((t >> 2) & 1u) << 1) | (((t >> 1) & 1u) << 2) | ((t & 1u) << 3) | ((m & 1u) << 4) |
           ((d & 1u) << 5) | (((d >> 1) & 1u) << 6) | (((d >> 2) & 1u) << 7);
}

// One edge of green_edge between 8-neighbouring contour points (|dx|, |dy| <=
// 1) of a frame with both sides <= 512: every per-edge product fits in int32
// (|dxy| <= 1024, the largest term 1024 * 1.58e6 < 2^31), only the sums need
// int64 -- the same integers as green_edge with a fraction of the 64-bit
// multiplies.
__device__ __forceinline__ void green_edge_small(Green &g, int xi_1, int yi_1, int xi, int yi) {
    const int dxy = xi_1 * yi - xi * yi_1;
    const int xii_1 = xi_1 + xi, yii_1 = yi_1 + yi;
    g.a00 += dxy;
    g.a10 += dxy * xii_1;
    g.a01 += dxy * yii_1;
    g.a20 += dxy * (xi_1 * xii_1 + xi * xi);
    g.a11 += dxy * (xi_1 * (yii_1 + yi_1) + xi * (yii_1 + yi));
    g.a02 += dxy * (yi_1 * yii_1 + yi * yi);
}

template <bool SMALL>
__device__ Green trace_outer(const uint32_t *bits, int pww, int x0, int y0, long long max_steps) {
    Green g = {0, 0, 0, 0, 0, 0};
    // first fg neighbour clockwise from W: directions 3, 2, 1, 0, 7, 6, 5 (4 = none)
    const uint32_t nb0 = nbmask(bits, pww, x0, y0);
    int s = 4;
    {
        int k = 0;
        for (; k < 7; ++k) {
            const int d = (3 - k) & 7;
            if ((nb0 >> d) & 1u) {
                s = d;
                break;
            }
        }
        if (k == 7) return g;  // isolated pixel
    }
    const int x1 = x0 + dir_dx(s), y1 = y0 + dir_dy(s);
    int x3 = x0, y3 = y0;
    long long px = x0 - 1, py = y0 - 1;
    const long long sx = px, sy = py;
    bool first = true;
    for (long long step = 0; step < max_steps; ++step) {
        // next fg neighbour counter-clockwise from s + 1
        const uint32_t nb = nbmask(bits, pww, x3, y3);
        const int r = (s + 1) & 7;
        const uint32_t rot = ((nb | (nb << 8)) >> r) & 0xFFu;
        s = (r + __builtin_ctz(rot)) & 7;
        const int x4 = x3 + dir_dx(s), y4 = y3 + dir_dy(s);
        if (!first) {
            if constexpr (SMALL)
                green_edge_small(g, (int)px, (int)py, x3 - 1, y3 - 1);
            else
                green_edge(g, px, py, x3 - 1, y3 - 1);
            px = x3 - 1;
            py = y3 - 1;
        }
        first = false;
        if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
        x3 = x4;
        y3 = y4;
        s = (s + 4) & 7;
    }
    if constexpr (SMALL)
        green_edge_small(g, (int)px, (int)py, (int)sx, (int)sy);
    else
        green_edge(g, px, py, sx, sy);
    return g;
}

__device__ void moments_to_features(const Green &g, double *cen, double *ori, double *ax) {
    double m00 = 0, m10 = 0, m01 = 0, m20 = 0, m11 = 0, m02 = 0;
    const double a00 = (double)g.a00;
    if (fabs(a00) > FLT_EPSILON) {
        double db1_2, db1_6, db1_12, db1_24;
        if (a00 > 0) {
            db1_2 = 0.5; db1_6 = 0.16666666666666666666666666666667;
            db1_12 = 0.083333333333333333333333333333333; db1_24 = 0.041666666666666666666666666666667;
        } else {
            db1_2 = -0.5; db1_6 = -0.16666666666666666666666666666667;
            db1_12 = -0.083333333333333333333333333333333; db1_24 = -0.041666666666666666666666666666667;
        }
        m00 = a00 * db1_2;
        m10 = (double)g.a10 * db1_6;
        m01 = (double)g.a01 * db1_6;
        m20 = (double)g.a20 * db1_12;
        m11 = (double)g.a11 * db1_24;
        m02 = (double)g.a02 * db1_12;
    }
    double mcx = 0, mcy = 0;
    if (fabs(m00) > DBL_EPSILON) {
        const double inv_m00 = 1. / m00;
        mcx = m10 * inv_m00;
        mcy = m01 * inv_m00;
    }
    const double mu20 = m20 - m10 * mcx;
    const double mu11 = m11 - m10 * mcy;
    const double mu02 = m02 - m01 * mcy;
    if (m00 == 0) {
        cen[0] = cen[1] = ori[0] = ax[0] = ax[1] = __builtin_nan("");
        return;
    }
    const double num = 2 * mu11;
    const double den = mu20 - mu02;
    const double common = sqrt(4 * (mu11 * mu11) + den * den);
    ori[0] = -.5 * atan2(num, den);
    cen[0] = m10 / m00;
    cen[1] = m01 / m00;
    const double k = 2 * sqrt(2.0);
    ax[0] = k * sqrt((mu20 + mu02 + common) / m00);
    ax[1] = k * sqrt((mu20 + mu02 - common) / m00);
}

// The blob mask bit-packed by every CU (the threshold / mask pass is
// embarrassingly parallel; only the contour following is per frame): one
// wave per 64 padded pixels of a row, one byte of frame and mask per lane,
// the predicate gathered by one ballot into two words of the padded layout
// k_moments uses (bit b of word (py, wx) = pixel (py - 1, 32 wx + b - 1)).
// Per frame PH * pww words + one zero slack word.
__global__ __launch_bounds__(256) void k_moments_pack(const uint8_t *__restrict__ frames,
                                                      const uint8_t *__restrict__ mask, int H, int W, int ithr,
                                                      int pww, int chunks, long long nwaves,
                                                      uint32_t *__restrict__ bits) {
    const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= nwaves) return;  // whole waves
    const int lane = threadIdx.x & 63;
    const int PH = H + 2;
    const int c = (int)(gw % chunks);
    const long long rowg = gw / chunks;
    const int py = (int)(rowg % PH);
    const long long f = rowg / PH;
    const int x = 64 * c - 1 + lane;
    bool b = false;
    if (py >= 1 && py <= H && x >= 0 && x < W) {
        const long long i = f * (long long)H * W + (long long)(py - 1) * W + x;
        b = (int)frames[i] > ithr && (!mask || mask[i]);
    }
    const unsigned long long m = __ballot(b);
    uint32_t *o = bits + f * ((long long)PH * pww + 1) + (long long)py * pww;
    if (lane == 0) o[2 * c] = (uint32_t)m;
    if (lane == 1 && 2 * c + 1 < pww) o[2 * c + 1] = (uint32_t)(m >> 32);
    if (lane == 2 && c == 0 && py == PH - 1) o[pww] = 0u;  // the slack word after the last row
}

// ithr: the threshold as an integer, v > thr <=> (int)v > ithr for uint8 v.
// PRE: the bits come packed from k_moments_pack (`pre`), else packed here.
template <bool SMALL, bool PRE>
__global__ __launch_bounds__(MOM_THREADS) void k_moments(const uint8_t *__restrict__ frames,
                                                         const uint8_t *__restrict__ mask, int H, int W,
                                                         int ithr, double *__restrict__ cen,
                                                         double *__restrict__ ori, double *__restrict__ axl,
                                                         double *__restrict__ area, int pww,
                                                         const uint32_t *__restrict__ pre) {
    extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
    __shared__ unsigned long long s_best;
    __shared__ Green s_g;
    const int64_t f = blockIdx.x;
    const uint8_t *fr = frames + f * (int64_t)H * W;
    const uint8_t *mk = mask ? mask + f * (int64_t)H * W : nullptr;
    const int PH = H + 2, PW = W + 2;
    const int nwords = PH * pww;
    if (threadIdx.x == 0) s_best = 0ull;
    if constexpr (PRE) {
        const uint32_t *src = pre + f * ((int64_t)nwords + 1);
        for (int w = threadIdx.x; w <= nwords; w += MOM_THREADS) bits[w] = src[w];
    } else
    // bit-pack (frame > thr) & mask into LDS, one padded 32-pixel word per
    // lane: bit b of word (py, wx) is unpadded pixel (py - 1, 32 wx + b - 1).
    // Interior words read their 32 pixels [32 wx, 32 wx + 32) with two 16-B
    // loads (bits 1..31 + the next word's bit 0) plus the byte at 32 wx - 1.
    {
        const bool vec = (W % 16) == 0 && ((reinterpret_cast<uintptr_t>(fr) | reinterpret_cast<uintptr_t>(mk)) & 15) == 0;
        for (int w = threadIdx.x; w < nwords; w += MOM_THREADS) {
            const int py = w / pww, wx = w - py * pww;
            uint32_t word = 0;
            if (py >= 1 && py <= H) {
                const uint8_t *fy = fr + (py - 1) * W;
                const uint8_t *my = mk ? mk + (py - 1) * W : nullptr;
                const int xb = 32 * wx;  // pixel of bit 1
                if (vec && xb + 32 <= W) {
                    uint4 fv[2], mv[2];
                    fv[0] = *reinterpret_cast<const uint4 *>(fy + xb);
                    fv[1] = *reinterpret_cast<const uint4 *>(fy + xb + 16);
                    if (my) {
                        mv[0] = *reinterpret_cast<const uint4 *>(my + xb);
                        mv[1] = *reinterpret_cast<const uint4 *>(my + xb + 16);
                    }
                    const uint8_t *fe = reinterpret_cast<const uint8_t *>(fv);
                    const uint8_t *me = reinterpret_cast<const uint8_t *>(mv);
                    uint32_t u = 0;
#pragma unroll
                    for (int k = 0; k < 31; ++k) u |= (uint32_t)((int)fe[k] > ithr && (!my || me[k])) << (k + 1);
                    if (xb > 0) u |= (uint32_t)((int)fy[xb - 1] > ithr && (!my || my[xb - 1]));
                    word = u;
                } else {
                    for (int k = 0; k < 32; ++k) {
                        const int x = xb + k - 1;
                        if (x >= 0 && x < W) word |= (uint32_t)((int)fy[x] > ithr && (!my || my[x])) << k;
                    }
                }
            }
            bits[w] = word;
        }
        if (threadIdx.x == 0) bits[nwords] = 0u;  // slack word read by row3
    }
    __syncthreads();
    unsigned long long best = 0ull;
    Green bg = {0, 0, 0, 0, 0, 0};
    const long long max_steps = 8ll * PH * PW + 16;
    for (int w = threadIdx.x; w < nwords; w += MOM_THREADS) {
        const uint32_t word = bits[w];
        if (!word) continue;
        const int py = w / pww, wx = w - py * pww;
        const uint32_t prev = wx > 0 ? bits[w - 1] : 0u;
        const uint32_t up = bits[w - pww];  // py >= 1 for any set bit
        const uint32_t upprev = wx > 0 ? bits[w - pww - 1] : 0u;
        const uint32_t upnext = wx + 1 < pww ? bits[w - pww + 1] : 0u;
        const uint32_t L = (word << 1) | (prev >> 31);
        const uint32_t UL = (up << 1) | (upprev >> 31);
        const uint32_t UR = (up >> 1) | (upnext << 31);
        uint32_t cand = word & ~L & ~up & ~UL & ~UR;
        while (cand) {
            const int b = __builtin_ctz(cand);
            cand &= cand - 1;
            const int px = wx * 32 + b;
            const Green g = trace_outer<SMALL>(bits, pww, px, py, max_steps);
            const unsigned long long a = (unsigned long long)(g.a00 < 0 ? -g.a00 : g.a00);
            const unsigned long long start = (unsigned long long)py * PW + px;
            const unsigned long long key = (a << 32) | (0xFFFFFFFFull - start);
            if (key > best) {
                best = key;
                bg = g;
            }
        }
    }
    atomicMax(&s_best, best);
    __syncthreads();
    if (best != 0ull && best == s_best) s_g = bg;  // keys are unique (start index)
    __syncthreads();
    if (threadIdx.x == 0) {
        double c[2], o, a[2];
        if (s_best == 0ull) {
            c[0] = c[1] = o = a[0] = a[1] = __builtin_nan("");
            if (area) area[f] = __builtin_nan("");
        } else {
            moments_to_features(s_g, c, &o, a);
            if (area) area[f] = fabs((double)s_g.a00 * 0.5);
        }
        cen[2 * f] = c[0];
        cen[2 * f + 1] = c[1];
        ori[f] = o;
        axl[2 * f] = a[0];
        axl[2 * f + 1] = a[1];
    }
}

// ---------------------------------------------------------------------------
// crop_and_rotate_frame: one workgroup per frame, both sources share the map.
// ---------------------------------------------------------------------------
// (blockIdx.y: a block of output rows, so a batch's crops spread over
// several workgroups per frame; each recomputes the 6-double map)
constexpr int CROP_RB = 4;

__global__ __launch_bounds__(256) void k_crop(const uint8_t *__restrict__ src0, const uint8_t *__restrict__ src1,
                                              int H, int W, const double *__restrict__ center,
                                              const double *__restrict__ angle, int cw, int ch,
                                              uint8_t *__restrict__ out0, uint8_t *__restrict__ out1,
                                              int *__restrict__ window) {
    const int64_t f = blockIdx.x;
    const bool lead = blockIdx.y == 0 && threadIdx.x == 0;  // writes the window
    const double cxc = center[2 * f], cyc = center[2 * f + 1], ang_deg = angle[f];
    uint8_t *o0 = out0 + f * (int64_t)cw * ch;
    uint8_t *o1 = out1 ? out1 + f * (int64_t)cw * ch : nullptr;
    bool zero = isnan(ang_deg) || isnan(cxc) || isnan(cyc) || cxc < 0 || cyc < 0;
    int xmin = 0, ymin = 0, pw = 0, ph = 0;
    double M[6] = {0, 0, 0, 0, 0, 0};
    if (window && lead) {  // -1 x4: the reference returns zeros before computing a window
        window[4 * f] = window[4 * f + 1] = window[4 * f + 2] = window[4 * f + 3] = -1;
    }
    if (!zero) {
        xmin = (int)(cxc - cw / 2) + cw;
        const int xmax = (int)(cxc + cw / 2) + cw;
        ymin = (int)(cyc - ch / 2) + ch;
        const int ymax = (int)(cyc + ch / 2) + ch;
        if (window && lead) {
            window[4 * f] = xmin;
            window[4 * f + 1] = xmax;
            window[4 * f + 2] = ymin;
            window[4 * f + 3] = ymax;
        }
        const int PWd = W + 2 * cw, PHd = H + 2 * ch;
        const int sx0 = xmin < 0 ? 0 : (xmin > PWd ? PWd : xmin);
        const int sx1 = xmax < 0 ? 0 : (xmax > PWd ? PWd : xmax);
        const int sy0 = ymin < 0 ? 0 : (ymin > PHd ? PHd : ymin);
        const int sy1 = ymax < 0 ? 0 : (ymax > PHd ? PHd : ymax);
        xmin = sx0;
        ymin = sy0;
        pw = sx1 - sx0;
        ph = sy1 - sy0;
        if (pw <= 0 || ph <= 0) zero = true;
        const double CV_PI_ = 3.1415926535897932384626433832795;
        const double ang = ang_deg * (CV_PI_ / 180);
        const double alpha = cos(ang) * 1.0, beta = sin(ang) * 1.0;
        const double ccx = (double)(float)(cw / 2), ccy = (double)(float)(ch / 2);
        M[0] = alpha; M[1] = beta; M[2] = (1 - alpha) * ccx - beta * ccy;
        M[3] = -beta; M[4] = alpha; M[5] = beta * ccx + (1 - alpha) * ccy;
        double D = M[0] * M[4] - M[1] * M[3];
        D = D != 0 ? 1. / D : 0;
        const double A11 = M[4] * D, A22 = M[0] * D;
        M[0] = A11; M[1] *= -D;
        M[3] *= -D; M[4] = A22;
        const double b1 = -M[0] * M[2] - M[1] * M[5];
        const double b2 = -M[3] * M[2] - M[4] * M[5];
        M[2] = b1; M[5] = b2;
    }
    const int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5, TAB = 1 << INTER_BITS;
    const int round_delta = AB_SCALE / TAB / 2;
    const uint8_t *s0 = src0 + f * (int64_t)H * W;
    const uint8_t *s1 = src1 ? src1 + f * (int64_t)H * W : nullptr;
    const int rows = (ch + CROP_RB - 1) / CROP_RB;
    const int i0 = (int)blockIdx.y * rows * cw, i1 = min(ch, ((int)blockIdx.y + 1) * rows) * cw;
    for (int i = i0 + threadIdx.x; i < i1; i += 256) {
        if (zero) {
            o0[i] = 0;
            if (o1) o1[i] = 0;
            continue;
        }
        const int y = i / cw, x = i - y * cw;
        const int X0 = __double2int_rn((M[1] * y + M[2]) * AB_SCALE) + round_delta;
        const int Y0 = __double2int_rn((M[4] * y + M[5]) * AB_SCALE) + round_delta;
        const int adelta = __double2int_rn(M[0] * x * AB_SCALE);
        const int bdelta = __double2int_rn(M[3] * x * AB_SCALE);
        const int X = (X0 + adelta) >> (AB_BITS - INTER_BITS);
        const int Y = (Y0 + bdelta) >> (AB_BITS - INTER_BITS);
        const int sx = X >> INTER_BITS, sy = Y >> INTER_BITS;
        const int tx = X & (TAB - 1), ty = Y & (TAB - 1);
        const int w[4] = {(32 - ty) * (32 - tx) * 32, (32 - ty) * tx * 32, ty * (32 - tx) * 32, ty * tx * 32};
        int acc0 = 0, acc1 = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int qx = sx + (t & 1), qy = sy + (t >> 1);
            if (qx >= 0 && qx < pw && qy >= 0 && qy < ph) {
                const int fx = xmin + qx - cw, fy = ymin + qy - ch;
                if (fx >= 0 && fx < W && fy >= 0 && fy < H) {
                    acc0 += s0[(int64_t)fy * W + fx] * w[t];
                    if (s1) acc1 += s1[(int64_t)fy * W + fx] * w[t];
                }
            }
        }
        acc0 = (acc0 + (1 << 14)) >> 15;
        o0[i] = (uint8_t)(acc0 < 0 ? 0 : (acc0 > 255 ? 255 : acc0));
        if (o1) {
            acc1 = (acc1 + (1 << 14)) >> 15;
            o1[i] = (uint8_t)(acc1 < 0 ? 0 : (acc1 > 255 ? 255 : acc1));
        }
    }
}

// ---------------------------------------------------------------------------
// per-frame reductions of compute_scalars (M/proc/scalars.py:79-103) on
// frames * masks (M/pipeline/process_features_step.py:165) and the keypoint
// z lookup of keypoints_to_dict (M/proc/keypoints.py:122-130).  One
// workgroup per frame; 16-B loads; integer sums (exact).
// ---------------------------------------------------------------------------
constexpr int SC_THREADS = 256;

// np.clip(np.floor(v).astype(int), 0, hi): NaN / +-inf / |v| >= 2^63 become
// INT64_MIN on x86 (cvttsd2si's integer indefinite) and clip to 0
__device__ __forceinline__ int np_floor_clip(double v, int hi) {
    if (!(fabs(v) < 9.2233720368547758e18)) return 0;
    const double fl = floor(v);
    return fl < 0.0 ? 0 : (fl > (double)hi ? hi : (int)fl);
}

__device__ __forceinline__ void sc_acc1(uint32_t f8, uint32_t m8, double lo, double hi, unsigned &cnt,
                                        unsigned &sum) {
    const uint32_t v = (f8 * m8) & 255u;  // uint8 product
    const bool in = (double)v > lo && (double)v < hi;
    cnt += in;
    sum += in ? v : 0u;
}

__device__ __forceinline__ void sc_acc(uint32_t fw, uint32_t mw, double lo, double hi, unsigned &cnt,
                                       unsigned &sum) {
#pragma unroll
    for (int b = 0; b < 4; ++b) sc_acc1((fw >> (8 * b)) & 255u, (mw >> (8 * b)) & 255u, lo, hi, cnt, sum);
}

__global__ __launch_bounds__(SC_THREADS) void k_frame_scalars(const uint8_t *__restrict__ frames,
                                                              const uint8_t *__restrict__ masks, int H, int W,
                                                              double lo, double hi, const double *__restrict__ kpts,
                                                              int K, const uint8_t *__restrict__ zsrc,
                                                              long long *__restrict__ area,
                                                              double *__restrict__ mean_h, double *__restrict__ z) {
    __shared__ unsigned long long s_c, s_s;
    const int64_t f = blockIdx.x;
    const int64_t hw = (int64_t)H * W;
    const uint8_t *fr = frames + f * hw;
    const uint8_t *mk = masks ? masks + f * hw : nullptr;
    if (threadIdx.x == 0) s_c = s_s = 0ull;
    __syncthreads();
    unsigned cnt = 0, sum = 0;  // <= 256 * 255 per lane per 16-B word: no overflow at frame sizes < 2^24
    int64_t p0 = 0;
    if ((((uintptr_t)fr | (uintptr_t)mk) & 15) == 0) {
        const int64_t nv = hw / 16;
        for (int64_t v = threadIdx.x; v < nv; v += SC_THREADS) {
            const uint4 a = reinterpret_cast<const uint4 *>(fr)[v];
            const uint4 m = mk ? reinterpret_cast<const uint4 *>(mk)[v] : make_uint4(0x01010101u, 0x01010101u,
                                                                                     0x01010101u, 0x01010101u);
            sc_acc(a.x, m.x, lo, hi, cnt, sum);
            sc_acc(a.y, m.y, lo, hi, cnt, sum);
            sc_acc(a.z, m.z, lo, hi, cnt, sum);
            sc_acc(a.w, m.w, lo, hi, cnt, sum);
        }
        p0 = nv * 16;
    }
    for (int64_t p = p0 + threadIdx.x; p < hw; p += SC_THREADS)
        sc_acc1(fr[p], mk ? mk[p] : 1u, lo, hi, cnt, sum);
    unsigned long long c = cnt, sm = sum;
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o);
        sm += __shfl_xor(sm, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_c, c);
        atomicAdd(&s_s, sm);
    }
    if (kpts && zsrc && threadIdx.x < K) {
        const double *kp = kpts + (f * K + threadIdx.x) * 3;
        const int x = np_floor_clip(kp[0], W - 1), y = np_floor_clip(kp[1], H - 1);
        z[f * K + threadIdx.x] = (double)zsrc[f * hw + (int64_t)y * W + x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        area[f] = (long long)s_c;
        // np.mean over the selected uint8 values: exact integer sum / count
        mean_h[f] = s_c ? (double)s_s / (double)s_c : 0.0;
    }
}

}  // namespace mdx

using namespace mdx;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int mdx_prep_frames(const int16_t *raw, int64_t n, int H, int W, const double *bg, const uint8_t *roi,
                               int y0, int y1, int x0, int x1, int flags, double vmin, double vmax, uint8_t *out,
                               uint8_t *invalid, mdx_stream_t stream) {
    MDX_REQUIRE(raw && out, "mdx_prep_frames: null raw/out");
    MDX_REQUIRE(n >= 0 && H > 0 && W > 0, "mdx_prep_frames: bad shape n=%lld H=%d W=%d", (long long)n, H, W);
    MDX_REQUIRE(0 <= y0 && y0 <= y1 && y1 <= H && 0 <= x0 && x0 <= x1 && x1 <= W,
                "mdx_prep_frames: bad crop [%d,%d)x[%d,%d) for %dx%d", y0, y1, x0, x1, H, W);
    const int oh = y1 - y0, ow = x1 - x0;
    if (n == 0 || oh == 0 || ow == 0) return MDX_OK;
    MDX_REQUIRE(ceil_div(n, PREP_FRAMES_PER_BLOCK) <= 65535, "mdx_prep_frames: too many frames");
    return launch_prep(raw, n, H, W, bg, roi, y0, y1, x0, x1, flags, vmin, vmax, out, invalid, nullptr, 0, 0,
                       as_stream(stream));
}

extern "C" int mdx_build_scale_lut(double vmin, double vmax, int int_vmin, uint8_t lut[256]) {
    MDX_REQUIRE(lut != nullptr, "mdx_build_scale_lut: null lut");
    const double k = (255.0 - 0.0) / (vmax - vmin);
    for (int v = 0; v < 256; ++v) {
        const double d = int_vmin ? (double)(uint8_t)(v - (int)vmin) : (double)v - vmin;
        const double r = d * k + 0.0;
        lut[v] = (uint8_t)(int32_t)r;
    }
    return MDX_OK;
}

extern "C" int mdx_scale_frames(const uint8_t *in, int64_t count, const uint8_t lut[256], uint8_t *out,
                                mdx_stream_t stream) {
    MDX_REQUIRE(in && out && lut, "mdx_scale_frames: null pointer");
    if (count <= 0) return MDX_OK;
    MDX_REQUIRE(((uintptr_t)in % 16) == 0 && ((uintptr_t)out % 16) == 0, "mdx_scale_frames: buffers must be 16-B aligned");
    Lut256 L;
    memcpy(L.v, lut, 256);
    const int64_t nvec = count / 16;
    int blocks = (int)std::min<int64_t>(std::max<int64_t>(ceil_div(nvec, 256), 1), 2048);
    hipLaunchKernelGGL(k_scale, dim3(blocks), dim3(256), 0, as_stream(stream), in, count, L, out);
    MDX_CHECK_LAUNCH("mdx_scale_frames");
    return MDX_OK;
}

extern "C" int64_t mdx_clean_workspace_bytes(int64_t n, int H, int W) { return n * H * W; }

// clean_frames kernel choice: 0 = one launch per pass (k_median3, k_morph),
// 1 = the fused streaming kernel, strip width by batch size (default: 512
// columns from 16 strips per launch on, else 256), 2 = 256-column strips,
// 3 = 512-column strips.  The fused kernel
// serves the extract path's chain (median 3, opening with the 9x9 ellipse,
// 3 iterations); anything else runs the per-pass kernels.  Returns the
// previous mode.
static int g_clean_mode = 1;
extern "C" int mdx_clean_set_mode(int mode) {
    const int old = g_clean_mode;
    if (mode >= 0 && mode <= 3) g_clean_mode = mode;
    return old;
}

extern "C" int mdx_clean_frames(const uint8_t *src, int64_t n, int H, int W, int median_k, const uint8_t *strel,
                                int kh, int kw, int iters, uint8_t *out, uint8_t *workspace, mdx_stream_t stream) {
    MDX_REQUIRE(src && out && src != out, "mdx_clean_frames: null or aliased buffers");
    MDX_REQUIRE(median_k == 0 || median_k == 3, "mdx_clean_frames: median_k must be 0 or 3 (got %d)", median_k);
    MDX_REQUIRE(iters >= 0, "mdx_clean_frames: iters < 0");
    MDX_REQUIRE(iters == 0 || (workspace && workspace != src && workspace != out),
                "mdx_clean_frames: the opening needs a distinct workspace of n*H*W bytes");
    StrelSpans st{};
    if (iters > 0) {
        MDX_REQUIRE(strel && kh > 0 && kw > 0 && kh <= MAX_KH && kw <= MAX_KH, "mdx_clean_frames: strel %dx%d", kh, kw);
        st.kh = kh;
        st.kw = kw;
        st.ay = kh / 2;
        st.ax = kw / 2;
        for (int r = 0; r < kh; ++r) {
            int j1 = -1, j2 = -1;
            for (int c = 0; c < kw; ++c) {
                if (strel[r * kw + c]) {
                    if (j1 < 0) j1 = c;
                    MDX_REQUIRE(j2 < 0, "mdx_clean_frames: strel row %d is not one contiguous run", r);
                    if (c + 1 == kw || !strel[r * kw + c + 1]) j2 = c + 1;
                }
            }
            if (j1 < 0) j1 = j2 = 0;
            st.j1[r] = (int8_t)j1;
            st.j2[r] = (int8_t)j2;
        }
        st.nspan = 0;
        for (int r = 0; r < kh; ++r) {
            st.rspan[r] = -1;
            if (st.j2[r] <= st.j1[r]) continue;
            int k = 0;
            for (; k < st.nspan; ++k)
                if (st.sj1[k] == st.j1[r] && st.sj2[k] == st.j2[r]) break;
            if (k == st.nspan) {
                st.sj1[k] = st.j1[r];
                st.sj2[k] = st.j2[r];
                ++st.nspan;
            }
            st.rspan[r] = (int8_t)k;
        }
    }
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(n <= 65535, "mdx_clean_frames: n > 65535 per call");
    MDX_REQUIRE((long long)H * W < (1ll << 31), "mdx_clean_frames: frame too large");
    hipStream_t s = as_stream(stream);
    if (g_clean_mode != 0 && median_k == 3 && iters == 3 && is_ellipse9(strel, kh, kw)) {
        // auto: the 512-column strips (least halo work per frame: the kernel is
        // VALU-issue bound, and in the extract loop its CU time, not its
        // latency, is what the concurrent forwards feel) unless the batch is
        // too small to give a few dozen CUs work
        const bool wide = g_clean_mode == 3 || (g_clean_mode == 1 && n * ceil_div(W, 512) >= 16);
        if (wide) {
            const int strips = (int)ceil_div(W, 512);
            hipLaunchKernelGGL(k_clean_stream<512>, dim3((unsigned)(n * strips)), dim3(CleanStream<512>::THREADS), 0,
                               s, src, H, W, strips, out);
        } else {
            const int strips = (int)ceil_div(W, 256);
            hipLaunchKernelGGL(k_clean_stream<256>, dim3((unsigned)(n * strips)), dim3(CleanStream<256>::THREADS), 0,
                               s, src, H, W, strips, out);
        }
        MDX_CHECK_LAUNCH("mdx_clean_frames");
        return MDX_OK;
    }
    const int tiles_x = (int)ceil_div(W, CT_W), tiles_y = (int)ceil_div(H, CT_H);
    const dim3 grid(tiles_x * tiles_y, (unsigned)n);
    const int LW = CT_W + kw - 1, LH = CT_H + kh - 1, LP = (LW + 7) & ~3;
    const size_t lds = 2 * ((size_t)LH * LP + (size_t)std::max(st.nspan, 1) * LH * CT_W);
    // pass chain: the last pass writes `out`; ping-pong through the workspace
    const int npass = (median_k ? 1 : 0) + 2 * iters;
    const uint8_t *cur = src;
    for (int p = 0; p < npass; ++p) {
        uint8_t *dst = ((npass - 1 - p) % 2 == 0) ? out : workspace;
        if (median_k && p == 0) {
            hipLaunchKernelGGL(k_median3, grid, dim3(CT_THREADS), 0, s, cur, H, W, dst, tiles_x);
        } else {
            const int q = p - (median_k ? 1 : 0);
            if (q < iters)
                hipLaunchKernelGGL(k_morph<false>, grid, dim3(CT_THREADS), lds, s, cur, H, W, st, dst, tiles_x);
            else
                hipLaunchKernelGGL(k_morph<true>, grid, dim3(CT_THREADS), lds, s, cur, H, W, st, dst, tiles_x);
        }
        cur = dst;
    }
    MDX_CHECK_LAUNCH("mdx_clean_frames");
    return MDX_OK;
}

extern "C" int64_t mdx_frame_moments_workspace_bytes(int64_t n, int H, int W) {
    if (n <= 0 || H <= 0 || W <= 0) return 0;
    return n * ((int64_t)(H + 2) * ceil_div(W + 2, 32) + 1) * 4;
}

extern "C" int mdx_frame_moments_ws(const uint8_t *frames, const uint8_t *mask, int64_t n, int H, int W, double thr,
                                    double *centroid, double *orientation, double *axis_length, double *area,
                                    void *workspace, mdx_stream_t stream) {
    MDX_REQUIRE(frames && centroid && orientation && axis_length, "mdx_frame_moments: null pointer");
    MDX_REQUIRE(H > 0 && W > 0, "mdx_frame_moments: bad shape");
    if (n == 0) return MDX_OK;
    const int pww = (int)ceil_div(W + 2, 32);
    const size_t lds = ((size_t)(H + 2) * pww + 4) * 4;  // + slack words
    MDX_REQUIRE(lds <= 120 * 1024, "mdx_frame_moments: frame %dx%d too large for LDS", H, W);
    MDX_REQUIRE(n <= 0x7fffffff, "mdx_frame_moments: n too large");
    // v > thr for uint8 v <=> v > floor(thr) (NaN: never)
    const int ithr = thr != thr ? 255 : thr < 0 ? -1 : thr >= 255 ? 255 : (int)floor(thr);
    hipStream_t s = as_stream(stream);
    const uint32_t *pre = static_cast<const uint32_t *>(workspace);
    if (pre) {
        const int chunks = (pww + 1) / 2;
        const long long nwaves = n * (long long)(H + 2) * chunks;
        MDX_REQUIRE(ceil_div(nwaves, 4) < (1ll << 31), "mdx_frame_moments: too many frames per call");
        hipLaunchKernelGGL(k_moments_pack, dim3((unsigned)ceil_div(nwaves, 4)), dim3(256), 0, s, frames, mask, H, W,
                           ithr, pww, chunks, nwaves, (uint32_t *)workspace);
    }
    const bool small = H <= 512 && W <= 512;
    if (pre && small)
        hipLaunchKernelGGL((k_moments<true, true>), dim3((unsigned)n), dim3(MOM_THREADS), lds, s, frames, mask, H, W,
                           ithr, centroid, orientation, axis_length, area, pww, pre);
    else if (pre)
        hipLaunchKernelGGL((k_moments<false, true>), dim3((unsigned)n), dim3(MOM_THREADS), lds, s, frames, mask, H, W,
                           ithr, centroid, orientation, axis_length, area, pww, pre);
    else if (small)
        hipLaunchKernelGGL((k_moments<true, false>), dim3((unsigned)n), dim3(MOM_THREADS), lds, s, frames, mask, H, W,
                           ithr, centroid, orientation, axis_length, area, pww, pre);
    else
        hipLaunchKernelGGL((k_moments<false, false>), dim3((unsigned)n), dim3(MOM_THREADS), lds, s, frames, mask, H,
                           W, ithr, centroid, orientation, axis_length, area, pww, pre);
    MDX_CHECK_LAUNCH("mdx_frame_moments");
    return MDX_OK;
}

extern "C" int mdx_frame_moments(const uint8_t *frames, const uint8_t *mask, int64_t n, int H, int W, double thr,
                                 double *centroid, double *orientation, double *axis_length, double *area,
                                 mdx_stream_t stream) {
    return mdx_frame_moments_ws(frames, mask, n, H, W, thr, centroid, orientation, axis_length, area, nullptr,
                                stream);
}

extern "C" int mdx_crop_rotate(const uint8_t *src0, const uint8_t *src1, int64_t n, int H, int W,
                               const double *center, const double *angle_deg, int cw, int ch, uint8_t *out0,
                               uint8_t *out1, int32_t *window, mdx_stream_t stream) {
    MDX_REQUIRE(src0 && out0 && center && angle_deg, "mdx_crop_rotate: null pointer");
    MDX_REQUIRE(!src1 == !out1, "mdx_crop_rotate: src1/out1 must both be set or both NULL");
    MDX_REQUIRE(cw > 0 && ch > 0 && H > 0 && W > 0, "mdx_crop_rotate: bad shape");
    if (n == 0) return MDX_OK;
    hipLaunchKernelGGL(k_crop, dim3((unsigned)n, CROP_RB), dim3(256), 0, as_stream(stream), src0, src1, H, W, center,
                       angle_deg, cw, ch, out0, out1, (int *)window);
    MDX_CHECK_LAUNCH("mdx_crop_rotate");
    return MDX_OK;
}

extern "C" int mdx_frame_scalars(const uint8_t *frames, const uint8_t *masks, int64_t n, int H, int W,
                                 double min_height, double max_height, const double *keypoints, int K,
                                 const uint8_t *z_frames, int64_t *area_px, double *height_ave, double *z_data,
                                 mdx_stream_t stream) {
    MDX_REQUIRE(frames && area_px && height_ave, "mdx_frame_scalars: null pointer");
    MDX_REQUIRE(H > 0 && W > 0 && (int64_t)H * W < (1ll << 24), "mdx_frame_scalars: bad frame %dx%d", H, W);
    MDX_REQUIRE(K >= 0 && K <= SC_THREADS, "mdx_frame_scalars: K must be in [0, %d]", SC_THREADS);
    MDX_REQUIRE(K == 0 || (keypoints && z_frames && z_data), "mdx_frame_scalars: keypoints need z_frames and z_data");
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(n <= 0x7fffffff, "mdx_frame_scalars: n too large");
    hipLaunchKernelGGL(k_frame_scalars, dim3((unsigned)n), dim3(SC_THREADS), 0, as_stream(stream), frames, masks, H, W,
                       min_height, max_height, K ? keypoints : nullptr, K, K ? z_frames : nullptr,
                       (long long *)area_px, height_ave, z_data);
    MDX_CHECK_LAUNCH("mdx_frame_scalars");
    return MDX_OK;
}
