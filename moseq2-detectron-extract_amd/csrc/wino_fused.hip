// Fused Winograd F(4x4, 3x3) convolution, fp32, for gfx950 (k_wino_f4).
//
// The model's 3x3 stride-1 layers (ResNet bottleneck conv2, FPN outputs, RPN
// head, mask / keypoint head convs) as one launch each: input transform, the
// 36 tile-point GEMMs on v_mfma_f32_16x16x4_f32 and output transform + bias +
// ReLU, with V and M living only in LDS / registers (conv.hip's three-launch
// path writes both to HBM).  Built without packed FP32 (_build.py
// DEVICE_FLAGS): the transforms otherwise compile to v_pk forms outside the
// cleared set of _isa_lint.py.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "wino_tables.h"

namespace mdx {

typedef float float4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void *lds_ptr_t;

// F(4x4, 3x3) on points 0, +-1, +-2, inf (Lavin): B^T (6x6), A^T (4x6); G is
// applied on the host (mdx_winograd_weights, conv.hip)
struct WF4T {
    __device__ static constexpr float BT(int i, int j) {
        constexpr float t[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0}, {0, 4, -4, -1, 1, 0},
                                   {0, -2, -1, 2, 1, 0}, {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
        return t[i][j];
    }
    __device__ static constexpr float AT(int i, int j) {
        constexpr float t[4][6] = {{1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};
        return t[i][j];
    }
};

// ---------------------------------------------------------------------------
// Fused Winograd F(4x4, 3x3), fp32: input transform, the 36 tile-point GEMMs
// and the output transform (+ bias + ReLU) in one launch -- V and M never
// reach memory.
//
// Workgroup = one block of 32 tiles (bh x bw tiles of ipb images) x 32 output
// channels x all 36 points, 8 waves in two roles, one of each per SIMD so the
// producers' VALU overlaps the consumers' MFMAs:
//   consumers (waves 0-3): wave c owns points 9 c .. 9 c + 8 of the whole
//     32 x 32 block (per point 2 x 2 MFMA 16x16 tiles); accumulators 9 x 4 x 4
//     = 144 registers.  A fragments from LDS; B fragments straight from the
//     packed U (mdx_winograd_pack_f4: one coalesced 16-B load per lane and
//     point), one K-step ahead in registers;
//   producers (waves 4-7): copy the block's input region ((4 bh + 2) x (4 bw
//     + 2) pixels per image, 8 channels = two 16-B pieces per pixel) into LDS
//     by LDS-DMA three K-steps ahead (three raw buffers, no register round
//     trip; each input byte crosses L2 once per K-step instead of once per
//     overlapping 6x6 patch), then per (tile, channel) item read the 6x6
//     patch from LDS, zero the padding and write B^T d B into the A stage.
// K in steps of 8 input channels; the A stage ([36][4 k-pairs][32 slots][2]
// fp32, 36 KiB) is double-buffered: consumers multiply K-step k while
// producers transform k + 1, one barrier per K-step.  Slots are rotated per
// k-pair (wf4_idx) so each half-wave's 8-B fragment reads cover the 64 banks
// once and the transform's 4-B writes fold 2-way; raw pixels are XOR-permuted
// within groups of four (wf4_px) so the transform's reads of a row of tiles
// are conflict-free.  MFMA e of a K-step uses k = 2 (lane >> 4) + e on both
// operands (a permutation of the 8 channels).
// Epilogue, one 16 x 16 (tile, channel) quarter at a time: each consumer
// folds its points into per-row partials s_a[j] = sum_b AT[j][b] m[a][b] (two
// row slots per wave), the producers combine the eight slots (A^T over rows),
// add bias, ReLU and store.
// ---------------------------------------------------------------------------
constexpr int WF4_MT = 32, WF4_NC = 32, WF4_KC = 8, WF4_THREADS = 512, WF4_XW = 9;
constexpr int WF4_STAGE = 36 * WF4_MT * WF4_KC * 4;  // one A stage = 36 KiB
constexpr int WF4_MAXPX = 800;                       // raw region pixels per K-step (all images of a block)
constexpr int WF4_RAWZ = WF4_MAXPX * 32;             // zero pixel of a raw buffer (never DMA'd)
constexpr int WF4_RAW = WF4_RAWZ + 64;               // bytes of one raw buffer (2 x 16-B pieces per pixel)
constexpr int WF4_LDS = 2 * WF4_STAGE + 3 * WF4_RAW;  // 150,720 B

#define MDX_WAIT_VMN(n)                                                                        \
    do {                                                                                       \
        asm volatile("" ::: "memory");                                                         \
        __builtin_amdgcn_s_waitcnt(0x0F70 | ((n) & 15) | ((((n) >> 4) & 3) << 14));            \
        asm volatile("" ::: "memory");                                                         \
    } while (0)

struct WinoF4Args {
    const float *x;     // NHWC [N][H][W][Cin]
    const float *Up;    // packed U (mdx_winograd_pack_f4)
    const float *bias;  // [Cout] or null
    float *out;         // NHWC [N][H][W][Cout]
    int N, H, W, Cin, Cout, TH, TW;
    int relu, tblocks, nblocks;
    int bh, bw, ipb, nbx, nby;  // block geometry: bh x bw tiles of ipb images; blocks per image row / column
    int rh, rw, npx, ndma;      // raw region rows / columns per image, pixels, 64-piece DMA instructions
    int xbytes, ubytes;
    int dbg;  // timing experiments (MDX_WF4_DEBUG): bit 0 skips the producers' work, bit 1 the MFMAs
};

// float offset of (row, k) in one point's [4 k-pairs][32 slots][2] A-stage
// slice: slot = (row + f(kp)) mod 32, f = 16 (kp & 1) + 4 (kp >> 1)
__host__ __device__ constexpr int wf4_idx(int row, int k) {
    return (k >> 1) * 64 + (((row + 16 * ((k >> 1) & 1) + 4 * (k >> 2)) & 31) << 1) + (k & 1);
}
// LDS pixel slot of raw region pixel p (an involution: low two bits XOR the next two)
__device__ __forceinline__ int wf4_px(int p) { return p ^ ((p >> 2) & 3); }

__global__ __launch_bounds__(WF4_THREADS, 2) void k_wino_f4(WinoF4Args a) {
    using WT = WF4T;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *Abuf = reinterpret_cast<float *>(smem);  // A stage s at s * STAGE / 4 floats
    char *Raw = smem + 2 * WF4_STAGE;               // raw buffer r at r * WF4_RAW
    // XCD-contiguous remap (the channel blocks of one tile block share its
    // input region in one L2)
    int id;
    {
        const int L = blockIdx.x, nwg = a.tblocks * a.nblocks;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tb = id / a.nblocks, nb = id - tb * a.nblocks;
    const int bx = tb % a.nbx, tr_ = tb / a.nbx;
    const int by = tr_ % a.nby, g = tr_ / a.nby;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int KS = a.Cin / WF4_KC;
    const int bt = a.bh * a.bw;
    // tile slot s -> (image n, tile row ty, tile column tx, image of the block i)
    auto slot_tile = [&](int s, int &n, int &ty, int &tx, int &img) {
        img = s / bt;
        const int l = s - img * bt;
        const int ly = l / a.bw, lx = l - ly * a.bw;
        n = g * a.ipb + img;
        ty = by * a.bh + ly;
        tx = bx * a.bw + lx;
        return img < a.ipb && n < a.N && ty < a.TH && tx < a.TW;
    };

    if (wid >= 4) {
        // ================= producers =================
        const int pt = tid - 256, pw = pt >> 6;
        const int ch = pt & 7, tl = pt >> 3;
        // DMA pieces of this lane: instruction d = 4 j + pw, piece d * 64 + lane =
        // (LDS pixel slot P, half h), source pixel wf4_px(P) of the region
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)a.x, (short)0, a.xbytes,
                                                                            0x00020000);
        const int nd = (a.ndma - pw + 3) / 4;  // this wave's DMA instructions (<= 7)
        unsigned src[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int q = (4 * j + pw) * 64 + lane;
            const int P = q >> 1, h = q & 1;
            unsigned off = 0;  // (pieces past the region / outside the image fetch offset 0: never read unmasked)
            if (P < a.npx) {
                const int p = wf4_px(P);
                const int img = p / (a.rh * a.rw), r = p - img * (a.rh * a.rw);
                const int ry = r / a.rw, rxx = r - ry * a.rw;
                const int n = g * a.ipb + img, y = by * a.bh * 4 - 1 + ry, xx = bx * a.bw * 4 - 1 + rxx;
                if (n < a.N && y >= 0 && y < a.H && xx >= 0 && xx < a.W)
                    off = (unsigned)(((((long long)n * a.H + y) * a.W + xx) * a.Cin + 4 * h) * 4);
            }
            src[j] = off;
        }
        auto dma = [&](int ks) {
            char *rb = Raw + (ks % 3) * WF4_RAW;
            const int kb = ks * (WF4_KC * 4);
#pragma unroll
            for (int j = 0; j < 7; ++j)
                if (j < nd)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(rb + (4 * j + pw) * 1024), 16, src[j], kb,
                                                             0, 0);
        };
        // the item: tile slot tl, channel ch; patch validity masks and the
        // raw-region pixel of its patch origin
        int n, ty, tx, img;
        const bool tok = slot_tile(tl, n, ty, tx, img);
        int rowok = 0, colok = 0;
        if (tok) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                rowok |= (4 * ty - 1 + i >= 0 && 4 * ty - 1 + i < a.H) << i;
                colok |= (4 * tx - 1 + i >= 0 && 4 * tx - 1 + i < a.W) << i;
            }
        }
        const int ly = (tl - img * bt) / a.bw, lx = (tl - img * bt) - ly * a.bw;
        const int pbase = (img * a.rh + 4 * ly) * a.rw + 4 * lx;  // region pixel of patch (0, 0)
        // byte offsets (within a raw buffer) of the 36 patch values; padding
        // and invalid tiles read the buffer's zero pixel
        int xo[36];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j)
                xo[6 * i + j] = ((rowok >> i) & (colok >> j) & 1) ? wf4_px(pbase + i * a.rw + j) * 32 + ch * 4
                                                                  : WF4_RAWZ;
        if (pt < 3 * 16) reinterpret_cast<float *>(Raw + (pt >> 4) * WF4_RAW + WF4_RAWZ)[pt & 15] = 0.f;
        float *aw = nullptr;
        auto transform = [&](int ks) {
            const char *rb = Raw + (ks % 3) * WF4_RAW;
            float xv[36];
#pragma unroll
            for (int q = 0; q < 36; ++q) xv[q] = *reinterpret_cast<const float *>(rb + xo[q]);
            aw = Abuf + (ks & 1) * (WF4_STAGE / 4) + wf4_idx(tl, ch);
#pragma unroll
            for (int p = 0; p < 6; ++p) {
                float r[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    float acc = 0.f;
#pragma unroll
                    for (int i = 0; i < 6; ++i)
                        if (WT::BT(p, i) != 0.f) acc = acc + WT::BT(p, i) * xv[6 * i + j];
                    r[j] = acc;
                }
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    float acc = 0.f;
#pragma unroll
                    for (int j = 0; j < 6; ++j)
                        if (WT::BT(q, j) != 0.f) acc = acc + r[j] * WT::BT(q, j);
                    aw[(6 * p + q) * (WF4_MT * WF4_KC)] = acc;
                }
            }
        };
        const bool work = !(a.dbg & 1);
        // prologue: raw K-steps 0, 1, 2 in flight; 0 and 1 landed before P0
        dma(0);
        if (KS > 1) dma(1);
        if (KS > 2) {
            dma(2);
            if (nd == 7) MDX_WAIT_VMN(7); else if (nd == 6) MDX_WAIT_VMN(6); else if (nd == 5) MDX_WAIT_VMN(5);
            else if (nd == 4) MDX_WAIT_VMN(4); else if (nd == 3) MDX_WAIT_VMN(3); else if (nd == 2) MDX_WAIT_VMN(2);
            else if (nd == 1) MDX_WAIT_VMN(1); else MDX_WAIT_VMN(0);
        } else {
            MDX_WAIT_VMN(0);
        }
        __syncthreads();  // P0: raw 0 (and 1) visible
        transform(0);
        __syncthreads();  // P1: A stage 0 visible
        for (int k = 0; k < KS; ++k) {
            // transform K-step k + 1 (raw visible since the last barrier), put
            // K-step k + 3 in flight, then make sure k + 2 has landed
            if (work && k + 1 < KS) transform(k + 1);
            if (k + 3 < KS) {
                dma(k + 3);
                if (nd == 7) MDX_WAIT_VMN(7); else if (nd == 6) MDX_WAIT_VMN(6); else if (nd == 5) MDX_WAIT_VMN(5);
                else if (nd == 4) MDX_WAIT_VMN(4); else if (nd == 3) MDX_WAIT_VMN(3); else if (nd == 2) MDX_WAIT_VMN(2);
                else if (nd == 1) MDX_WAIT_VMN(1); else MDX_WAIT_VMN(0);
            } else {
                MDX_WAIT_VMN(0);
            }
            __syncthreads();
        }
        // ---- epilogue store phase: (tile th * 16 + etl, channel nh * 16 + ech)
        const int ech = pt & 15, etl = pt >> 4;
        const float *red = reinterpret_cast<const float *>(smem);
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
            for (int nh = 0; nh < 2; ++nh) {
                __syncthreads();  // the quarter's row slots are in LDS
                int tn, tty, ttx, timg;
                if (slot_tile(th * 16 + etl, tn, tty, ttx, timg)) {
                    const int co = nb * WF4_NC + nh * 16 + ech;
                    const float bv = a.bias ? a.bias[co] : 0.f;
                    // red[slot 8][j 4][tile 16][ch 16]; rows 1 and 4 are split over two slots
                    float t[6][4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float sl[8];
#pragma unroll
                        for (int q = 0; q < 8; ++q) sl[q] = red[((q * 4 + j) * 16 + etl) * 16 + ech];
                        t[0][j] = sl[0];
                        t[1][j] = sl[1] + sl[2];
                        t[2][j] = sl[3];
                        t[3][j] = sl[4];
                        t[4][j] = sl[5] + sl[6];
                        t[5][j] = sl[7];
                    }
                    float *ob = a.out + ((long long)tn * a.H * a.W) * a.Cout + co;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int oy = 4 * tty + i;
                        if (oy >= a.H) continue;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int ox = 4 * ttx + j;
                            if (ox >= a.W) continue;
                            float v = bv;
#pragma unroll
                            for (int r = 0; r < 6; ++r)
                                if (WT::AT(i, r) != 0.f) v = v + WT::AT(i, r) * t[r][j];
                            if (a.relu) v = v > 0.f ? v : 0.f;
                            ob[((long long)oy * a.W + ox) * a.Cout] = v;
                        }
                    }
                }
                __syncthreads();  // quarter stored: red free
            }
    } else {
        // ================= consumers =================
        float4v acc[WF4_XW][2][2];
#pragma unroll
        for (int x = 0; x < WF4_XW; ++x)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[x][i][j] = float4v{0.f, 0.f, 0.f, 0.f};
        const int f0 = wf4_idx(lane & 15, 2 * (lane >> 4));
        const int f1 = wf4_idx(16 + (lane & 15), 2 * (lane >> 4));
        // B fragments: point xi's 1-KiB piece of K-step ks at ((nb KS + ks) 36 + xi) KiB
        const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc((void *)a.Up, (short)0, a.ubytes,
                                                                            0x00020000);
        const unsigned ub = (unsigned)(nb * KS) * 36u * 1024u + (unsigned)(wid * WF4_XW) * 1024u + (unsigned)lane * 16u;
        float4v bq[WF4_XW];
#pragma unroll
        for (int x = 0; x < WF4_XW; ++x)
            bq[x] = __builtin_bit_cast(float4v, __builtin_amdgcn_raw_buffer_load_b128(ru, ub + x * 1024u, 0, 0));
        __syncthreads();  // P0
        __syncthreads();  // P1
        const bool mma = !(a.dbg & 2);
        for (int k = 0; k < KS; ++k) {
            const float *Aw = Abuf + (k & 1) * (WF4_STAGE / 4) + wid * WF4_XW * (WF4_MT * WF4_KC);
            const unsigned nxt = ub + (unsigned)(k + 1 < KS ? k + 1 : k) * 36u * 1024u;
            if (mma) {
                float2 fa[2][2];
                fa[0][0] = *reinterpret_cast<const float2 *>(Aw + f0);
                fa[0][1] = *reinterpret_cast<const float2 *>(Aw + f1);
#pragma unroll
                for (int x = 0; x < WF4_XW; ++x) {
                    const int c = x & 1;
                    if (x + 1 < WF4_XW) {
                        const int o = (x + 1) * (WF4_MT * WF4_KC);
                        fa[c ^ 1][0] = *reinterpret_cast<const float2 *>(Aw + o + f0);
                        fa[c ^ 1][1] = *reinterpret_cast<const float2 *>(Aw + o + f1);
                    }
                    const float4v b = bq[x];
                    __builtin_amdgcn_sched_barrier(0);
                    // point x's B for K-step k + 1 into the freed registers
                    bq[x] = __builtin_bit_cast(float4v,
                                               __builtin_amdgcn_raw_buffer_load_b128(ru, nxt + x * 1024u, 0, 0));
#pragma unroll
                    for (int th = 0; th < 2; ++th) {
                        acc[x][th][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[c][th].x, b[0], acc[x][th][0], 0, 0, 0);
                        acc[x][th][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[c][th].x, b[2], acc[x][th][1], 0, 0, 0);
                    }
#pragma unroll
                    for (int th = 0; th < 2; ++th) {
                        acc[x][th][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[c][th].y, b[1], acc[x][th][0], 0, 0, 0);
                        acc[x][th][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[c][th].y, b[3], acc[x][th][1], 0, 0, 0);
                    }
                }
            }
            __syncthreads();  // stage k & 1 read; stage (k + 1) & 1 filled
        }
        // ---- epilogue: row-slot partials of quarter (th, nh) -> red
        // red[slot 8][j 4][tile 16][ch 16]: wave c writes slots 2c, 2c + 1
        float *red = reinterpret_cast<float *>(smem);
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
            for (int nh = 0; nh < 2; ++nh) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int tt = 4 * (lane >> 4) + r, cc = lane & 15;
                    float s0[4], s1[4];
                    // points 9 wid + x: slot 2 wid holds its first row, slot 2 wid + 1 its second
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        s0[j] = 0.f;
                        s1[j] = 0.f;
                    }
                    switch (wid) {
#define MDX_WF4_ROWS(W)                                                                              \
    case W:                                                                                          \
        _Pragma("unroll") for (int x = 0; x < WF4_XW; ++x) {                                         \
            constexpr int r0 = (W * WF4_XW) / 6;                                                     \
            const int xi = W * WF4_XW + x, ra = xi / 6, cb = xi % 6;                                 \
            const float m = acc[x][th][nh][r];                                                       \
            _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                          \
                if (WT::AT(j, cb) == 0.f) continue;                                                  \
                if (ra == r0) s0[j] = s0[j] + WT::AT(j, cb) * m; else s1[j] = s1[j] + WT::AT(j, cb) * m; \
            }                                                                                        \
        }                                                                                            \
        break;
                        MDX_WF4_ROWS(0)
                        MDX_WF4_ROWS(1)
                        MDX_WF4_ROWS(2)
                        MDX_WF4_ROWS(3)
#undef MDX_WF4_ROWS
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        red[(((2 * wid) * 4 + j) * 16 + tt) * 16 + cc] = s0[j];
                        red[(((2 * wid + 1) * 4 + j) * 16 + tt) * 16 + cc] = s1[j];
                    }
                }
                __syncthreads();  // the quarter's row slots are in LDS
                __syncthreads();  // quarter stored: red free
            }
    }
}

// k_wino_in (conv.hip) with two channels per thread (8-B loads and stores: half the
// memory instructions per byte); the same sums per channel, in the same order.
// B^T d is formed in place column by column, then each row of (B^T d) B is
// stored as it is formed (d plus one 8-entry temporary stay live)
template <int M>
__global__ __launch_bounds__(256) void k_wino_in2(const float *__restrict__ x, int N, int H, int W, int C, int TH,
                                                  int TW, float *__restrict__ V) {
    constexpr int A = WinoT<M>::A;
    const int t = blockIdx.x;
    const int c = 2 * (blockIdx.y * blockDim.x + threadIdx.x);
    if (c >= C) return;
    const long long T = (long long)N * TH * TW;
    const long long xs = T * C;
    const int tx = t % TW, r = t / TW;
    const int ty = r % TH, n = r / TH;
    const int y0 = M * ty - 1, x0 = M * tx - 1;
    const float *xb = x + (long long)n * H * W * C + c;
    float2 d[A][A];
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {
            const int yy = y0 + i, xx = x0 + j;
            d[i][j] = (yy >= 0 && yy < H && xx >= 0 && xx < W)
                          ? *reinterpret_cast<const float2 *>(xb + ((long long)yy * W + xx) * C)
                          : make_float2(0.f, 0.f);
        }
#pragma unroll
    for (int j = 0; j < A; ++j) {  // B^T d, column j, in place
        float2 col[A];
#pragma unroll
        for (int i = 0; i < A; ++i) {
            float ax = 0.f, ay = 0.f;
#pragma unroll
            for (int k = 0; k < A; ++k)
                if (WinoT<M>::BT(i, k) != 0.f) {
                    ax = ax + WinoT<M>::BT(i, k) * d[k][j].x;
                    ay = ay + WinoT<M>::BT(i, k) * d[k][j].y;
                }
            col[i] = make_float2(ax, ay);
        }
#pragma unroll
        for (int i = 0; i < A; ++i) d[i][j] = col[i];
    }
    float *vo = V + (long long)t * C + c;
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {  // (B^T d) B
            float ax = 0.f, ay = 0.f;
#pragma unroll
            for (int k = 0; k < A; ++k)
                if (WinoT<M>::BT(j, k) != 0.f) {
                    ax = ax + d[i][k].x * WinoT<M>::BT(j, k);
                    ay = ay + d[i][k].y * WinoT<M>::BT(j, k);
                }
            *reinterpret_cast<float2 *>(vo + (A * i + j) * xs) = make_float2(ax, ay);
        }
}

void launch_wino_in2(int m, dim3 grid, unsigned bd, hipStream_t s, const float *x, int N, int H, int W, int C,
                     int TH, int TW, float *V) {
    if (m == 2)
        hipLaunchKernelGGL(k_wino_in2<2>, grid, dim3(bd), 0, s, x, N, H, W, C, TH, TW, V);
    else if (m == 4)
        hipLaunchKernelGGL(k_wino_in2<4>, grid, dim3(bd), 0, s, x, N, H, W, C, TH, TW, V);
    else
        hipLaunchKernelGGL(k_wino_in2<6>, grid, dim3(bd), 0, s, x, N, H, W, C, TH, TW, V);
}

}  // namespace mdx

using namespace mdx;

// fused F(4,3) policy of the model handle: 0 never (default: measured slower
// than the three-launch path on every layer but res2's 64-channel ones, see
// DESIGN.md), 1 when the launch has at least min_wgs workgroups, 2 whenever
// the shape allows
static int g_wino_fused = 0, g_wino_fused_min_wgs = 384;
extern "C" int mdx_conv_set_winograd_fused(int mode, int min_wgs) {
    const int old = g_wino_fused;
    g_wino_fused = mode;
    if (min_wgs > 0) g_wino_fused_min_wgs = min_wgs;
    return old;
}
static bool wf4_geometry(int N, int TH, int TW, int &bh, int &bw, int &ipb);
static bool wino_fused_shape_ok(int N, int H, int W, int Cin, int Cout) {
    int bh, bw, ipb;
    if (N > 0 && H > 0 && W > 0 && !wf4_geometry(N, (H + 3) / 4, (W + 3) / 4, bh, bw, ipb)) return false;
    return N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && Cin % WF4_KC == 0 && Cout % WF4_NC == 0 &&
           (long long)N * H * W * Cin * 4 < (1ll << 31) && 36ll * Cout * Cin * 4 < (1ll << 31) &&
           (long long)N * ((H + 3) / 4) * ((W + 3) / 4) < (1ll << 31);
}
extern "C" int mdx_winograd_fused_eligible(int N, int H, int W, int Cin, int Cout) {
    if (!g_wino_fused || mdx_conv_fp32_split() || !wino_fused_shape_ok(N, H, W, Cin, Cout)) return 0;
    int bh, bw, ipb;
    wf4_geometry(N, (H + 3) / 4, (W + 3) / 4, bh, bw, ipb);
    const long long blocks = ceil_div(N, ipb) * ceil_div((H + 3) / 4, bh) * ceil_div((W + 3) / 4, bw);
    return g_wino_fused == 2 || blocks * (Cout / WF4_NC) >= g_wino_fused_min_wgs;
}

// U [36][Cout][Cin] -> the consumers' B fragments: [Cout / 32][Cin / 8][36]
// pieces of [64 lanes][4]: lane l = (channel n = l & 15, k-pair kp = l >> 4)
// holds U at (n, 2 kp), (n, 2 kp + 1), (n + 16, 2 kp), (n + 16, 2 kp + 1)
extern "C" int mdx_winograd_pack_f4(const float *U, int Cout, int Cin, float *Up) {
    MDX_REQUIRE(U && Up && Cout > 0 && Cin > 0 && Cout % WF4_NC == 0 && Cin % WF4_KC == 0,
                "mdx_winograd_pack_f4: Cout %% 32 == 0 and Cin %% 8 == 0 required");
    const int KS = Cin / WF4_KC;
    for (int nb = 0; nb < Cout / WF4_NC; ++nb)
        for (int ks = 0; ks < KS; ++ks)
            for (int xi = 0; xi < 36; ++xi) {
                float *dst = Up + ((long long)(nb * KS + ks) * 36 + xi) * 256;
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 4; ++e) {
                        const int n = nb * WF4_NC + (l & 15) + 16 * (e >> 1), k = ks * WF4_KC + 2 * (l >> 4) + (e & 1);
                        dst[l * 4 + e] = U[((long long)xi * Cout + n) * Cin + k];
                    }
            }
    return MDX_OK;
}

// block geometry for a TH x TW tile grid: bh x bw tiles (bh bw = 32) of one
// image, or whole small images ipb at a time; fewest empty slots, then the
// smallest raw region; false when no region fits the raw buffer
static bool wf4_geometry(int N, int TH, int TW, int &bh, int &bw, int &ipb) {
    long long best = -1, bestpx = 0;
    if (TH * TW <= 16) {
        bh = TH;
        bw = TW;
        ipb = std::max(1, std::min(32 / (TH * TW), N));
        return ipb * (4 * bh + 2) * (4 * bw + 2) <= WF4_MAXPX;
    }
    ipb = 1;
    for (int c = 0; c < 6; ++c) {
        const int h = 1 << c, w = 32 >> c;
        const long long px = (4ll * h + 2) * (4 * w + 2);
        if (px > WF4_MAXPX) continue;
        const long long waste = (long long)((TH + h - 1) / h) * ((TW + w - 1) / w) * 32 - (long long)TH * TW;
        if (best < 0 || waste < best || (waste == best && px < bestpx)) {
            best = waste;
            bestpx = px;
            bh = h;
            bw = w;
        }
    }
    return best >= 0;
}

extern "C" int mdx_conv3x3_winograd_fused(const float *x, int N, int H, int W, int Cin, const float *Up,
                                          const float *bias, int Cout, int relu, float *out, mdx_stream_t stream) {
    MDX_REQUIRE(x && Up && out, "mdx_conv3x3_winograd_fused: null pointer");
    MDX_REQUIRE(wino_fused_shape_ok(N, H, W, Cin, Cout),
                "mdx_conv3x3_winograd_fused: Cin %% 8 == 0, Cout %% 32 == 0 and operands < 2 GiB required");
    hipStream_t s = as_stream(stream);
    WinoF4Args f{};
    f.x = x; f.Up = Up; f.bias = bias; f.out = out;
    f.N = N; f.H = H; f.W = W; f.Cin = Cin; f.Cout = Cout;
    f.TH = (H + 3) / 4; f.TW = (W + 3) / 4;
    f.relu = relu;
    MDX_REQUIRE(wf4_geometry(N, f.TH, f.TW, f.bh, f.bw, f.ipb),
                "mdx_conv3x3_winograd_fused: no tile block fits (map %dx%d)", H, W);
    f.nbx = (f.TW + f.bw - 1) / f.bw;
    f.nby = (f.TH + f.bh - 1) / f.bh;
    f.tblocks = (int)ceil_div(N, f.ipb) * f.nbx * f.nby;
    f.nblocks = Cout / WF4_NC;
    f.rh = 4 * f.bh + 2;
    f.rw = 4 * f.bw + 2;
    f.npx = f.ipb * f.rh * f.rw;
    f.ndma = (2 * f.npx + 63) / 64;
    f.xbytes = (int)((long long)N * H * W * Cin * 4);
    f.ubytes = (int)(36ll * Cout * Cin * 4);
    static const int dbg = getenv("MDX_WF4_DEBUG") ? atoi(getenv("MDX_WF4_DEBUG")) : 0;
    f.dbg = dbg;
    WinoProbe *probe = wino_probe_current();
    if (probe) (void)hipEventRecord(probe->ev[2], s);
    hipLaunchKernelGGL(k_wino_f4, dim3((unsigned)(f.tblocks * f.nblocks)), dim3(WF4_THREADS), WF4_LDS, s, f);
    if (probe) {
        (void)hipEventRecord(probe->ev[3], s);
        probe->gemm_kernel = MDX_CONV_KERNEL_WINO_FUSED;
    }
    set_last_plan(MDX_CONV_KERNEL_WINO_FUSED, 1);
    MDX_CHECK_LAUNCH("mdx_conv3x3_winograd_fused");
    return MDX_OK;
}
