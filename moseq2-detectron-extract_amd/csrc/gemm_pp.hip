// fp32 GEMM for the pointwise layers (1x1 convs with any stride, FC layers,
// the batched Winograd tile-point GEMMs) on v_mfma_f32_16x16x4_f32, as two
// wave groups in ping-pong:
//
//   out[m][n] = act( sum_k A[m][k] * B[n][k] + bias[n] (+ res[m][n]) )
//   A row m = the NHWC pixel of output row m (stride s), B = weights [N][K].
//
// Tile 256 x 256 per 512-thread workgroup (one per CU), 8 waves: group g =
// wid >> 2 owns output rows 128 g .. 128 g + 127, wave (g, wn) a 128 x 64
// block = 8 x 4 MFMA tiles (128 fp32 accumulators per lane).  K in tiles of
// 32 floats (128-B LDS rows), A and B of a K-tile staged by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave instruction, 8 per wave and
// K-tile), two K-tile buffers (128 KiB).
//
// A K-tile is two phases (16-deep halves).  Every phase is, per wave,
//   R: 12 ds_read_b128 fragments (8 A + 4 B) [+ DMA issue / wait] lgkmcnt(0)
//      barrier
//   M: 128 MFMAs barrier
// and group 1 runs one barrier behind group 0, so between any two barriers
// one wave of every SIMD multiplies while the other reads: the MFMA pipe
// never waits for a fragment read, a barrier or an LDS-DMA, and a single
// fragment set per wave suffices (the 256-register budget of two waves per
// SIMD: 128 accumulators + 48 fragment registers).
//
// Global barrier b opens interval b.  Group 0 runs R(p) in interval 2p and
// M(p) in 2p + 1; group 1 R(p) in 2p + 1 and M(p) in 2p + 2.  K-tile t is
// phases 2t, 2t + 1 in buffer t & 1:
//   * its last reads (phase 2t + 1) retire (lgkmcnt(0)) before barriers
//     4t + 3 (group 0) and 4t + 4 (group 1);
//   * the DMA of K-tile t + 2 into the same buffer is issued in R(2t + 2),
//     intervals 4t + 4 / 4t + 5: after both (WAR);
//   * each wave waits for its own DMA of K-tile t + 1 (vmcnt(0): the only
//     vector-memory operations in the loop) in R(2t + 1), before barrier
//     4t + 3 / 4t + 4, and the first read of K-tile t + 1 is group 0's
//     R(2t + 2) in interval 4t + 4: after both (RAW; LDS-DMA data is
//     ordered for ds_read only by the issuer's vmcnt and a barrier).
// Rows past M / N are clamped to the last row (their products only reach
// outputs that are never stored), so no load is predicated.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace mdx {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void *lds_t;

constexpr int PP_BM = 256, PP_BN = 256, PP_THREADS = 512;
constexpr int PP_BK = 32;                  // floats per K-tile (one 128-B LDS row)
constexpr int PP_ROWB = PP_BK * 4;
constexpr int PP_OPND = PP_BM * PP_ROWB;   // one operand of one K-tile: 32 KiB
constexpr int PP_BUF = 2 * PP_OPND;        // A then B
constexpr int PP_LDS = 2 * PP_BUF;         // two K-tile buffers: 128 KiB

// s_waitcnt through the builtin (visible to the compiler's waitcnt pass),
// fenced so no memory operation moves across it.  gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14
#define PP_WAIT_VM0()                                                                            \
    do {                                                                                         \
        asm volatile("" ::: "memory");                                                           \
        __builtin_amdgcn_s_waitcnt(0x0F70);                                                      \
        asm volatile("" ::: "memory");                                                           \
    } while (0)
#define PP_WAIT_LGKM0()                                                                          \
    do {                                                                                         \
        asm volatile("" ::: "memory");                                                           \
        __builtin_amdgcn_s_waitcnt(0xC07F);                                                      \
        asm volatile("" ::: "memory");                                                           \
    } while (0)

__device__ __forceinline__ void barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <bool M32, bool PRIO>
__global__ __launch_bounds__(PP_THREADS, 1) void k_gemm_pp(GemmPP a) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass cannot type the 32x32 accumulators; it only needs the stub)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (gridDim.z > 1) {  // batch entry z (the Winograd tile points)
        const long long z = blockIdx.z;
        a.x += z * a.bsx;
        a.w += z * a.bsw;
        a.out += z * a.bso;
    }
    // XCD-contiguous remap of the linear block id (bijective): the column
    // tiles of a row panel run on one XCD's L2
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * PP_BM, n0 = tn * PP_BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wn = wid & 3;

    // ---- LDS-DMA sources: instruction j of wave w fills tile rows
    // 32 w + 8 j .. + 7 of A (and of B); lane l writes row + (l >> 3), 16-B
    // slot l & 7, which holds the row's logical piece (l & 7) ^ ((row >> 1) & 7)
    const float *asrc[4], *bsrc[4];
    const int ohw = a.OH * a.OW;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = 32 * wid + 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int gm = min(m0 + r, a.M - 1), gn = min(n0 + r, a.N - 1);
        long long pix;
        if (a.stride == 1) {
            pix = gm;
        } else {
            const int b = gm / ohw, rem = gm - b * ohw, oy = rem / a.OW, ox = rem - oy * a.OW;
            pix = ((long long)b * a.H + (long long)oy * a.stride) * a.W + (long long)ox * a.stride;
        }
        asrc[j] = a.x + pix * a.K + 4 * c;
        bsrc[j] = a.w + (long long)gn * a.K + 4 * c;
    }
    char *const adst = smem + (32 * wid) * PP_ROWB;  // wave-uniform DMA bases (+ buffer, + j KiB)
    auto dma = [&](int t) {
        char *d = adst + (t & 1) * PP_BUF;
        const int k = t * PP_BK;
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_amdgcn_global_load_lds(asrc[j] + k, (lds_t)(d + j * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds(bsrc[j] + k, (lds_t)(d + PP_OPND + j * 1024), 16, 0, 0);
    };

    // ---- fragments.  16x16x4 (M32 false): lane l reads row (l & 15) of each
    // 16-row tile, logical piece 4 s + (l >> 4) of the phase's half s; element
    // e of the piece is the k of MFMA e (the same permutation of k on both
    // operands).  32x32x2 (M32): lane l reads row (l & 31) of each 32-row
    // tile, pieces 4 s + 2 u + (l >> 5), u = 0, 1.
    constexpr int FR = M32 ? 32 : 16;
    const int fr = lane & (FR - 1), fsw = (fr >> 1) & 7, fh = M32 ? lane >> 5 : lane >> 4;
    const char *abase = smem + (grp * 128 + fr) * PP_ROWB;
    const char *bbase = smem + PP_OPND + (wn * 64 + fr) * PP_ROWB;
    constexpr int TI = 128 / FR, TJ = 64 / FR, NU = M32 ? 2 : 1;
    f4 fa[TI][NU], fb[TJ][NU];
    auto read_frags = [&](int buf, int s) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int piece = M32 ? 4 * s + 2 * u + fh : 4 * s + fh;
            const int off = buf * PP_BUF + ((piece ^ fsw) << 4);
#pragma unroll
            for (int j = 0; j < TJ; ++j) fb[j][u] = *reinterpret_cast<const f4 *>(bbase + off + j * FR * PP_ROWB);
#pragma unroll
            for (int i = 0; i < TI; ++i) fa[i][u] = *reinterpret_cast<const f4 *>(abase + off + i * FR * PP_ROWB);
        }
    };

    using acc_t = typename std::conditional<M32, f16, f4>::type;
    acc_t acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = acc_t{};

    const int KT = a.K / PP_BK;
    dma(0);
    PP_WAIT_VM0();
    barrier();               // K-tile 0 in LDS
    if (grp == 1) barrier();  // group 1 one barrier behind
    for (int t = 0; t < KT; ++t) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // R
            read_frags(t & 1, s);
            if (t + 1 < KT) {
                if (s == 0) dma(t + 1);
                else PP_WAIT_VM0();
            }
            PP_WAIT_LGKM0();
            barrier();
            // M: row tile outermost (the MFMAs of tile i need fa[i] only)
            if (PRIO) __builtin_amdgcn_s_setprio(1);
            if constexpr (M32) {
#pragma unroll
                for (int u = 0; u < NU; ++u)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int i = 0; i < TI; ++i)
#pragma unroll
                            for (int j = 0; j < TJ; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][u][e], fb[j][u][e], acc[i][j],
                                                                                 0, 0, 0);
            } else {
                // four independent accumulators between two into one
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][0][e], fb[j][0][e], acc[i][j], 0,
                                                                             0, 0);
            }
            if (PRIO) __builtin_amdgcn_s_setprio(0);
            barrier();
        }
    }
    if (grp == 0) barrier();  // every wave crosses the same number of barriers

    // ---- epilogue straight from the accumulators.  16x16: lane l holds rows
    // 4 (l >> 4) + r of each tile, column l & 15 (16 lanes store 64
    // contiguous bytes of a row); 32x32: rows (r & 3) + 8 (r >> 2) + 4 (l >> 5),
    // column l & 31 (128 contiguous bytes)
    constexpr int NR = M32 ? 16 : 4;
    const int rowb = m0 + grp * 128 + fh * 4;
    const int colb = n0 + wn * 64 + fr;
    float bj[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int gn = colb + FR * j;
        bj[j] = (a.bias && gn < a.N) ? a.bias[gn] : 0.f;
    }
    auto row_of = [&](int i, int r) { return rowb + FR * i + (M32 ? (r & 3) + 8 * (r >> 2) : r); };
    if (a.relu == 2) {  // diagnostics: no epilogue
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
        float rv[TJ][NR];
        if (a.res) {
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const int gm = row_of(i, r), gn = colb + FR * j;
                    rv[j][r] = (gm < a.M && gn < a.N) ? a.res[(long long)gm * a.N + gn] : 0.f;
                }
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int gm = row_of(i, r), gn = colb + FR * j;
                float v = acc[i][j][r] + bj[j];
                if (a.res) v += rv[j][r];
                if (a.relu) v = v > 0.f ? v : 0.f;
                if (gm < a.M && gn < a.N) a.out[(long long)gm * a.N + gn] = v;
            }
    }
#endif
}

// One wave per SIMD: 256 x 256 tile, 4 waves (2 x 2), wave tile 128 x 128 =
// 8 x 8 MFMA tiles (256 accumulators, in AGPRs), fragments double-buffered in
// VGPRs (the next half K-tile's 16 are read while the current 256 MFMAs
// issue), the next K-tile's LDS-DMA pieces and fragment reads interleaved one
// per 16 MFMAs, one barrier per K-tile (32 floats, two 16-deep halves).
constexpr int W1_THREADS = 256;
template <int UNUSED>
__global__ __launch_bounds__(W1_THREADS, 1) void k_gemm_w1(GemmPP a) {
#if defined(__HIP_DEVICE_COMPILE__)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (gridDim.z > 1) {
        const long long z = blockIdx.z;
        a.x += z * a.bsx;
        a.w += z * a.bsw;
        a.out += z * a.bso;
    }
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * PP_BM, n0 = tn * PP_BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    // DMA: instruction j (0..7) of wave w fills rows 64 w + 8 j .. + 7 of A and of B
    const float *asrc[8], *bsrc[8];
    const int ohw = a.OH * a.OW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int r = 64 * wid + 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int gm = min(m0 + r, a.M - 1), gn = min(n0 + r, a.N - 1);
        long long pix;
        if (a.stride == 1) {
            pix = gm;
        } else {
            const int b = gm / ohw, rem = gm - b * ohw, oy = rem / a.OW, ox = rem - oy * a.OW;
            pix = ((long long)b * a.H + (long long)oy * a.stride) * a.W + (long long)ox * a.stride;
        }
        asrc[j] = a.x + pix * a.K + 4 * c;
        bsrc[j] = a.w + (long long)gn * a.K + 4 * c;
    }
    char *const ddst = smem + (64 * wid) * PP_ROWB;
    auto dma_piece = [&](int t, int q) {  // q < 8: A rows, else B rows
        char *d = ddst + (t & 1) * PP_BUF + (q & 7) * 1024 + (q >= 8 ? PP_OPND : 0);
        const float *src = (q < 8 ? asrc[q & 7] : bsrc[q & 7]) + t * PP_BK;
        __builtin_amdgcn_global_load_lds(src, (lds_t)d, 16, 0, 0);
    };
    const int fr = lane & 15, fsw = (fr >> 1) & 7, fh = lane >> 4;
    const char *abase = smem + (wm * 128 + fr) * PP_ROWB;
    const char *bbase = smem + PP_OPND + (wn * 128 + fr) * PP_ROWB;
    f4 fa[2][8], fb[2][8];
    // fragment q (0..15) of half s of K-tile t into set `set`: q < 8 A row tile q, else B col tile q - 8
    auto read_frag = [&](int t, int s, int set, int q) {
        const int off = (t & 1) * PP_BUF + (((4 * s + fh) ^ fsw) << 4);
        if (q < 8)
            fa[set][q] = *reinterpret_cast<const f4 *>(abase + off + q * 16 * PP_ROWB);
        else
            fb[set][q - 8] = *reinterpret_cast<const f4 *>(bbase + off + (q - 8) * 16 * PP_ROWB);
    };
    f4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    // 16 MFMAs of group g (row tile i = g / 2, column tiles 4 (g & 1) .. + 3, e = 0..3) from fragment set `set`
    auto mma16 = [&](int set, int g) {
        const int i = g >> 1, j0 = 4 * (g & 1);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[set][i][e], fb[set][j0 + j][e],
                                                                       acc[i][j0 + j], 0, 0, 0);
    };
    const int KT = a.K / PP_BK;
#pragma unroll
    for (int q = 0; q < 16; ++q) dma_piece(0, q);
    PP_WAIT_VM0();
    barrier();
#pragma unroll
    for (int q = 0; q < 16; ++q) read_frag(0, 0, 0, q);
    for (int t = 0; t < KT; ++t) {
        const bool more = t + 1 < KT;
        // half 0 (set 0): per 16 MFMAs one DMA piece of K-tile t + 1 and one
        // fragment of half 1 (set 1)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (more) dma_piece(t + 1, g);
            read_frag(t, 1, 1, g);
            __builtin_amdgcn_sched_barrier(0);
            mma16(0, g);
        }
        // half 1 (set 1): 240 MFMAs, then the K-tile boundary (DMA landed,
        // barrier), the next K-tile's half-0 fragments, the last 16 MFMAs
#pragma unroll
        for (int g = 0; g < 15; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            mma16(1, g);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
            PP_WAIT_VM0();
            barrier();
#pragma unroll
            for (int q = 0; q < 16; ++q) read_frag(t + 1, 0, 0, q);
        }
        __builtin_amdgcn_sched_barrier(0);
        mma16(1, 15);
    }
    // epilogue straight from the accumulators
    const int rowb = m0 + wm * 128 + fh * 4;
    const int colb = n0 + wn * 128 + fr;
    float bj[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int gn = colb + 16 * j;
        bj[j] = (a.bias && gn < a.N) ? a.bias[gn] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gm = rowb + 16 * i + r, gn = colb + 16 * j;
                if (gm >= a.M || gn >= a.N) continue;
                float v = acc[i][j][r] + bj[j];
                if (a.res) v += a.res[(long long)gm * a.N + gn];
                if (a.relu) v = v > 0.f ? v : 0.f;
                a.out[(long long)gm * a.N + gn] = v;
            }
#endif
}

bool gemm_pp_eligible(int M, int N, int K) { return M > 0 && N > 0 && K >= PP_BK && K % PP_BK == 0; }

int gemm_pp(GemmPP a, int batch, hipStream_t s) {
    MDX_REQUIRE(a.x && a.w && a.out, "gemm_pp: null pointer");
    MDX_REQUIRE(gemm_pp_eligible(a.M, a.N, a.K), "gemm_pp: K=%d must be a positive multiple of %d", a.K, PP_BK);
    MDX_REQUIRE(batch >= 1, "gemm_pp: batch >= 1");
    if (a.stride <= 0) a.stride = 1;
    if (a.OH <= 0 || a.OW <= 0) {  // plain GEMM: row m is row m of A
        a.OH = a.M;
        a.OW = 1;
        a.H = a.M;
        a.W = 1;
        a.stride = 1;
    }
    a.tiles_n = (int)ceil_div(a.N, PP_BN);
    const long long tiles = ceil_div(a.M, PP_BM) * a.tiles_n;
    MDX_REQUIRE(tiles < (1ll << 31), "gemm_pp: too many tiles");
    a.tiles_total = (int)tiles;
    // MDX_PP_VAR (experiments): bit 0 s_setprio around the MFMA clusters,
    // bit 1 the 32x32x2 MFMA
    static const int var = getenv("MDX_PP_VAR") ? atoi(getenv("MDX_PP_VAR")) : 0;
    const dim3 grid((unsigned)a.tiles_total, 1, (unsigned)batch);
    if (var == 4)
        hipLaunchKernelGGL((k_gemm_w1<0>), grid, dim3(W1_THREADS), PP_LDS, s, a);
    else if (var == 1)
        hipLaunchKernelGGL((k_gemm_pp<false, true>), grid, dim3(PP_THREADS), PP_LDS, s, a);
    else if (var == 2)
        hipLaunchKernelGGL((k_gemm_pp<true, false>), grid, dim3(PP_THREADS), PP_LDS, s, a);
    else if (var == 3)
        hipLaunchKernelGGL((k_gemm_pp<true, true>), grid, dim3(PP_THREADS), PP_LDS, s, a);
    else
        hipLaunchKernelGGL((k_gemm_pp<false, false>), grid, dim3(PP_THREADS), PP_LDS, s, a);
    MDX_CHECK_LAUNCH("gemm_pp");
    return MDX_OK;
}

}  // namespace mdx

// C ABI (include/mdx.h): C[z] = act(A[z] . B[z]^T + bias (+ R[z])), row-major,
// A [M][K], B [N][K], C / R [M][N], z < batch at the given element strides.
extern "C" int mdx_gemm_f32(const float *A, const float *B, const float *bias, const float *residual, int relu,
                            float *C, int M, int N, int K, int batch, int64_t stride_a, int64_t stride_b,
                            int64_t stride_c, mdx_stream_t stream) {
    MDX_REQUIRE(M > 0 && N > 0 && K > 0, "mdx_gemm_f32: M, N, K must be positive");
    MDX_REQUIRE(batch == 1 || !residual, "mdx_gemm_f32: a residual needs batch == 1");
    mdx::GemmPP a{};
    a.x = A; a.w = B; a.bias = bias; a.res = residual; a.out = C;
    a.M = M; a.N = N; a.K = K; a.relu = relu;
    a.bsx = stride_a; a.bsw = stride_b; a.bso = stride_c;
    mdx::set_last_plan(MDX_CONV_KERNEL_PP256, 1);
    return mdx::gemm_pp(a, batch, mdx::as_stream(stream));
}
