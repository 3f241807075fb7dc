// Implicit-GEMM convolution / linear layer on MFMA (gfx950).
//
// Every convolution and FC layer of the Mask/Keypoint R-CNN forward (ResNet
// stem + bottlenecks, FPN lateral/output, RPN head, box FCs, mask and keypoint
// head convs, the 2x2/s2 mask deconv) is one launch of this kernel.
//
//   out[m][n] = act( sum_k A[m][k] * B[n][k] + bias[n] (+ res[m][n]) )
//   m = (b, oy, ox) output pixel (NHWC rows), n = output channel,
//   k = (ky, kx, ci), A gathered on the fly from the NHWC input (zero padding),
//   B = weights packed [Cout][KH][KW][Cin] (Cin fastest, BN folded).
//
// Tiles: 128(M) x 128(N) per 256-thread workgroup, 4 waves as 2x2, each wave
// 64x64 = 4x4 MFMA tiles of 16x16.  K staged through LDS in 128-byte rows
// (BK = 64 halves or 32 floats), double-buffered, register-staged global loads
// of 16 B per lane issued one K-step ahead.
//   fp16:  v_mfma_f32_16x16x32_f16  (fp32 accumulate)
//   fp32:  v_mfma_f32_16x16x4_f32   (exact fp32 products, fp32 accumulate)
// Output modes: NHWC, or the ConvTranspose(k=2,s=2) pixel shuffle (N = 4*Co).
// Blocks are remapped XCD-contiguously so the tiles that share an input row
// panel run on one XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "wino_tables.h"

namespace mdx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

template <typename T>
struct Prec;
template <>
struct Prec<_Float16> {
    static constexpr int BK = 64, VEC = 8;
};
template <>
struct Prec<float> {
    static constexpr int BK = 32, VEC = 4;
};

constexpr int BM = 128, BN = 128, CONV_THREADS = 256;
constexpr int ROWB = 128;          // bytes of K per LDS row
constexpr int PITCH = ROWB;        // row pitch (bytes); 16-B pieces XOR-swizzled by (row >> 1) & 7
constexpr int TILE_BYTES = BM * PITCH;

template <typename TO>
__device__ __forceinline__ void store_out(TO *p, float v) { *p = (TO)v; }

template <typename TO>
__device__ __forceinline__ void load8(const TO *p, float *v) {
    if constexpr (sizeof(TO) == 2) {
        const uint4 u = *reinterpret_cast<const uint4 *>(p);
        const TO *e = reinterpret_cast<const TO *>(&u);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)e[i];
    } else {
        const float4 x = *reinterpret_cast<const float4 *>(p), y = *reinterpret_cast<const float4 *>(p + 4);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    }
}
template <typename TO>
__device__ __forceinline__ void store8(TO *p, const float *v) {
    if constexpr (sizeof(TO) == 2) {
        uint4 u;
        TO *e = reinterpret_cast<TO *>(&u);
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = (TO)v[i];
        *reinterpret_cast<uint4 *>(p) = u;
    } else {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4 *>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

struct ConvArgs {
    const void *x;
    const void *w;
    const float *bias;  // [N] or null
    const void *res;    // [M][N] (same dtype as out) or null
    void *out;
    int H, W, Cin, Cout, KH, KW, stride, pad, OH, OW;
    int M, K;
    int relu;
    int out_mode;  // 0: NHWC, 1: deconv2x2 pixel shuffle
    int tiles_n, tiles_total;
    int ksplit, ksteps;  // split-K: K range of slice z = [z*ksteps*BK, (z+1)*ksteps*BK)
    float *part;         // [ksplit][M][Cout] fp32 partial sums (ksplit > 1)
    int xbytes, wbytes;  // operand sizes for the range-checked buffer descriptors (< 2^31)
    int rbytes;          // residual size (bytes), same purpose
    long long bsx, bsw, bso;  // batched GEMMs (grid.z): byte strides of x, w, out per batch entry
    // second A source (k_conv<..., DUAL>): K values [K1, K) of row m = (b, oy, ox)
    // come from x2[b][oy * stride2][ox * stride2][k - K1] (a bottleneck's
    // projection shortcut concatenated onto its conv3 GEMM)
    const void *x2;
    int K1, H2, W2, Cin2, stride2, x2bytes;
    int epi_direct;  // k_conv_sb: accumulators stored straight from registers (conv_body)
};

// bias / residual / ReLU on 8 consecutive output channels gn0.. of row gm and
// the 16-B store (or the scalar path for ragged channel counts)
template <typename TO>
__device__ __forceinline__ void finish8(const ConvArgs &a, int gm, int gn0, float *v) {
    TO *O = reinterpret_cast<TO *>(a.out);
    const TO *RS = reinterpret_cast<const TO *>(a.res);
    const int Co = a.out_mode == 1 ? a.Cout / 4 : a.Cout;
    const bool vec_ok = (a.Cout % 8) == 0 && (Co % 8) == 0;
    const int ohw = a.OH * a.OW;
    auto out_index = [&](int gn) -> long long {
        if (a.out_mode == 0) return (long long)gm * a.Cout + gn;
        const int q = gn / Co, co = gn - q * Co;
        const int b = gm / ohw, rem = gm - b * ohw;
        const int y = rem / a.OW, xx = rem - y * a.OW;
        return (((long long)b * (2 * a.OH) + 2 * y + (q >> 1)) * (2 * a.OW) + 2 * xx + (q & 1)) * Co + co;
    };
    if (vec_ok) {
        const long long obase = out_index(gn0);
        if (a.bias) {
            const float4 b0 = *reinterpret_cast<const float4 *>(a.bias + gn0);
            const float4 b1 = *reinterpret_cast<const float4 *>(a.bias + gn0 + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (RS) {
            float rv[8];
            load8<TO>(RS + obase, rv);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += rv[k];
        }
        if (a.relu) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
        }
        store8<TO>(O + obase, v);
    } else {
        for (int k = 0; k < 8; ++k) {
            const int gn = gn0 + k;
            if (gn >= a.Cout) break;
            const long long oi = out_index(gn);
            float x = v[k] + (a.bias ? a.bias[gn] : 0.f);
            if (RS) x += (float)RS[oi];
            if (a.relu) x = x > 0.f ? x : 0.f;
            store_out<TO>(O + oi, x);
        }
    }
}

// NQ epilogue items per lane, residual loads for all of them issued before any
// store (out and res may alias as far as the compiler knows, so a per-item
// load -> store sequence would serialise every load behind the previous
// store).  item(q, gm, gn0, src): row (-1 = skip), first channel, fp32 values.
template <typename TO, int NQ, typename F>
__device__ __forceinline__ void finish_batch(const ConvArgs &a, F item) {
    TO *O = reinterpret_cast<TO *>(a.out);
    const TO *RS = reinterpret_cast<const TO *>(a.res);
    const int Co = a.out_mode == 1 ? a.Cout / 4 : a.Cout;
    const bool vec_ok = (a.Cout % 8) == 0 && (Co % 8) == 0 && a.out_mode == 0;
    constexpr int RW = sizeof(TO) == 2 ? 1 : 2;  // 16-B words of 8 residual values
    uint4 rr[NQ][RW];
    int gms[NQ], gns[NQ];
    const float *srcs[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) item(q, gms[q], gns[q], srcs[q]);
    if (vec_ok && RS) {
        // residual rows through a range-checked descriptor: skipped items read
        // zeros past the end, so all loads issue back to back (no per-item
        // branch and vmcnt(0))
        const __amdgpu_buffer_rsrc_t rr_d = __builtin_amdgcn_make_buffer_rsrc((void *)a.res, (short)0, a.rbytes,
                                                                            0x00020000);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const unsigned off = gms[q] >= 0
                                     ? (unsigned)(((long long)gms[q] * a.Cout + gns[q]) * (long long)sizeof(TO))
                                     : 0xFFFFFFE0u;
#pragma unroll
            for (int w = 0; w < RW; ++w)
                rr[q][w] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rr_d, off + 16u * w, 0, 0));
        }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (gms[q] < 0) continue;
        const float *src = srcs[q];
        const float4 x0 = *reinterpret_cast<const float4 *>(src), x1 = *reinterpret_cast<const float4 *>(src + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        if (!vec_ok) {
            finish8<TO>(a, gms[q], gns[q], v);
            continue;
        }
        const int gn0 = gns[q];
        if (a.bias) {
            const float4 b0 = *reinterpret_cast<const float4 *>(a.bias + gn0);
            const float4 b1 = *reinterpret_cast<const float4 *>(a.bias + gn0 + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (RS) {
            const TO *e = reinterpret_cast<const TO *>(&rr[q][0]);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += (float)e[k];
        }
        if (a.relu) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
        }
        store8<TO>(O + (long long)gms[q] * a.Cout + gn0, v);
    }
}

// BN_: N tile (128 or 64).  4 waves as 2x2; wave tile (BM/2) x (BN_/2) =
// TI x TJ MFMA tiles of 16x16.
// PW: pointwise layer (1x1, no padding, any stride -- the 1x1 convs and the
// Winograd GEMMs): a row's A bytes start at its pixel's offset, so every load
// address is that offset + k, precomputed per row (no per-K-step bounds
// arithmetic, which compiles to exec-masked branches around every load).
// SB: one LDS stage instead of two (a second barrier per K-step before the
// next stage overwrites it), so three workgroups fit a CU instead of two
// (launched as k_conv_sb).
template <typename T, typename TO, int BN_, bool DUAL, bool PW, bool SB>
__device__ __forceinline__ void conv_body(ConvArgs &a) {
    constexpr int BK = Prec<T>::BK, VEC = Prec<T>::VEC;
    constexpr int TI = BM / 32, TJ = BN_ / 32;
    constexpr int A_TILE = BM * PITCH, B_TILE = BN_ * PITCH;
    constexpr int BLOADS = BN_ * 8 / CONV_THREADS;  // 16-B chunks of B per thread
    constexpr int STAGE = A_TILE + B_TILE;  // one K-step buffer: A tile then B tile
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *As = smem;                   // buffer b: A at b * STAGE, B at b * STAGE + A_TILE
    char *Bs = smem + A_TILE;          // (a one-step K needs buffer 0 only)
    if (gridDim.z > 1) {  // batch entry z of a batched GEMM
        const long long z = blockIdx.z;
        a.x = reinterpret_cast<const char *>(a.x) + z * a.bsx;
        a.w = reinterpret_cast<const char *>(a.w) + z * a.bsw;
        a.out = reinterpret_cast<char *>(a.out) + z * a.bso;
    }

    // XCD-contiguous remap of the linear block id (bijective)
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN_;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // ---- per-thread load descriptors: rows tid/8 + 32*i, 16-byte chunk tid%8
    const int kc = tid & 7;
    const int lrow = tid >> 3;
    int a_iy0[4], a_ix0[4];
    long long a_base[4];
    unsigned a2_off[DUAL ? 4 : 1];  // DUAL: byte offset of row i's pixel in x2
    bool a_ok[4];
    const int ohw = a.OH * a.OW;
    // stride-1 pointwise layers (the 1x1 convs without a stride, FC layers,
    // the Winograd GEMMs): row gm's pixel is pixel gm, no index division
    const bool pw1 = PW && !DUAL && a.stride == 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int gm = m0 + lrow + 32 * i;
        a_ok[i] = gm < a.M;
        if (pw1) {
            a_base[i] = a_ok[i] ? (long long)gm * a.Cin * (long long)sizeof(T) : 0xFFFFFFF0ll;
            continue;
        }
        const int gmc = a_ok[i] ? gm : 0;
        const int b = gmc / ohw, rem = gmc - b * ohw;
        const int oy = rem / a.OW, ox = rem - oy * a.OW;
        a_iy0[i] = oy * a.stride - a.pad;
        a_ix0[i] = ox * a.stride - a.pad;
        a_base[i] = (long long)b * a.H * a.W * a.Cin;
        if constexpr (DUAL)
            a2_off[i] = a_ok[i] ? (unsigned)((((long long)b * a.H2 + (long long)oy * a.stride2) * a.W2 +
                                              (long long)ox * a.stride2) * a.Cin2 * (long long)sizeof(T))
                                : 0xFFFFFFF0u;
        if constexpr (PW)  // (a_base[i] reused: byte offset of the row's pixel, or OOB)
            a_base[i] = a_ok[i] ? (long long)(((long long)b * a.H + (long long)oy * a.stride) * a.W +
                                              (long long)ox * a.stride) * a.Cin * (long long)sizeof(T)
                                : 0xFFFFFFF0ll;
    }
    const int kz = blockIdx.y;
    int kglob = kz * a.ksteps * BK + kc * VEC;
    int kci = kglob % a.Cin;
    int kr = kglob / a.Cin;
    int kkx = kr % a.KW, kky = kr / a.KW;

    // two register stages: the global loads of K-step t + 2 are issued while
    // step t is multiplied, and stored to LDS at the end of step t + 1
    uint4 ra[2][4], rb[2][BLOADS];

    // buffer loads through range-checked descriptors: a padding / out-of-range
    // piece gets an offset past the end and reads zeros from the hardware, so
    // every lane issues every load with no branch (a per-piece "load or zero"
    // select compiles to a branch + vmcnt(0) around each load)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)a.x, (short)0, a.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)a.w, (short)0, a.wbytes, 0x00020000);
    constexpr unsigned OOB = 0xFFFFFFF0u;
    // K a multiple of BK (every layer of the models): each issued piece lies
    // inside K, so a pointwise load is base + k with the out-of-range rows
    // based at 2^31 (past any buffer: sizes are < 2^31, and base + k does not
    // wrap), no per-load compare or select
    const bool kfull = PW && !DUAL && (a.K % BK) == 0;
    constexpr unsigned FAR = 0x80000000u;
    unsigned a_far[PW ? 4 : 1], b_far[BLOADS];
#pragma unroll
    for (int i = 0; i < (PW ? 4 : 1); ++i) a_far[i] = (unsigned)a_base[i] != OOB ? (unsigned)a_base[i] : FAR;
#pragma unroll
    for (int i = 0; i < BLOADS; ++i) {
        const int gn = n0 + lrow + 32 * i;
        b_far[i] = gn < a.Cout ? (unsigned)((long long)gn * a.K * (long long)sizeof(T)) : FAR;
    }
    auto load_global = [&](uint4 (&A)[4], uint4 (&Bv)[BLOADS]) {
        if (kfull) {
            const unsigned kb = (unsigned)(kglob * (int)sizeof(T));
#pragma unroll
            for (int i = 0; i < 4; ++i)
                A[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, a_far[PW ? i : 0] + kb, 0, 0));
#pragma unroll
            for (int i = 0; i < BLOADS; ++i)
                Bv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, b_far[i] + kb, 0, 0));
            return;
        }
        const bool kok = kglob < a.K;
        // (K1 is a multiple of BK: the whole K-step reads one source)
        if (DUAL && kglob >= a.K1) {
            const __amdgpu_buffer_rsrc_t rx2 =
                __builtin_amdgcn_make_buffer_rsrc((void *)a.x2, (short)0, a.x2bytes, 0x00020000);
            const unsigned kb = (unsigned)((kglob - a.K1) * (int)sizeof(T));
#pragma unroll
            for (int i = 0; i < (DUAL ? 4 : 0); ++i)
                A[i] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rx2, (kok && a2_off[i] != OOB) ? a2_off[i] + kb : OOB,
                                                                 0, 0));
        } else if constexpr (PW) {
            const unsigned kb = (unsigned)(kglob * (int)sizeof(T));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned ro = (unsigned)a_base[i];
                A[i] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, (kok && ro != OOB) ? ro + kb : OOB, 0, 0));
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int iy = a_iy0[i] + kky, ix = a_ix0[i] + kkx;
                const bool ok = kok && a_ok[i] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                const unsigned off =
                    (unsigned)((a_base[i] + ((long long)iy * a.W + ix) * a.Cin + kci) * (long long)sizeof(T));
                A[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : OOB, 0, 0));
            }
        }
#pragma unroll
        for (int i = 0; i < BLOADS; ++i) {
            const int gn = n0 + lrow + 32 * i;
            const unsigned off = (unsigned)(((long long)gn * a.K + kglob) * (long long)sizeof(T));
            Bv[i] = __builtin_bit_cast(uint4,
                                       __builtin_amdgcn_raw_buffer_load_b128(rw, (kok && gn < a.Cout) ? off : OOB, 0, 0));
        }
    };
    auto advance_k = [&]() {
        kglob += BK;
        if constexpr (PW) return;
        kci += BK;
        while (kci >= a.Cin) {
            kci -= a.Cin;
            if (++kkx == a.KW) {
                kkx = 0;
                ++kky;
            }
        }
    };
    // piece kc of row R lives at physical piece kc ^ ((R >> 1) & 7): the
    // fragment reads (rows l & 15, pieces 4 s + (l >> 4)) are then
    // bank-conflict-free for every ds_read_b128 lane group
    const int wpiece = (kc ^ ((lrow >> 1) & 7)) * 16;  // (lrow + 32 i) >> 1 & 7 == lrow >> 1 & 7
    auto store_lds = [&](int buf, const uint4 (&A)[4], const uint4 (&Bv)[BLOADS]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<uint4 *>(As + buf * STAGE + (lrow + 32 * i) * PITCH + wpiece) = A[i];
#pragma unroll
        for (int i = 0; i < BLOADS; ++i)
            *reinterpret_cast<uint4 *>(Bs + buf * STAGE + (lrow + 32 * i) * PITCH + wpiece) = Bv[i];
    };

    float4v acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    const int nk_all = (a.K + BK - 1) / BK;
    const int nk = min(a.ksteps, nk_all - kz * a.ksteps);
    load_global(ra[0], rb[0]);
    advance_k();
    store_lds(0, ra[0], rb[0]);
    if (nk > 1) {
        // (SB: one register stage; step 1 reuses set 0 once its store issued)
        load_global(ra[SB ? 0 : 1], rb[SB ? 0 : 1]);
        advance_k();
    }
    __syncthreads();
    // iteration kt: registers [kt & 1] are free (their step is in LDS), [(kt +
    // 1) & 1] hold step kt + 1
    auto kstep = [&](int kt, uint4 (&Ai)[4], uint4 (&Bi)[BLOADS], const uint4 (&As_)[4],
                     const uint4 (&Bs_)[BLOADS]) {
        const int cur = SB ? 0 : (kt & 1);
        if (!SB && kt + 2 < nk) {
            load_global(Ai, Bi);
            advance_k();
        }
        const char *Ab = As + cur * STAGE + (wm * (BM / 2) + (lane & 15)) * PITCH;
        const char *Bb = Bs + cur * STAGE + (wn * (BN_ / 2) + (lane & 15)) * PITCH;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int koff = ((4 * s + (lane >> 4)) ^ ((lane & 15) >> 1)) * 16;
            if constexpr (sizeof(T) == 2) {
                half8 af[TI], bf[TJ];
#pragma unroll
                for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const half8 *>(Ab + i * 16 * PITCH + koff);
#pragma unroll
                for (int j = 0; j < TJ; ++j) bf[j] = *reinterpret_cast<const half8 *>(Bb + j * 16 * PITCH + koff);
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
            } else {
                // B fragments first and the row tile outermost: the MFMAs of
                // tile i start once bf and af[i] have arrived (per accumulator
                // the e order is unchanged: bit-identical sums)
                float4v af[TI], bf[TJ];
#pragma unroll
                for (int j = 0; j < TJ; ++j) bf[j] = *reinterpret_cast<const float4v *>(Bb + j * 16 * PITCH + koff);
#pragma unroll
                for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const float4v *>(Ab + i * 16 * PITCH + koff);
                // (row tiles in groups of IG so >= 4 independent MFMAs separate
                // two into one accumulator)
                constexpr int IG = TJ >= 4 ? 1 : 4 / TJ;
#pragma unroll
                for (int i0 = 0; i0 < TI; i0 += IG)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int i = i0; i < i0 + IG; ++i)
#pragma unroll
                            for (int j = 0; j < TJ; ++j)
                                acc[i][j] =
                                    __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
            }
        }
        if constexpr (SB) {
            // one LDS stage, one register stage: [MFMAs of kt] barrier [store
            // kt + 1, then load kt + 2 into the same registers] barrier
            __syncthreads();  // every wave is done reading the stage
            if (kt + 1 < nk) store_lds(0, Ai, Bi);
            if (kt + 2 < nk) {
                load_global(Ai, Bi);
                advance_k();
            }
        } else if (kt + 1 < nk) {
            store_lds(cur ^ 1, As_, Bs_);
        }
        __syncthreads();
    };
    int kt = 0;
    if constexpr (SB) {
        for (; kt < nk; ++kt) kstep(kt, ra[0], rb[0], ra[0], rb[0]);
    } else {
    for (; kt + 1 < nk; kt += 2) {
        kstep(kt, ra[0], rb[0], ra[1], rb[1]);
        kstep(kt + 1, ra[1], rb[1], ra[0], rb[0]);
    }
    if (kt < nk) kstep(kt, ra[0], rb[0], ra[1], rb[1]);
    }

    // ---- direct epilogue (a.epi_direct: fp32 NHWC out, no split-K): every
    // lane adds bias / residual / ReLU to its own accumulators and stores
    // them, 16 lanes writing 64 contiguous bytes of a row -- no LDS image and
    // no barrier.  The residuals are all loaded before any store (out and
    // res may alias)
    // (scalar adds written out: the packed forms the compiler picks for a
    // broadcast bias are not among the cleared ones, _isa_lint.CLEARED)
    auto sadd = [](float x, float y) {
        float d;
        asm("v_add_f32 %0, %1, %2" : "=v"(d) : "v"(x), "v"(y));
        return d;
    };
    if constexpr (sizeof(TO) == 4) {
        if (a.epi_direct && a.ksplit == 1 && a.out_mode == 0) {
            TO *O = reinterpret_cast<TO *>(a.out);
            const int rowb = m0 + wm * (BM / 2) + (lane >> 4) * 4;
            const int colb = n0 + wn * (BN_ / 2) + (lane & 15);
            float bj[TJ];
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int gn = colb + 16 * j;
                bj[j] = (a.bias && gn < a.Cout) ? a.bias[gn] : 0.f;
            }
            if (a.bias) {
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = sadd(acc[i][j][r], bj[j]);
            }
            if (a.res) {
                const __amdgpu_buffer_rsrc_t rr =
                    __builtin_amdgcn_make_buffer_rsrc((void *)a.res, (short)0, a.rbytes, 0x00020000);
                float rv[TI][TJ][4];
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int gm = rowb + 16 * i + r, gn = colb + 16 * j;
                            const unsigned off =
                                (gm < a.M && gn < a.Cout) ? (unsigned)(((long long)gm * a.Cout + gn) * 4) : OOB;
                            rv[i][j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, off, 0, 0));
                        }
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = sadd(acc[i][j][r], rv[i][j][r]);
            }
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int gm = rowb + 16 * i + r, gn = colb + 16 * j;
                        float v = acc[i][j][r];
                        if (a.relu) v = v > 0.f ? v : 0.f;
                        if (gm < a.M && gn < a.Cout) O[(long long)gm * a.Cout + gn] = v;
                    }
            return;
        }
    }

    // ---- epilogue, in two halves of BM/2 rows (the LDS image is half the
    // tile, so a one-step-K launch fits 4 workgroups per CU): the waves owning
    // the half write their accumulators to LDS (fp32, row-major), then all
    // threads apply bias / residual / ReLU and store 8 consecutive output
    // channels per 16-byte store
    constexpr int CP = BN_ + 4;  // fp32 pitch (16-B aligned rows, bank spread)
    constexpr int HM = BM / 2;
    float *Cs = reinterpret_cast<float *>(smem);
    constexpr int CPR = BN_ / 8;  // 8-wide chunks per row
    constexpr int NQ = HM * CPR / CONV_THREADS;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (wm == h) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = i * 16 + (lane >> 4) * 4 + r;
                        const int col = wn * (BN_ / 2) + j * 16 + (lane & 15);
                        Cs[row * CP + col] = acc[i][j][r];
                    }
        }
        __syncthreads();
        const int mh = m0 + h * HM;
        if (a.ksplit > 1) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int c = tid + q * CONV_THREADS;
                const int row = c / CPR, ch = c - row * CPR;
                const int gm = mh + row, gn0 = n0 + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) continue;
                // raw partial; Cout % 8 == 0 is required for split-K
                const float *src = Cs + row * CP + ch * 8;
                float *pp = a.part + ((long long)kz * a.M + gm) * a.Cout + gn0;
                *reinterpret_cast<float4 *>(pp) = *reinterpret_cast<const float4 *>(src);
                *reinterpret_cast<float4 *>(pp + 4) = *reinterpret_cast<const float4 *>(src + 4);
            }
        } else {
            finish_batch<TO, NQ>(a, [&](int q, int &gm, int &gn0, const float *&src) {
                const int c = tid + q * CONV_THREADS;
                const int row = c / CPR, ch = c - row * CPR;
                gm = mh + row;
                gn0 = n0 + ch * 8;
                src = Cs + row * CP + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) gm = -1;
            });
        }
        if (h == 0) __syncthreads();
    }
}

template <typename T, typename TO, int BN_, bool DUAL = false, bool PW = false>
__global__ __launch_bounds__(CONV_THREADS, 2) void k_conv(ConvArgs a) {
    conv_body<T, TO, BN_, DUAL, PW, false>(a);
}
template <typename T, typename TO, int BN_, bool DUAL = false>
__global__ __launch_bounds__(CONV_THREADS, BN_ == 64 ? 4 : 3) void k_conv_sb(ConvArgs a) {
    conv_body<T, TO, BN_, DUAL, true, true>(a);
}
// the single-stage schedule for general layers (padded / KxK: the stem, the
// Cin < 128 3x3 layers)
template <typename T, typename TO, int BN_>
__global__ __launch_bounds__(CONV_THREADS, BN_ == 64 ? 4 : 3) void k_conv_sbg(ConvArgs a) {
    conv_body<T, TO, BN_, false, false, true>(a);
}

template <typename TO>
__global__ __launch_bounds__(256) void k_conv_reduce(ConvArgs a) {
    const int cpr = a.Cout / 8;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)a.M * cpr) return;
    const int gm = (int)(i / cpr), gn0 = (int)(i - (long long)gm * cpr) * 8;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const long long slice = (long long)a.M * a.Cout;
    const float *pp = a.part + (long long)gm * a.Cout + gn0;
    for (int z = 0; z < a.ksplit; ++z) {
        const float4 x0 = *reinterpret_cast<const float4 *>(pp + z * slice);
        const float4 x1 = *reinterpret_cast<const float4 *>(pp + z * slice + 4);
        v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w; v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
    }
    finish8<TO>(a, gm, gn0, v);
}

// ---------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores (the fp32 model's layers when
// mdx_policy.fp32_split = 6 | 9).  Every fp32 operand is split into three
// bf16 values x = hi + mid + lo (hi = RN(x), mid = RN(x - hi), lo = x - hi -
// mid): each subtraction is exact (Sterbenz) and the last residual has at most
// 8 significant bits, so the three parts represent x EXACTLY (normal range).
// A bf16 x bf16 product (8 x 8 significant bits) is exact in fp32, so
// sum_k a_k b_k = sum of the nine plane products, accumulated in fp32 by
// v_mfma_f32_16x16x32_bf16 at 16x the f32 MFMA rate.  NP = 9 forms all nine;
// NP = 6 drops mid*lo, lo*mid, lo*lo (each <= 2^-24 |a b|, the size of one
// fp32 rounding).  The hi*hi products accumulate in their own registers, the
// smaller cross products in a second set, added once at the end.
//
// Same tile, loads and epilogue as k_conv<float, float, BN_>: 128 x BN_ per
// 256-thread workgroup, K-steps of 32 fp32 loaded 16 B per lane through the
// range-checked descriptors one step ahead; the split happens between the
// register stage and LDS, which holds 3 planes per operand of 64-B rows (32
// bf16 of one K-step: a wave's 16-row x 4-piece fragment read is 1 KB
// contiguous, no swizzle needed).  96 KB of LDS: one workgroup per CU.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int X3_ROWB = 64;

// two values at a time: one v_cvt_pk_bf16_f32 per plane, the bf16 pair back
// to fp32 by a shift and a mask, the exact remainder by one v_pk_add_f32
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 bf2_to_f2(unsigned u) {
    return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
__device__ __forceinline__ void split3_pair(f32x2 x, unsigned &h, unsigned &m, unsigned &l) {
    h = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
    const f32x2 r1 = x - bf2_to_f2(h);
    m = __builtin_bit_cast(unsigned, __builtin_convertvector(r1, bf16x2));
    const f32x2 r2 = r1 - bf2_to_f2(m);
    l = __builtin_bit_cast(unsigned, __builtin_convertvector(r2, bf16x2));
}
__device__ __forceinline__ void split3_store(const uint4 &v, char *p0, int plane_bytes) {
    uint2 h, m, l;
    split3_pair(f32x2{__uint_as_float(v.x), __uint_as_float(v.y)}, h.x, m.x, l.x);
    split3_pair(f32x2{__uint_as_float(v.z), __uint_as_float(v.w)}, h.y, m.y, l.y);
    *reinterpret_cast<uint2 *>(p0) = h;
    *reinterpret_cast<uint2 *>(p0 + plane_bytes) = m;
    *reinterpret_cast<uint2 *>(p0 + 2 * plane_bytes) = l;
}

// LDS rows of 64 B, four 16-B chunks: chunk c of row r lives at position
// c ^ x3_swz(r), so that each 16-lane group of a fragment ds_read_b128 (rows
// 0-15 x one chunk, groups {0-3,12-15,20-27}, ...) hits 16 distinct 16-B bank
// slots; unswizzled, rows r and r + 4 of a group share banks (2-way: the
// kernel measured 3.7 conflict cycles per LDS instruction, SQ_LDS_BANK_CONFLICT)
__device__ __forceinline__ int x3_swz(int r) { return ((r >> 3) & 1) << 1; }

// BP: the weights (B operand) arrive already split, as bf16 planes in the
// mdx_split_x6 layout (per row, 96 B per 16 K = hi | mid | lo; a.w, a.wbytes
// and a.bsw in plane bytes, K % 32 == 0): each 16-B piece is copied to its
// plane row in LDS, and only the activations are split in the kernel.
// PW: 1x1 / stride 1 / unpadded layers and the Winograd GEMMs -- row m of A is
// pixel m, so a lane's A address is its row's offset + the K offset (no
// per-K-step tap / bounds arithmetic on the VALU the split already loads).
// SB: one LDS stage and one register stage (36 KB of LDS at BN 64), the
// plane products of all six pairs summed in one accumulator set -- three
// workgroups per CU instead of two; two barriers per K-step (as k_conv_sb).
template <typename TO, int BN_, int NP, bool BP = false, bool PW = false, bool SB = false>
__global__ __launch_bounds__(CONV_THREADS, BN_ == 64 ? (SB ? 3 : 2) : 1) void k_conv_x3(ConvArgs a) {
    static_assert(NP == 6 || NP == 9, "x6 or x9 plane products");
    constexpr int BK = 32, VEC = 4;
    constexpr int TI = BM / 32, TJ = BN_ / 32;
    // B loads per thread and K-step: 16-B fp32 chunks, or 16-B plane pieces (12 per row)
    constexpr int BLOADS = BP ? BN_ * 12 / CONV_THREADS : BN_ * 8 / CONV_THREADS;
    constexpr int APL = BM * X3_ROWB, BPL = BN_ * X3_ROWB;  // bytes of one plane
    constexpr int STAGE = 3 * (APL + BPL);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (gridDim.z > 1) {  // batch entry z of a batched GEMM
        const long long z = blockIdx.z;
        a.x = reinterpret_cast<const char *>(a.x) + z * a.bsx;
        a.w = reinterpret_cast<const char *>(a.w) + z * a.bsw;
        a.out = reinterpret_cast<char *>(a.out) + z * a.bso;
    }
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN_;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // ---- global loads: as k_conv (rows tid/8 + 32 i, 16-byte chunk tid % 8)
    const int kc = tid & 7;
    const int lrow = tid >> 3;
    int a_iy0[4], a_ix0[4];
    long long a_base[4];
    bool a_ok[4];
    const int ohw = a.OH * a.OW;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int gm = m0 + lrow + 32 * i;
        a_ok[i] = gm < a.M;
        const int gmc = a_ok[i] ? gm : 0;
        const int b = gmc / ohw, rem = gmc - b * ohw;
        const int oy = rem / a.OW, ox = rem - oy * a.OW;
        a_iy0[i] = oy * a.stride - a.pad;
        a_ix0[i] = ox * a.stride - a.pad;
        a_base[i] = (long long)b * a.H * a.W * a.Cin;
    }
    const int kz = blockIdx.y;
    int kglob = kz * a.ksteps * BK + kc * VEC;
    int kci = kglob % a.Cin;
    int kr = kglob / a.Cin;
    int kkx = kr % a.KW, kky = kr / a.KW;
    uint4 ra[SB ? 1 : 2][4], rb[SB ? 1 : 2][BLOADS];
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)a.x, (short)0, a.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)a.w, (short)0, a.wbytes, 0x00020000);
    constexpr unsigned OOB = 0xFFFFFFF0u;
    // PW: byte offset of each A row (pixel m0 + lrow + 32 i), OOB for rows past M
    unsigned a_rowoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a_rowoff[i] = a_ok[i] ? (unsigned)((long long)(m0 + lrow + 32 * i) * a.Cin * 4) : OOB;
    auto load_global = [&](uint4 (&A)[4], uint4 (&Bv)[BLOADS]) {
        const bool kok = kglob < a.K;
        if constexpr (PW) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                A[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rx, (kok && a_rowoff[i] != OOB) ? a_rowoff[i] + kglob * 4 : OOB, 0, 0));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int iy = a_iy0[i] + kky, ix = a_ix0[i] + kkx;
                const bool ok = kok && a_ok[i] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                const unsigned off = (unsigned)((a_base[i] + ((long long)iy * a.W + ix) * a.Cin + kci) * 4ll);
                A[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : OOB, 0, 0));
            }
        }
        if constexpr (BP) {
            const int kb = kglob - kc * VEC;  // the K-step's first K value
#pragma unroll
            for (int i = 0; i < BLOADS; ++i) {
                // piece c = (plane p, row, chunk q = 2 g + h): 8 consecutive
                // lanes fill two whole 64-B rows of one plane (conflict-free stores)
                const int c = tid + CONV_THREADS * i, p = c / (BN_ * 4), rem = c - p * (BN_ * 4);
                const int row = rem >> 2, q = rem & 3;
                const int gn = n0 + row;
                const unsigned off = (unsigned)(((long long)gn * a.K + kb) * 6ll + (q >> 1) * 96 + p * 32 + (q & 1) * 16);
                Bv[i] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, (kb < a.K && gn < a.Cout) ? off : OOB, 0, 0));
            }
        } else {
#pragma unroll
            for (int i = 0; i < BLOADS; ++i) {
                const int gn = n0 + lrow + 32 * i;
                const unsigned off = (unsigned)(((long long)gn * a.K + kglob) * 4ll);
                Bv[i] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, (kok && gn < a.Cout) ? off : OOB, 0, 0));
            }
        }
    };
    auto advance_k = [&]() {
        kglob += BK;
        if constexpr (PW) return;  // one tap: the K offset is kglob itself
        kci += BK;
        while (kci >= a.Cin) {
            kci -= a.Cin;
            if (++kkx == a.KW) {
                kkx = 0;
                ++kky;
            }
        }
    };
    // the 4 fp32 of chunk kc become 8 B at byte 8 kc of the row in each plane
    auto store_lds = [&](int buf, const uint4 (&A)[4], const uint4 (&Bv)[BLOADS]) {
        char *st = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = lrow + 32 * i;
            split3_store(A[i], st + row * X3_ROWB + (((kc >> 1) ^ x3_swz(row)) << 4) + (kc & 1) * 8, APL);
        }
        if constexpr (BP) {
#pragma unroll
            for (int i = 0; i < BLOADS; ++i) {
                const int c = tid + CONV_THREADS * i, p = c / (BN_ * 4), rem = c - p * (BN_ * 4);
                const int row = rem >> 2, q = rem & 3;
                *reinterpret_cast<uint4 *>(st + 3 * APL + p * BPL + row * X3_ROWB + ((q ^ x3_swz(row)) << 4)) = Bv[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < BLOADS; ++i) {
                const int row = lrow + 32 * i;
                split3_store(Bv[i], st + 3 * APL + row * X3_ROWB + (((kc >> 1) ^ x3_swz(row)) << 4) + (kc & 1) * 8,
                             BPL);
            }
        }
    };

    // (SB: acc_x is acc_h -- one accumulator set)
    float4v acc_h[TI][TJ], acc_xs[SB ? 1 : TI][SB ? 1 : TJ];
    auto acc_x = [&](int i, int j) -> float4v & {
        if constexpr (SB) return acc_h[i][j];
        else return acc_xs[i][j];
    };
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            acc_h[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
            if constexpr (!SB) acc_xs[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
        }

    const int nk_all = (a.K + BK - 1) / BK;
    const int nk = min(a.ksteps, nk_all - kz * a.ksteps);
    load_global(ra[0], rb[0]);
    advance_k();
    store_lds(0, ra[0], rb[0]);
    if (nk > 1) {
        load_global(ra[SB ? 0 : 1], rb[SB ? 0 : 1]);
        advance_k();
    }
    __syncthreads();
    // cross products (plane of A, plane of B; 0 hi, 1 mid, 2 lo), smallest
    // first, into acc_x: lo*lo, mid*lo, lo*mid (x9 only), mid*mid, hi*lo,
    // lo*hi, hi*mid, mid*hi; hi*hi into acc_h
    constexpr int PA[8] = {2, 1, 2, 1, 0, 2, 0, 1}, PB[8] = {2, 2, 1, 1, 2, 0, 1, 0};
    constexpr int P0 = NP == 9 ? 0 : 3;
    auto kstep = [&](int kt, uint4 (&Ai)[4], uint4 (&Bi)[BLOADS], const uint4 (&As_)[4],
                     const uint4 (&Bs_)[BLOADS]) {
        const int cur = SB ? 0 : (kt & 1);
        if (!SB && kt + 2 < nk) {
            load_global(Ai, Bi);
            advance_k();
        }
        const int fo = ((lane >> 4) ^ x3_swz(lane & 15)) << 4;  // (row bits 0-3 = lane & 15)
        const char *Ab = smem + cur * STAGE + (wm * (BM / 2) + (lane & 15)) * X3_ROWB + fo;
        const char *Bb = smem + cur * STAGE + 3 * APL + (wn * (BN_ / 2) + (lane & 15)) * X3_ROWB + fo;
        bf16x8 af[3][TI], bf[3][TJ];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int i = 0; i < TI; ++i) af[p][i] = *reinterpret_cast<const bf16x8 *>(Ab + p * APL + i * 16 * X3_ROWB);
#pragma unroll
            for (int j = 0; j < TJ; ++j) bf[p][j] = *reinterpret_cast<const bf16x8 *>(Bb + p * BPL + j * 16 * X3_ROWB);
        }
#pragma unroll
        for (int q = P0; q < 8; ++q)
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc_x(i, j) = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[PA[q]][i], bf[PB[q]][j], acc_x(i, j), 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bf[0][j], acc_h[i][j], 0, 0, 0);
        if constexpr (SB) {
            // [MFMAs of kt] barrier [store kt + 1, load kt + 2 into the same registers] barrier
            __syncthreads();
            if (kt + 1 < nk) store_lds(0, Ai, Bi);
            if (kt + 2 < nk) {
                load_global(Ai, Bi);
                advance_k();
            }
        } else if (kt + 1 < nk) {
            store_lds(cur ^ 1, As_, Bs_);
        }
        __syncthreads();
    };
    int kt = 0;
    if constexpr (SB) {
        for (; kt < nk; ++kt) kstep(kt, ra[0], rb[0], ra[0], rb[0]);
    } else {
        for (; kt + 1 < nk; kt += 2) {
            kstep(kt, ra[0], rb[0], ra[SB ? 0 : 1], rb[SB ? 0 : 1]);
            kstep(kt + 1, ra[SB ? 0 : 1], rb[SB ? 0 : 1], ra[0], rb[0]);
        }
        if (kt < nk) kstep(kt, ra[0], rb[0], ra[SB ? 0 : 1], rb[SB ? 0 : 1]);
    }

    // ---- epilogue: as k_conv, in two halves of BM/2 rows
    constexpr int CP = BN_ + 4;
    constexpr int HM = BM / 2;
    float *Cs = reinterpret_cast<float *>(smem);
    constexpr int CPR = BN_ / 8;
    constexpr int NQ = HM * CPR / CONV_THREADS;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (wm == h) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = i * 16 + (lane >> 4) * 4 + r;
                        const int col = wn * (BN_ / 2) + j * 16 + (lane & 15);
                        Cs[row * CP + col] = SB ? acc_h[i][j][r] : acc_h[i][j][r] + acc_x(i, j)[r];
                    }
        }
        __syncthreads();
        const int mh = m0 + h * HM;
        if (a.ksplit > 1) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int c = tid + q * CONV_THREADS;
                const int row = c / CPR, ch = c - row * CPR;
                const int gm = mh + row, gn0 = n0 + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) continue;
                const float *src = Cs + row * CP + ch * 8;
                float *pp = a.part + ((long long)kz * a.M + gm) * a.Cout + gn0;
                *reinterpret_cast<float4 *>(pp) = *reinterpret_cast<const float4 *>(src);
                *reinterpret_cast<float4 *>(pp + 4) = *reinterpret_cast<const float4 *>(src + 4);
            }
        } else {
            finish_batch<TO, NQ>(a, [&](int q, int &gm, int &gn0, const float *&src) {
                const int c = tid + q * CONV_THREADS;
                const int row = c / CPR, ch = c - row * CPR;
                gm = mh + row;
                gn0 = n0 + ch * 8;
                src = Cs + row * CP + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) gm = -1;
            });
        }
        if (h == 0) __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Large-layer kernel (fp16, Cin % 64 == 0): 256x256 tile, 512 threads = 8
// waves as 2(M) x 4(N), each wave 128x64 = 8x4 MFMA 16x16x32 tiles.  Both
// operands are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, no
// VGPR round trip) in K-substeps of 32 halves (A 256 x 64 B + B 256 x 64 B =
// 32 KiB), four substep buffers, three substeps in flight ahead of the one
// being multiplied (counted vmcnt + raw s_barrier, one barrier per substep).
// A 64-half chunk of K lies inside one (ky, kx) tap because Cin % 64 == 0, so
// the implicit-im2col source of each 16-B piece is a plain per-row offset;
// chunks are visited channel-chunk outer, tap inner (input rows re-read from
// L2 across the taps).  LDS image: row r (64 B) holds logical 16-B piece c at
// physical piece c ^ (((r >> 3) & 1) << 1) -- lane-linear DMA destination, the
// swizzle is applied on the global source address; fragment reads are then
// bank-conflict-free for the ds_read_b128 lane groups.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Streaming 1x1 kernel for HBM-bound layers (fp16, stride 1, K = Cin in
// {64, 128, 256}, Cout % 64 == 0): out = act(X W^T + b (+ res)) with M in the
// hundreds of thousands and a small K.  Workgroup = 4 waves = 128 pixels x 64
// output channels; the 64 x K weight slice is staged in LDS once, the
// activations go straight from HBM into MFMA operand registers (no LDS pass,
// no barrier in the loop), and the product is formed transposed (D = W X^T)
// so each lane ends with 4 consecutive channels of one pixel: 8-byte
// residual loads and stores, no LDS epilogue.
//   lane l, MFMA 16x16x32:  W operand  = W[n0 + 16 ns + (l & 15)][32 kc + 8 (l >> 4) ..+8]
//                           X operand  = X[m0 + 16 ms + (l & 15)][32 kc + 8 (l >> 4) ..+8]
//                           D[ms][ns][r] = out[m0 + 16 ms + (l & 15)][n0 + 16 ns + 4 (l >> 4) + r]
// ---------------------------------------------------------------------------
template <int KC>
__global__ __launch_bounds__(256) void k_conv1x1_stream(ConvArgs a) {
    constexpr int K = 32 * KC, WPITCH = 2 * K + 16;  // LDS row pitch (bytes): +16 spreads rows over banks
    __shared__ __attribute__((aligned(16))) char sw[64 * WPITCH];
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int n0 = tn * 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const _Float16 *Wt = reinterpret_cast<const _Float16 *>(a.w);
    const int m0 = tm * 128 + wid * 32;
    // Output layout of the epilogue: per pixel row and pair of 16-channel
    // blocks (2p, 2p+1), lane group g = lane >> 4 owns 8 consecutive channels
    // -- block 2p + (g & 1), channels 8 (g >> 1) .. +8 -- after one exchange
    // with lane ^ 16, so residual loads and output stores are 16 B per lane
    // (8-B accesses run at ~0.6x the 16-B rate).
    const int g = lane >> 4;
    const int ch_in_pair = 16 * (g & 1) + 8 * (g >> 1);  // channel offset within a 32-channel pair
    // residual first: its loads are the longest stream and depend on nothing
    half8 rr[2][2];
    if (a.res) {
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void *)a.res, (short)0, a.rbytes,
                                                                            0x00020000);
#pragma unroll
        for (int ms = 0; ms < 2; ++ms) {
            const int m = m0 + 16 * ms + (lane & 15);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const unsigned off =
                    m < a.M ? (unsigned)(((long long)m * a.Cout + n0 + 32 * pp + ch_in_pair) * 2) : 0xFFFFFFF0u;
                rr[ms][pp] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0));
            }
        }
    }
    // stage the 64 x K weight slice
    for (int i = tid; i < 64 * K / 8; i += 256) {
        const int r = i / (K / 8), c = i - r * (K / 8);
        *reinterpret_cast<uint4 *>(sw + r * WPITCH + c * 16) =
            *reinterpret_cast<const uint4 *>(Wt + (long long)(n0 + r) * K + c * 8);
    }
    // this wave's 32 pixels and their activation fragments
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)a.x, (short)0, a.xbytes, 0x00020000);
    half8 xf[2][KC];
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
        const int m = m0 + 16 * ms + (lane & 15);
        const unsigned base = (unsigned)((long long)m * K * 2) + 16u * (lane >> 4);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
            xf[ms][kc] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rx, m < a.M ? base + 64u * kc : 0xFFFFFFF0u, 0, 0));
    }
    __syncthreads();
    float4v acc[2][4];
#pragma unroll
    for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = float4v{0.f, 0.f, 0.f, 0.f};
    const char *wl = sw + (lane & 15) * WPITCH + 16 * (lane >> 4);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
        half8 wf[4];
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) wf[ns] = *reinterpret_cast<const half8 *>(wl + 16 * ns * WPITCH + 64 * kc);
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
            for (int ns = 0; ns < 4; ++ns)
                acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ns], xf[ms][kc], acc[ms][ns], 0, 0, 0);
    }
    // epilogue: exchange halves with lane ^ 16, bias, residual, ReLU, fp16,
    // 16-byte stores
    const bool odd = (g & 1) != 0;
    _Float16 *O = reinterpret_cast<_Float16 *>(a.out);
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        const int c0 = n0 + 32 * pp + ch_in_pair;
        float bv[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float4 b4 = a.bias ? *reinterpret_cast<const float4 *>(a.bias + c0 + 4 * h)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            bv[4 * h] = b4.x; bv[4 * h + 1] = b4.y; bv[4 * h + 2] = b4.z; bv[4 * h + 3] = b4.w;
        }
#pragma unroll
        for (int ms = 0; ms < 2; ++ms) {
            // even groups keep block 2pp and receive its upper 4 channels; odd
            // groups keep block 2pp+1 and receive its lower 4 channels
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float keep = odd ? acc[ms][2 * pp + 1][r] : acc[ms][2 * pp][r];
                const float send = odd ? acc[ms][2 * pp][r] : acc[ms][2 * pp + 1][r];
                const float recv = __shfl_xor(send, 16);
                v[odd ? 4 + r : r] = keep;
                v[odd ? r : 4 + r] = recv;
            }
            const int m = m0 + 16 * ms + (lane & 15);
            if (m >= a.M) continue;
            half8 o;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                float x = v[r] + bv[r];
                if (a.res) x += (float)rr[ms][pp][r];
                if (a.relu) x = x > 0.f ? x : 0.f;
                o[r] = (_Float16)x;
            }
            *reinterpret_cast<half8 *>(O + (long long)m * a.Cout + c0) = o;
        }
    }
}

// Narrow-output streaming 1x1 kernel (RPN head: 256 -> 15 logits/deltas,
// fp32 out): one 16-row MFMA block of output channels (rows >= Cout read as
// zero weights), no LDS and no barrier -- each wave loads its 16 x K weight
// fragments straight from L2 and streams 32 pixels' activations into the B
// operands, so the launch runs at the activation read rate.
template <int KC>
__global__ __launch_bounds__(256) void k_conv1x1_head(ConvArgs a) {
    constexpr int K = 32 * KC;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m0 = (int)blockIdx.x * 128 + wid * 32;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)a.x, (short)0, a.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)a.w, (short)0, a.wbytes, 0x00020000);
    half8 xf[2][KC], wf[KC];
    const int orow = lane & 15;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
        wf[kc] = __builtin_bit_cast(
            half8, __builtin_amdgcn_raw_buffer_load_b128(
                       rw, orow < a.Cout ? (unsigned)((orow * K + 8 * (lane >> 4) + 32 * kc) * 2) : 0xFFFFFFF0u, 0, 0));
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
        const int m = m0 + 16 * ms + (lane & 15);
        const unsigned base = (unsigned)((long long)m * K * 2) + 16u * (lane >> 4);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
            xf[ms][kc] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rx, m < a.M ? base + 64u * kc : 0xFFFFFFF0u, 0, 0));
    }
    float4v acc[2] = {float4v{0.f, 0.f, 0.f, 0.f}, float4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
            acc[ms] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[kc], xf[ms][kc], acc[ms], 0, 0, 0);
    // D[och = 4 (lane >> 4) + r][pixel = lane & 15]
    const int oc = 4 * (lane >> 4);
    float* O = reinterpret_cast<float *>(a.out);
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
        const int m = m0 + 16 * ms + (lane & 15);
        if (m >= a.M) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = oc + r;
            if (c >= a.Cout) continue;
            float v = acc[ms][r] + (a.bias ? a.bias[c] : 0.f);
            if (a.relu) v = v > 0.f ? v : 0.f;
            O[(long long)m * a.Cout + c] = v;
        }
    }
}

// Narrow-output fp32 1x1 kernel (RPN head 256 -> 15, mask predictor 256 ->
// 1, box predictor 1024 -> 6): out[m][o] = sum_k W[o][k] X[m][k] + bias[o],
// Cout <= 16, K % 16 == 0, K <= 1024.  D = W X^T on 16x16x4 f32 MFMAs: each
// lane holds float4 pieces k = 16 c + 4 (lane >> 4) .. +3 of one weight row
// (lane & 15) and of one pixel row, the four MFMAs of a piece take element e
// of both (the same permutation of k on both operands); the wave keeps W in
// registers and walks 16-pixel groups grid-stride, so the launch runs at the
// activation read rate.
template <int KC>
__global__ __launch_bounds__(256) void k_head_f32(ConvArgs a) {
    constexpr int K = 16 * KC;
    // K in chunks of up to 256: the weights stay in registers when K <= 256,
    // else each chunk's weight pieces are re-read (from L1 / L2) per group
    constexpr int CH = KC < 16 ? KC : 16;
    constexpr bool HOLD = KC <= 16;
    const int lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
    const float *X = reinterpret_cast<const float *>(a.x);
    const float *Wt = reinterpret_cast<const float *>(a.w);
    float *O = reinterpret_cast<float *>(a.out);
    float4 wf[CH];
    auto load_w = [&](int c0) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
            wf[c] = r16 < a.Cout ? *reinterpret_cast<const float4 *>(Wt + (long long)r16 * K + 16 * (c0 + c) + 4 * g)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    if (HOLD) load_w(0);
    const long long groups = ((long long)a.M + 15) / 16;
    const long long wave0 = (long long)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (long long)gridDim.x * 4;
    for (long long grp = wave0; grp < groups; grp += nwaves) {
        const long long m = grp * 16 + r16;
        const bool ok = m < a.M;
        const float *xr = X + (ok ? m : 0) * K + 4 * g;
        float4v acc = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c0 = 0; c0 < KC; c0 += CH) {
            if (!HOLD) load_w(c0);
            float4 xf[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c)
                xf[c] = ok ? *reinterpret_cast<const float4 *>(xr + 16 * (c0 + c)) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[c].x, xf[c].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[c].y, xf[c].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[c].z, xf[c].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[c].w, xf[c].w, acc, 0, 0, 0);
            }
        }
        // D[o = 4 g + r][pixel = lane & 15]
        if (ok) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = 4 * g + r;
                if (o < a.Cout) {
                    float v = acc[r] + (a.bias ? a.bias[o] : 0.f);
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    O[m * a.Cout + o] = v;
                }
            }
        }
    }
}


// Tile codes: 8 = 256x256 (8 waves), 4 = 128x128 (4 waves), both 4 LDS
// buffers; 6 = 256x128 (4 waves, 3 buffers: 72 KiB, so two workgroups share
// a CU and fill each other's barrier gaps).  Waves form 2 x WN; wave tile
// (BM/2) x (BN/WN).
template <int NW>
struct GTile {
    static constexpr int WAVES = NW == 6 ? 4 : NW;
    static constexpr int THREADS = 64 * WAVES, BM = NW == 6 ? 256 : 32 * NW, BN = NW == 6 ? 128 : 32 * NW;
    static constexpr int WM = 2, WN = WAVES / 2;
    static constexpr int WROWS = BM / WM, WCOLS = BN / WN;      // wave tile
    static constexpr int TI = WROWS / 16, TJ = WCOLS / 16;      // MFMA tiles per wave
    static constexpr int AJ = BM / (16 * WAVES), BJ = BN / (16 * WAVES);  // DMA instructions per wave and substep
    static constexpr int SUB = (BM + BN) * 64;                  // bytes per 32-deep K-substep
    static constexpr int NBUF = NW == 6 ? 3 : 4;
    static constexpr int EPI_PITCH = 68;                        // fp32 pitch of a wave's 64-column block
    static constexpr int EPI_ROWS = 64;                         // rows per epilogue pass
    static constexpr int EPI = WAVES * EPI_ROWS * EPI_PITCH * 4;
    static constexpr int LDS = NBUF * SUB > EPI ? NBUF * SUB : EPI;
};
constexpr int G_BM = GTile<8>::BM, G_BN = GTile<8>::BN, G_THREADS = GTile<8>::THREADS;
constexpr int G_LDS = GTile<8>::LDS;

__device__ __attribute__((aligned(64))) uint4 g_zero16[4];  // zero source for padding / out-of-range rows

typedef __attribute__((address_space(3))) void *lds_ptr_t;

__device__ __forceinline__ void glds16(const void *src, char *dst) {
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)dst, 16, 0, 0);
}

__device__ __forceinline__ int g_swz(int r) { return ((r >> 3) & 1) << 1; }

// s_waitcnt the compiler's waitcnt pass can see (an inline-asm waitcnt is
// opaque to it: it then re-waits for loads this one already drained), fenced
// by empty memory clobbers so no memory operation moves across it.
// gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14
#define MDX_WAIT_VM(n) \
    do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_waitcnt(0x0F70 | (n)); asm volatile("" ::: "memory"); } while (0)
#define MDX_WAIT_LGKM0() \
    do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_waitcnt(0xC07F); asm volatile("" ::: "memory"); } while (0)

// TIN: operand type.  fp16: a 64-B LDS row is 32 halves (one 16x16x32 f16
// MFMA per fragment pair); fp32: 16 floats, and each 16-B fragment feeds four
// 16x16x4 f32 MFMAs (element e of lane (row, piece) is k = 4 piece + e, the
// same permutation on both operands, so the dot products are unchanged).
// A K "chunk" is one 128-B run of input channels (64 halves / 32 floats),
// split into two 64-B substeps.
template <typename TIN, typename TO, int NW, bool ILV>
__global__ __launch_bounds__(GTile<NW>::THREADS, NW == 8 ? 1 : 2) void k_convg(ConvArgs a) {
    using GT = GTile<NW>;
    constexpr int BM = GT::BM, SUB = GT::SUB, TI = GT::TI, TJ = GT::TJ;
    constexpr int AJ = GT::AJ, BJ = GT::BJ, NBUF = GT::NBUF, PIECES = AJ + BJ;
    constexpr bool F32 = sizeof(TIN) == 4;
    constexpr int VEC = 16 / (int)sizeof(TIN);  // elements per 16-B piece
    constexpr int SUBK = 4 * VEC;               // K elements per substep (one 64-B row)
    constexpr int CHK = 2 * SUBK;               // channels per chunk
    static_assert(!(F32 && ILV), "the interleaved DMA schedule is fp16-only");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (gridDim.z > 1) {  // batch entry z of a batched GEMM (the Winograd GEMMs)
        const long long z = blockIdx.z;
        a.x = reinterpret_cast<const char *>(a.x) + z * a.bsx;
        a.w = reinterpret_cast<const char *>(a.w) + z * a.bsw;
        a.out = reinterpret_cast<char *>(a.out) + z * a.bso;
    }
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * GT::BM, n0 = tn * GT::BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / GT::WN, wn = wid - wm * GT::WN;

    // DMA descriptors: A instruction j of wave w fills LDS rows 16 (AJ w + j)
    // .. +16, B instruction j rows 16 (BJ w + j) .. +16
    const TIN *X = reinterpret_cast<const TIN *>(a.x);
    const TIN *Wt = reinterpret_cast<const TIN *>(a.w);
    const int ohw = a.OH * a.OW;
    int a_iy0[AJ], a_ix0[AJ];
    long long a_base[AJ];
    bool a_ok[AJ];
    const TIN *b_src[BJ];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
        const int r = 16 * (AJ * wid + j) + (lane >> 2);
        const int c = (lane & 3) ^ g_swz(r);
        const int gm = m0 + r;
        a_ok[j] = gm < a.M;
        const int gmc = a_ok[j] ? gm : 0;
        const int b = gmc / ohw, rem = gmc - b * ohw;
        const int oy = rem / a.OW, ox = rem - oy * a.OW;
        a_iy0[j] = oy * a.stride - a.pad;
        a_ix0[j] = ox * a.stride - a.pad;
        a_base[j] = (long long)b * a.H * a.W * a.Cin + c * VEC;
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
        const int r = 16 * (BJ * wid + j) + (lane >> 2);
        const int c = (lane & 3) ^ g_swz(r);
        const int gn = n0 + r;
        b_src[j] = gn < a.Cout ? Wt + (long long)gn * a.K + c * VEC : nullptr;
    }
    // 1x1 / unpadded layers (FC layers, 1x1 convs): every valid row's source
    // is in range, so the A piece address is a row pointer + the K offset
    // (fp32 only: the fp16 tile has no registers to spare for the pointers)
    const bool pointwise = F32 && a.KH == 1 && a.KW == 1 && a.pad == 0;
    const TIN *a_row[AJ] = {};
    if constexpr (F32) {
#pragma unroll
        for (int j = 0; j < AJ; ++j)
            a_row[j] = a_ok[j] ? X + a_base[j] + ((long long)a_iy0[j] * a.W + a_ix0[j]) * a.Cin : nullptr;
    }
    // issue state (uniform): the 64-chunk being issued and its tap
    // split-K: slice z = blockIdx.y multiplies substeps [s0, s0 + T) of the
    // K order (channel chunk outer, tap, half inner)
    const int s0 = (int)blockIdx.y * a.ksteps;
    int i_kci, i_kkx, i_kky, i_half;
    {
        const int q = s0 >> 1, taps = a.KH * a.KW;
        i_half = s0 & 1;
        const int tap = q % taps;
        i_kci = (q / taps) * CHK;
        i_kky = tap / a.KW;
        i_kkx = tap - i_kky * a.KW;
    }
    // DMA piece p of the substep being issued into buffer buf: p < AJ the A
    // rows of instruction j = p, then the B rows of j = p - AJ
    auto issue_piece = [&](int buf, int p) {
        const int kofs = i_kci + SUBK * i_half;
        if (p < AJ) {
            const int j = p;
            const void *src;
            if (F32 && pointwise) {
                src = a_row[j] ? (const void *)(a_row[j] + kofs) : (const void *)g_zero16;
            } else {
                const int iy = a_iy0[j] + i_kky, ix = a_ix0[j] + i_kkx;
                const bool ok = a_ok[j] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                src = ok ? (const void *)(X + a_base[j] + ((long long)iy * a.W + ix) * a.Cin + kofs)
                         : (const void *)g_zero16;
            }
            glds16(src, smem + buf * SUB + 16 * AJ * wid * 64 + j * 1024);
        } else {
            const int j = p - AJ;
            const int kglob = (i_kky * a.KW + i_kkx) * a.Cin + kofs;
            glds16(b_src[j] ? (const void *)(b_src[j] + kglob) : (const void *)g_zero16,
                   smem + buf * SUB + BM * 64 + 16 * BJ * wid * 64 + j * 1024);
        }
    };
    auto issue = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PIECES; ++p) issue_piece(buf, p);
        // next substep: half, then tap, then channel chunk
        if (++i_half == 2) {
            i_half = 0;
            if (++i_kkx == a.KW) {
                i_kkx = 0;
                if (++i_kky == a.KH) {
                    i_kky = 0;
                    i_kci += CHK;
                }
            }
        }
    };

    float4v acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    const int T = min(a.K / SUBK - s0, a.ksteps);  // substeps of this slice
    // fragment rows of this lane: r = 16 i + (lane & 15) (+ multiples of 64)
    const int off = ((lane >> 4) ^ g_swz(lane & 15)) * 16;
    const char *Abase = smem + (wm * GT::WROWS + (lane & 15)) * 64 + off;
    const char *Bbase = smem + BM * 64 + (wn * GT::WCOLS + (lane & 15)) * 64 + off;
    // fragments are register double-buffered: the LDS reads of substep t+1
    // are in flight while the MFMAs of substep t run from registers
    using frag_t = typename std::conditional<F32, float4v, half8>::type;
    // fp16: register double-buffered fragments; fp32: one set (its MFMA burst
    // per substep is 8x longer, the other wave of the SIMD covers the reads,
    // and two sets would spill at the 256-VGPR budget)
    // (the 256x128 tile: one set, so two workgroups fit a CU's registers;
    // the other workgroup's waves cover the fragment reads)
    constexpr int NSET = ((F32 && NW == 8) || NW == 6) ? 1 : 2;
    frag_t fa[NSET][TI], fb[NSET][TJ];
    auto read_frags = [&](int t, int set) {
        const char *Ab = Abase + (t % NBUF) * SUB;
        const char *Bb = Bbase + (t % NBUF) * SUB;
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[set][j] = *reinterpret_cast<const frag_t *>(Bb + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < TI; ++i) fa[set][i] = *reinterpret_cast<const frag_t *>(Ab + i * 16 * 64);
    };
    auto mma = [&](int set) {
        if constexpr (F32) {
            // row tile outermost: the MFMAs of tile i need only fb and fa[i],
            // so they start while the later A fragments are still arriving
            // (same e order per accumulator: bit-identical sums)
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[set][i][e], fb[set][j][e], acc[i][j], 0,
                                                                          0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[set][i], fb[set][j], acc[i][j], 0, 0, 0);
        }
    };
    // wait until substep u has landed (PIECES DMAs per thread per substep;
    // at most NBUF - 2 substeps in flight beyond it)
    auto wait_landed = [&](int u, int issued_upto) {
        const int ahead = issued_upto - u;
        if (NBUF >= 4 && ahead >= 2)
            MDX_WAIT_VM(2 * PIECES);
        else if (ahead >= 1)
            MDX_WAIT_VM(PIECES);
        else
            MDX_WAIT_VM(0);
    };
    issue(0);
    if (T > 1) issue(1);
    if (NBUF >= 4 && T > 2) issue(2);
    int issued = T < NBUF ? T - 1 : NBUF - 2;
    if constexpr (NSET == 1) {
        // substep t: [wait t, barrier, DMA t+3, read frags t] then its MFMAs
        // (buffer (t+3)&3 == (t-1)&3: every wave drained its reads of t-1
        // before the barrier).  DMA first, then all twelve fragment reads,
        // then the burst: 6165 vs 6384 us on box fc1 for reads-then-DMA (a
        // split burst overlapping the next substep's reads with the second
        // half of the MFMAs measured 6374 us)
        for (int t = 0; t < T; ++t) {
            wait_landed(t, issued);
            MDX_WAIT_LGKM0();
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (t + NBUF - 1 < T) {
                issue((t + NBUF - 1) % NBUF);
                issued = t + NBUF - 1;
            }
            read_frags(t, 0);
            // all fragment reads issue before the first MFMA (the scheduler
            // would otherwise sink each A read to its use and wait on it alone)
            __builtin_amdgcn_sched_barrier(0);
            mma(0);
        }
    } else {
    wait_landed(0, issued);
    __builtin_amdgcn_s_barrier();
    read_frags(0, 0);
    // iteration t: [wait t+1, barrier, DMA t+3, read frags t+1] then MFMAs of t
    // MFMAs q0 .. q1 - 1 of the wave's TI x TJ tile loop
    auto mma_range = [&](int set, int q0, int q1) {
        if constexpr (!F32) {
#pragma unroll
            for (int q = 0; q < TI * TJ; ++q) {
                if (q < q0 || q >= q1) continue;
                const int i = q / TJ, j = q - i * TJ;
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[set][i], fb[set][j], acc[i][j], 0, 0, 0);
            }
        }
    };
    // Every step -- the last one too -- waits, crosses the barrier and reads
    // the next fragment set (after the last substep: a harmless read of a
    // stale buffer).  With no path skipping the reads, the compiler's waitcnt
    // pass sees the same state on every path into mma() and never waits for
    // the set being read before the MFMAs of the other one.
    auto step = [&](int t, int cur) {
        {
            wait_landed(t + 1, issued);
            // drain this wave's pending fragment reads (those of substep t)
            // before the barrier: after it no wave still reads buffer
            // (t + 3) & 3 == (t - 1) & 3, which the next DMA overwrites
            MDX_WAIT_LGKM0();
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            read_frags(t + 1, cur ^ 1);
            if (t + 3 < T) {
                if constexpr (ILV) {
                    // the four DMA pieces ride in the MFMA issue gaps instead of
                    // stalling every wave right after the barrier
                    constexpr int QP = TI * TJ / 4;
                    const int buf = (t + 3) & 3;
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        __builtin_amdgcn_sched_barrier(0);
                        issue_piece(buf, p);
                        __builtin_amdgcn_sched_barrier(0);
                        mma_range(cur, p * QP, (p + 1) * QP);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (++i_half == 2) {
                        i_half = 0;
                        if (++i_kkx == a.KW) {
                            i_kkx = 0;
                            if (++i_kky == a.KH) {
                                i_kky = 0;
                                i_kci += 64;
                            }
                        }
                    }
                    issued = t + 3;
                    return;
                }
                issue((t + 3) & 3);
                issued = t + 3;
            }
        }
        mma(cur);
    };
    int t = 0;
    for (; t + 1 < T; t += 2) {
        step(t, 0);
        step(t + 1, 1);
    }
    if (t < T) step(t, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // epilogue: per wave, passes of 64 rows x WCOLS (= 64) columns through its
    // own LDS block
    static_assert(GT::WCOLS == 64, "epilogue stages 64-column wave blocks");
    constexpr int NPASS = GT::WROWS / GT::EPI_ROWS;
    constexpr int IPP = GT::EPI_ROWS / 16;  // MFMA row tiles per pass
    float *Cs = reinterpret_cast<float *>(smem) + wid * GT::EPI_ROWS * GT::EPI_PITCH;
#pragma unroll
    for (int h = 0; h < NPASS; ++h) {
#pragma unroll
        for (int i = 0; i < IPP; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cs[(i * 16 + (lane >> 4) * 4 + r) * GT::EPI_PITCH + j * 16 + (lane & 15)] = acc[IPP * h + i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (a.ksplit > 1) {
            // raw fp32 partial of this K slice (k_conv_reduce sums the slices)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int item = lane + 64 * q;
                const int row = item >> 3, ch = item & 7;
                const int gm = m0 + wm * GT::WROWS + GT::EPI_ROWS * h + row;
                const int gn0 = n0 + wn * GT::WCOLS + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) continue;
                const float *src = Cs + row * GT::EPI_PITCH + ch * 8;
                float *pp = a.part + ((long long)blockIdx.y * a.M + gm) * a.Cout + gn0;
                *reinterpret_cast<float4 *>(pp) = *reinterpret_cast<const float4 *>(src);
                *reinterpret_cast<float4 *>(pp + 4) = *reinterpret_cast<const float4 *>(src + 4);
            }
        } else {
            finish_batch<TO, 8>(a, [&](int q, int &gm, int &gn0, const float *&src) {
                const int item = lane + 64 * q;
                const int row = item >> 3, ch = item & 7;
                gm = m0 + wm * GT::WROWS + GT::EPI_ROWS * h + row;
                gn0 = n0 + wn * GT::WCOLS + ch * 8;
                src = Cs + row * GT::EPI_PITCH + ch * 8;
                if (gm >= a.M || gn0 >= a.Cout) gm = -1;
            });
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

// ---------------------------------------------------------------------------
// fp32 GEMM over operands split ONCE into bf16 planes in HBM ("x6 planes"),
// on the bf16 matrix cores through the LDS-DMA pipeline.
//
// Plane layout of an fp32 matrix X [rows][K] (K % 16 == 0): per row, K/16
// groups of 96 B = [hi k0-7 | hi k8-15 | mid k0-7 | mid k8-15 | lo k0-7 |
// lo k8-15] (bf16), x = hi + mid + lo exactly (the split3 of k_conv_x3).
//
// One 16x16x32 bf16 MFMA sums 32 K slots; lane group g = lane >> 4 supplies
// slots 8g..8g+7.  Feeding the two operands different planes per slot group
// (k = 8 (g & 1) + e of the 16-deep group in both) gives two plane products
// per MFMA, so three MFMAs per 16 K form the six products of k_conv_x3:
//   MFMA 1: A [hi  | hi ]  B [hi | mid]   -> hi*hi  + hi*mid
//   MFMA 2: A [mid | lo ]  B [hi | hi ]   -> mid*hi + lo*hi
//   MFMA 3: A [hi  | mid]  B [lo | mid]   -> hi*lo  + mid*mid
// (g < 2 | g >= 2), all into one fp32 accumulator per output element.
//
// Tile 256 x 256 per 512-thread workgroup (8 waves as 2 x 4, wave tile 128 x
// 64), substeps of 16 K = 96-B rows: A 24 KiB + B 24 KiB per substep staged by
// LDS-DMA (6 global_load_lds_dwordx4 per wave), three substep buffers, two in
// flight ahead of the one multiplied.  With 96-B rows the fragment reads of
// every ds_read_b128 lane group hit 16 distinct 16-B bank slots (6 r + piece
// mod 16 is a permutation over the group's rows), so no swizzle is needed.
// LDS bytes per FLOP are half the fp16 kernel's (three planes per operand
// serve six products).
// ---------------------------------------------------------------------------
constexpr int X6_ROWB = 96;             // bytes of one 16-deep K group of one row (3 planes)
constexpr int X6_BM = 256, X6_BN = 256, X6_THREADS = 512;
constexpr int X6_ASUB = X6_BM * X6_ROWB;  // 24 KiB
constexpr int X6_SUB = 2 * X6_ASUB;       // A + B of one substep
constexpr int X6_NBUF = 3;
constexpr int X6_LDS = X6_NBUF * X6_SUB > G_LDS ? X6_NBUF * X6_SUB : G_LDS;

// x [rows][ldx] fp32 (the first K columns) -> planes [rows][K/16][96 B]; one
// thread per 8 consecutive values (half a group)
__global__ __launch_bounds__(256) void k_split_x6(const float *__restrict__ x, long long rows, int K, long long ldx,
                                                  char *__restrict__ out) {
    const long long per_row = K / 8;
    const long long total = rows * per_row;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const long long r = i / per_row;
        const int c8 = (int)(i - r * per_row);
        const float *src = x + r * ldx + 8 * c8;
        const float4 u = *reinterpret_cast<const float4 *>(src), v = *reinterpret_cast<const float4 *>(src + 4);
        const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        bf16x8 h, m, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const __bf16 hb = (__bf16)f[e];
            const float r1 = f[e] - (float)hb;
            const __bf16 mb = (__bf16)r1;
            h[e] = hb;
            m[e] = mb;
            l[e] = (__bf16)(r1 - (float)mb);
        }
        char *o = out + r * (long long)K * 6 + (long long)(c8 >> 1) * X6_ROWB + (c8 & 1) * 16;
        *reinterpret_cast<bf16x8 *>(o) = h;
        *reinterpret_cast<bf16x8 *>(o + 32) = m;
        *reinterpret_cast<bf16x8 *>(o + 64) = l;
    }
}

// out[m][n] = act(sum_k A[m][k] B[n][k] + bias[n] (+ res)) with A = a.x, B =
// a.w in plane layout (K = a.K), M = a.M rows, N = a.Cout; batched over
// grid.z with byte strides bsx / bsw / bso.
__global__ __launch_bounds__(X6_THREADS, 1) void k_gemm_x6(ConvArgs a) {
    constexpr int WN = 4, WROWS = 128, WCOLS = 64, TI = WROWS / 16, TJ = WCOLS / 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (gridDim.z > 1) {
        const long long z = blockIdx.z;
        a.x = reinterpret_cast<const char *>(a.x) + z * a.bsx;
        a.w = reinterpret_cast<const char *>(a.w) + z * a.bsw;
        a.out = reinterpret_cast<char *>(a.out) + z * a.bso;
    }
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * X6_BM, n0 = tn * X6_BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid - wm * WN;
    const long long rowbytes = (long long)a.K * 6;

    // DMA instruction j (0..2) of wave w fills bytes [1 KiB (3 w + j), +1 KiB)
    // of the A (and the B) image of a substep: piece P = 64 (3 w + j) + lane
    // = row P / 6, 16-B piece P % 6 of that row's 96-B group
    const char *a_src[3], *b_src[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int P = 64 * (3 * wid + j) + lane;
        const int row = P / 6, pc = P - row * 6;
        const int gm = m0 + row, gn = n0 + row;
        a_src[j] = gm < a.M ? reinterpret_cast<const char *>(a.x) + gm * rowbytes + pc * 16 : nullptr;
        b_src[j] = gn < a.Cout ? reinterpret_cast<const char *>(a.w) + gn * rowbytes + pc * 16 : nullptr;
    }
    auto issue = [&](int buf, int kg) {
        char *dst = smem + buf * X6_SUB + 3 * wid * 1024;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            glds16(a_src[j] ? (const void *)(a_src[j] + (long long)kg * X6_ROWB) : (const void *)g_zero16,
                   dst + j * 1024);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            glds16(b_src[j] ? (const void *)(b_src[j] + (long long)kg * X6_ROWB) : (const void *)g_zero16,
                   dst + X6_ASUB + j * 1024);
    };

    float4v acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    // fragment addresses: row (lane & 15) of each 16-row tile, piece g & 1,
    // plane per operand / MFMA / lane half (see above)
    const int g = lane >> 4, hp = (g & 1) * 16;
    const bool lo_half = g < 2;
    const char *Ab = smem + (wm * WROWS + (lane & 15)) * X6_ROWB + hp;
    const char *Bb = smem + X6_ASUB + (wn * WCOLS + (lane & 15)) * X6_ROWB + hp;
    const int a1 = 0, a2 = lo_half ? 32 : 64, a3 = lo_half ? 0 : 32;
    const int b1 = lo_half ? 0 : 32, b2 = 0, b3 = lo_half ? 64 : 32;

    const int T = a.K / 16;
    issue(0, 0);
    if (T > 1) issue(1, 1);
    int issued = T > 1 ? 1 : 0;
    for (int t = 0; t < T; ++t) {
        // substep t landed (6 DMA instructions per substep per wave)
        if (issued - t >= 1)
            MDX_WAIT_VM(6);
        else
            MDX_WAIT_VM(0);
        MDX_WAIT_LGKM0();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // buffer (t + 2) % 3 == (t - 1) % 3: every wave is past its reads of t - 1
        if (t + 2 < T) {
            issue((t + 2) % 3, t + 2);
            issued = t + 2;
        }
        const int boff = (t % 3) * X6_SUB;
        bf16x8 fb[3][TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const char *p = Bb + boff + j * 16 * X6_ROWB;
            fb[0][j] = *reinterpret_cast<const bf16x8 *>(p + b1);
            fb[1][j] = *reinterpret_cast<const bf16x8 *>(p + b2);
            fb[2][j] = *reinterpret_cast<const bf16x8 *>(p + b3);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const char *p = Ab + boff + i * 16 * X6_ROWB;
            const bf16x8 f1 = *reinterpret_cast<const bf16x8 *>(p + a1);
            const bf16x8 f2 = *reinterpret_cast<const bf16x8 *>(p + a2);
            const bf16x8 f3 = *reinterpret_cast<const bf16x8 *>(p + a3);
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, fb[0][j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f2, fb[1][j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f3, fb[2][j], acc[i][j], 0, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // epilogue: as k_convg, per wave passes of 64 rows x 64 columns
    constexpr int EPI_ROWS = 64, EPI_PITCH = 68, NPASS = WROWS / EPI_ROWS, IPP = EPI_ROWS / 16;
    float *Cs = reinterpret_cast<float *>(smem) + wid * EPI_ROWS * EPI_PITCH;
#pragma unroll
    for (int h = 0; h < NPASS; ++h) {
#pragma unroll
        for (int i = 0; i < IPP; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    Cs[(i * 16 + (lane >> 4) * 4 + r) * EPI_PITCH + j * 16 + (lane & 15)] = acc[IPP * h + i][j][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        finish_batch<float, 8>(a, [&](int q, int &gm, int &gn0, const float *&src) {
            const int item = lane + 64 * q;
            const int row = item >> 3, ch = item & 7;
            gm = m0 + wm * WROWS + EPI_ROWS * h + row;
            gn0 = n0 + wn * WCOLS + ch * 8;
            src = Cs + row * EPI_PITCH + ch * 8;
            if (gm >= a.M || gn0 >= a.Cout) gm = -1;
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

// ---------------------------------------------------------------------------
// Winograd F(m x m, 3x3), m = 2, 4 or 6, for fp32 3x3 / stride 1 / pad 1
// convolutions (NHWC), a = m + 2:
//   V[xi][t][c] = (B^T d B)[xi] of the a x a input patch of output tile t
//   M[xi][t][k] = sum_c V[xi][t][c] U[xi][k][c]   (a*a batched GEMMs)
//   Y(t)        = A^T M A (+ bias, ReLU)           (m x m outputs)
// with U = G g G^T packed once per layer.  F(2,3): 2.25x fewer multiplies,
// transforms of 0/+-1 coefficients (error ~7e-7 relative in fp32 on
// 256-channel layers vs ~4e-7 direct); F(4,3): 4x fewer, coefficients up to
// 8 (Lavin's points 0, +-1, +-2; error ~1e-5); F(6,3): 5.06x fewer on whole
// tiles, points 0, +-1, +-2, +-1/2 (coefficients up to 32; error ~2x F(4,3)'s),
// used on the large maps where its 8x8 tiles waste little at the edges.
// ---------------------------------------------------------------------------
// one thread per (tile, channel): workgroup (blockIdx.x = tile, blockIdx.y =
// channel block of blockDim.x), so the tile coordinates are workgroup-uniform
// scalars (the per-thread 64-bit div / mod of a flat index cost more than the
// loads); sums over nonzero coefficients only
template <int M>
__global__ __launch_bounds__(256) void k_wino_in(const float *__restrict__ x, int N, int H, int W, int C, int TH,
                                                 int TW, float *__restrict__ V) {
    constexpr int A = WinoT<M>::A;
    const int t = blockIdx.x;
    const int c = blockIdx.y * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const long long T = (long long)N * TH * TW;
    const long long xs = T * C;  // stride between xi planes
    const int tx = t % TW, r = t / TW;
    const int ty = r % TH, n = r / TH;
    const int y0 = M * ty - 1, x0 = M * tx - 1;
    const float *xb = x + (long long)n * H * W * C + c;
    float d[A][A];
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {
            const int yy = y0 + i, xx = x0 + j;
            d[i][j] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? xb[((long long)yy * W + xx) * C] : 0.f;
        }
    float tt[A][A];  // B^T d
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < A; ++k)
                if (WinoT<M>::BT(i, k) != 0.f) acc = acc + WinoT<M>::BT(i, k) * d[k][j];
            tt[i][j] = acc;
        }
    float *vo = V + (long long)t * C + c;
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {  // (B^T d) B
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < A; ++k)
                if (WinoT<M>::BT(j, k) != 0.f) acc = acc + tt[i][k] * WinoT<M>::BT(j, k);
            vo[(A * i + j) * xs] = acc;
        }
}

// k_wino_in writing V straight into the bf16 plane layout of k_gemm_x6
// (split-plane mode): each thread transforms one channel of the tile into
// LDS ([xi][channel] fp32), then the workgroup re-reads 8 consecutive
// channels of one xi per item, splits them (x = hi + mid + lo exactly, as
// k_split_x6) and stores the three 16-B plane pieces.  Channel block = 256
// (or C); C % 16 == 0.
template <int M>
__global__ __launch_bounds__(256) void k_wino_in_x6(const float *__restrict__ x, int N, int H, int W, int C, int TH,
                                                    int TW, char *__restrict__ Vp) {
    constexpr int A = WinoT<M>::A, NB = A * A;
    __shared__ float s_v[NB * 256];
    const int t = blockIdx.x;
    const int cb = blockIdx.y * blockDim.x;
    const int c = cb + threadIdx.x;
    const long long T = (long long)N * TH * TW;
    const int tx = t % TW, r = t / TW;
    const int ty = r % TH, n = r / TH;
    const int y0 = M * ty - 1, x0 = M * tx - 1;
    if (c < C) {
        const float *xb = x + (long long)n * H * W * C + c;
        float d[A][A];
#pragma unroll
        for (int i = 0; i < A; ++i)
#pragma unroll
            for (int j = 0; j < A; ++j) {
                const int yy = y0 + i, xx = x0 + j;
                d[i][j] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? xb[((long long)yy * W + xx) * C] : 0.f;
            }
        float tt[A][A];
#pragma unroll
        for (int i = 0; i < A; ++i)
#pragma unroll
            for (int j = 0; j < A; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < A; ++k)
                    if (WinoT<M>::BT(i, k) != 0.f) acc = acc + WinoT<M>::BT(i, k) * d[k][j];
                tt[i][j] = acc;
            }
#pragma unroll
        for (int i = 0; i < A; ++i)
#pragma unroll
            for (int j = 0; j < A; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < A; ++k)
                    if (WinoT<M>::BT(j, k) != 0.f) acc = acc + tt[i][k] * WinoT<M>::BT(j, k);
                s_v[(A * i + j) * 256 + threadIdx.x] = acc;
            }
    }
    __syncthreads();
    const int g8n = (int)blockDim.x / 8;  // 8-channel groups of this block
    const long long rowb = (long long)C * 6;   // plane bytes of one V row (tile)
    for (int it = threadIdx.x; it < NB * g8n; it += blockDim.x) {
        const int xi = it / g8n, g8 = it - xi * g8n;
        const int c0 = cb + 8 * g8;
        if (c0 >= C) continue;
        const float4 u = *reinterpret_cast<const float4 *>(s_v + xi * 256 + 8 * g8);
        const float4 v = *reinterpret_cast<const float4 *>(s_v + xi * 256 + 8 * g8 + 4);
        const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        bf16x8 h, m, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const __bf16 hb = (__bf16)f[e];
            const float r1 = f[e] - (float)hb;
            const __bf16 mb = (__bf16)r1;
            h[e] = hb;
            m[e] = mb;
            l[e] = (__bf16)(r1 - (float)mb);
        }
        char *o = Vp + ((long long)xi * T + t) * rowb + (long long)(c0 >> 4) * X6_ROWB + ((c0 >> 3) & 1) * 16;
        *reinterpret_cast<bf16x8 *>(o) = h;
        *reinterpret_cast<bf16x8 *>(o + 32) = m;
        *reinterpret_cast<bf16x8 *>(o + 64) = l;
    }
}

// one thread per (tile, output channel), laid out as k_wino_in
template <int M>
__global__ __launch_bounds__(256) void k_wino_out(const float *__restrict__ Mx, int N, int OH, int OW, int K, int TH,
                                                  int TW, const float *__restrict__ bias, int relu,
                                                  float *__restrict__ out) {
    constexpr int A = WinoT<M>::A;
    const int t = blockIdx.x;
    const int k = blockIdx.y * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const long long T = (long long)N * TH * TW;
    const long long xs = T * K;
    const int tx = t % TW, r = t / TW;
    const int ty = r % TH, n = r / TH;
    const float *mi = Mx + (long long)t * K + k;
    float m[A][A];
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) m[i][j] = mi[(A * i + j) * xs];
    float sa[M][A];  // A^T m
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j < A; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q)
                if (WinoT<M>::AT(i, q) != 0.f) acc = acc + WinoT<M>::AT(i, q) * m[q][j];
            sa[i][j] = acc;
        }
    const float bv = bias ? bias[k] : 0.f;
    float *ob = out + (long long)n * OH * OW * K + k;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int oy = M * ty + i;
        if (oy >= OH) continue;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int ox = M * tx + j;
            if (ox >= OW) continue;
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q)
                if (WinoT<M>::AT(j, q) != 0.f) acc = acc + sa[i][q] * WinoT<M>::AT(j, q);
            float v = acc + bv;
            if (relu) v = v > 0.f ? v : 0.f;
            ob[((long long)oy * OW + ox) * K] = v;
        }
    }
}


// ---------------------------------------------------------------------------
// fp16 implicit-GEMM convolution on the ping-pong schedule (the fp16 layers
// the 256x256 tile takes: box head FCs, the FPN 3x3 outputs, the mask /
// keypoint head convs):  out[m][n] = act(sum_k A[m][k] W[n][k] + bias[n]
// (+ res)), A row m = the input pixels under output pixel m's taps (NHWC, K
// order tap outer, channel inner, Cin % 64 == 0), W = weights
// [Cout][KH][KW][Cin].
//
// Tile 256 x 256 per 512-thread workgroup (one per CU), 8 waves: group g =
// wid >> 2 owns output rows 128 g .. +127, wave (g, wn) a 128 x 64 block =
// 8 x 4 tiles of v_mfma_f32_16x16x32_f16 (128 fp32 accumulators per lane).
// K in tiles of 64 halves (128-B LDS rows, pieces XOR-swizzled by row), A and
// B of a K-tile staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, 8 per wave and K-tile; padding taps read a zero piece), two
// K-tile buffers (128 KiB).  (Measured against 32-deep K-tiles in four
// buffers with the DMA three K-tiles ahead: the deeper pipeline's extra
// barriers cost more than its lookahead gains, 3-7 % slower.)
//
// A K-tile is two phases (32-deep halves).  Every phase is, per wave,
//   R: 12 ds_read_b128 fragments (8 A + 4 B) [+ DMA issue / wait] lgkmcnt(0)
//      barrier
//   M: 32 MFMAs barrier
// and group 1 runs one barrier behind group 0, so between any two barriers
// one wave of every SIMD multiplies while the other reads.  Global barrier b
// opens interval b; group 0 runs R(p) in interval 2p and M(p) in 2p + 1,
// group 1 R(p) in 2p + 1 and M(p) in 2p + 2.  K-tile t is phases 2t, 2t + 1
// in buffer t & 1:
//   * its last reads (phase 2t + 1) retire (lgkmcnt(0)) before barriers
//     4t + 3 (group 0) and 4t + 4 (group 1);
//   * the DMA of K-tile t + 2 into the same buffer is issued in R(2t + 2),
//     intervals 4t + 4 / 4t + 5: after both (WAR);
//   * each wave waits for its own DMA of K-tile t + 1 (vmcnt(0): the only
//     vector-memory operations in the loop) in R(2t + 1), before barrier
//     4t + 3 / 4t + 4, and the first read of K-tile t + 1 is group 0's
//     R(2t + 2) in interval 4t + 4: after both (RAW; LDS-DMA data is
//     ordered for ds_read only by the issuer's vmcnt and a barrier).
// Rows past M / Cout are clamped to the last row (their products only reach
// outputs that are never stored).  The epilogue stages each wave's block
// through LDS (32 rows at a time) into finish_batch: bias, residual, ReLU,
// 16-B stores, the deconv pixel shuffle.
// fp16 layers (Cout >= 192, Cin % 64 == 0) from this many 256x256 tiles take
// the ping-pong kernel.  With eight forwards in flight every eligible layer
// on it ran the fp16 loop 2.8 % faster (thresholds 160 / 80 / 32 / 8 / 1:
// 4465-4491 / 4487-4497 / 4572-4584, then 4606-4615 / 4622-4650 / 4628-4648
// frames/s on a second box; profiles/r06_f16_pp_threshold/), but the small
// layers it takes over from the split-K register-staged kernel round
// differently, and the all-fp16 parity case of weight seed 35 then passes
// the detection checks on 23 of 32 frames, under its floor of 24 (150 -> 146
// of 160 over the five seeds): kept at 160
#ifndef MDX_F16_PP_MIN_TILES
#define MDX_F16_PP_MIN_TILES 160
#endif
constexpr int P16_THREADS = 512, P16_BM = 256, P16_BN = 256, P16_BK = 64;
constexpr int P16_ROWB = 128, P16_OPND = P16_BM * P16_ROWB, P16_BUF = 2 * P16_OPND, P16_LDS = 2 * P16_BUF;
constexpr int P16_EPI_PITCH = 68;  // floats per staged epilogue row (bank-conflict-free writes)

__device__ __forceinline__ void p16_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <typename TO>
__global__ __launch_bounds__(P16_THREADS, 1) void k_conv16_pp(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int tile;
    {
        const int L = blockIdx.x, nwg = a.tiles_total;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    }
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int m0 = tm * P16_BM, n0 = tn * P16_BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wn = wid & 3;

    // ---- LDS-DMA sources: instruction j of wave w fills tile rows
    // 32 w + 8 j .. + 7 of A (and of B); lane l writes row + (l >> 3), 16-B
    // slot l & 7, which holds the row's logical piece (l & 7) ^ ((row >> 1) & 7)
    const _Float16 *X = reinterpret_cast<const _Float16 *>(a.x);
    const _Float16 *Wt = reinterpret_cast<const _Float16 *>(a.w);
    const int ohw = a.OH * a.OW;
    int a_iy0[4], a_ix0[4];
    long long a_base[4];
    const _Float16 *b_src[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = 32 * wid + 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int gm = min(m0 + r, a.M - 1), gn = min(n0 + r, a.Cout - 1);
        const int b = gm / ohw, rem = gm - b * ohw, oy = rem / a.OW, ox = rem - oy * a.OW;
        a_iy0[j] = oy * a.stride - a.pad;
        a_ix0[j] = ox * a.stride - a.pad;
        a_base[j] = (long long)b * a.H * a.W * a.Cin + 8 * c;
        b_src[j] = Wt + (long long)gn * a.K + 8 * c;
    }
    char *const adst = smem + (32 * wid) * P16_ROWB;  // wave-uniform DMA bases (+ buffer, + j KiB)
    auto dma = [&](int t) {
        char *d = adst + (t & 1) * P16_BUF;
        const int k = t * P16_BK;
        const int tap = k / a.Cin, ci0 = k - tap * a.Cin;
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int iy = a_iy0[j] + ky, ix = a_ix0[j] + kx;
            const bool ok = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            const void *src = ok ? (const void *)(X + a_base[j] + ((long long)iy * a.W + ix) * a.Cin + ci0)
                                 : (const void *)g_zero16;
            glds16(src, d + j * 1024);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) glds16(b_src[j] + k, d + P16_OPND + j * 1024);
    };

    // ---- fragments: lane l reads row (l & 15) of each 16-row tile, logical
    // piece 4 s + (l >> 4) of the phase's half s (K elements 8 (l >> 4) ..
    // of the MFMA's 32)
    const int fr = lane & 15, fsw = (fr >> 1) & 7, fh = lane >> 4;
    const char *abase = smem + (grp * 128 + fr) * P16_ROWB;
    const char *bbase = smem + P16_OPND + (wn * 64 + fr) * P16_ROWB;
    half8 fa[8], fb[4];
    auto read_frags = [&](int buf, int s) {
        const int off = buf * P16_BUF + (((4 * s + fh) ^ fsw) << 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const half8 *>(bbase + off + j * 16 * P16_ROWB);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const half8 *>(abase + off + i * 16 * P16_ROWB);
    };

    float4v acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

    const int KT = a.K / P16_BK;
    dma(0);
    MDX_WAIT_VM(0);
    p16_barrier();               // K-tile 0 in LDS
    if (grp == 1) p16_barrier();  // group 1 one barrier behind
    for (int t = 0; t < KT; ++t) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            read_frags(t & 1, s);  // R
            if (t + 1 < KT) {
                if (s == 0)
                    dma(t + 1);
                else
                    MDX_WAIT_VM(0);
            }
            MDX_WAIT_LGKM0();
            p16_barrier();
#pragma unroll
            for (int i = 0; i < 8; ++i)  // M
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            p16_barrier();
        }
    }
    if (grp == 0) p16_barrier();  // every wave crosses the same number of barriers
    __syncthreads();              // the K-tile buffers become the epilogue staging

    // ---- epilogue: 32 rows of the wave's block at a time through its own
    // LDS rows (acc[i][j][r] = row 16 i + 4 (l >> 4) + r, column 16 j + (l & 15))
    float *ep = reinterpret_cast<float *>(smem) + wid * (32 * P16_EPI_PITCH);
    const int rowb = m0 + grp * 128, colb = n0 + wn * 64;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) ep[(16 * ii + 4 * fh + r) * P16_EPI_PITCH + 16 * j + fr] = acc[2 * p + ii][j][r];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        finish_batch<TO, 4>(a, [&](int q, int &gm, int &gn0, const float *&src) {
            const int c = lane + 64 * q, rr = c >> 3, cc = (c & 7) * 8;
            gm = rowb + 32 * p + rr;
            gn0 = colb + cc;
            if (gm >= a.M || gn0 >= a.Cout) gm = -1;
            src = ep + rr * P16_EPI_PITCH + cc;
        });
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

}  // namespace mdx

using namespace mdx;

// kernel chosen by the calling thread's last mdx_conv2d* call (measurement)
static thread_local int t_plan_kernel = -1, t_plan_ksplit = 0;

// dtype codes: 0 = fp32, 1 = fp16.  Kernel choice follows the policy in
// force on the calling thread (pol(): include/mdx.h, mdx_policy).
//
// LDS of a k_conv launch: stage buffers (one when the whole K is one step or
// the single-stage instance, else two) or the half-tile fp32 epilogue image
static size_t conv_lds(int bn, int ksteps, bool sb) {
    const size_t main_ = (ksteps == 1 || sb ? 1 : 2) * ((size_t)BM * PITCH + (size_t)bn * PITCH);
    const size_t epi = (size_t)(BM / 2) * (bn + 4) * 4;
    return main_ > epi ? main_ : epi;
}
// weight planes for the next split-plane launch on this thread (set by the
// model handle around a layer's conv call; see mdx::x3_weight_planes)
static thread_local const void *t_x3_wplanes = nullptr;
void mdx::x3_weight_planes(const void *planes) { t_x3_wplanes = planes; }

// launch of the split-plane fp32 kernel (LDS: double-buffered planes or the epilogue image)
// (with weight planes pending and K % 32 == 0: the pre-split-B instance; a.w,
// a.wbytes and a.bsw switch to the planes)
static void launch_x3(ConvArgs a, int bn, dim3 grid, hipStream_t s) {
    const mdx_policy &P = pol();
    const size_t stage = 3 * ((size_t)BM * X3_ROWB + (size_t)bn * X3_ROWB);
    const size_t lds_main = (a.ksteps == 1 ? 1 : 2) * stage;
    const size_t lds_epi = (size_t)(BM / 2) * (bn + 4) * 4;
    const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
    const bool pw = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && (long long)a.M * a.Cin * 4 < (1ll << 31);
    if (t_x3_wplanes && P.fp32_split == 6 && a.K % 32 == 0 && (long long)a.Cout * a.K * 6 < (1ll << 31)) {
        a.bsw = a.bsw / 4 * 6;
        a.w = t_x3_wplanes;
        a.wbytes = a.Cout * a.K * 6;
        if (bn == 64 && P.x3_single_stage) {
            // one LDS stage: the stage or the epilogue image
            const size_t lds1 = stage > lds_epi ? stage : lds_epi;
            if (pw)
                hipLaunchKernelGGL((k_conv_x3<float, 64, 6, true, true, true>), grid, dim3(CONV_THREADS), lds1, s, a);
            else
                hipLaunchKernelGGL((k_conv_x3<float, 64, 6, true, false, true>), grid, dim3(CONV_THREADS), lds1, s, a);
            return;
        }
        if (bn == 64 && pw)
            hipLaunchKernelGGL((k_conv_x3<float, 64, 6, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        else if (bn == 64)
            hipLaunchKernelGGL((k_conv_x3<float, 64, 6, true>), grid, dim3(CONV_THREADS), lds, s, a);
        else if (pw)
            hipLaunchKernelGGL((k_conv_x3<float, 128, 6, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        else
            hipLaunchKernelGGL((k_conv_x3<float, 128, 6, true>), grid, dim3(CONV_THREADS), lds, s, a);
        return;
    }
    if (bn == 64 && pw && P.fp32_split == 6) {
        hipLaunchKernelGGL((k_conv_x3<float, 64, 6, false, true>), grid, dim3(CONV_THREADS), lds, s, a);
        return;
    }
    if (bn == 64) {
        if (P.fp32_split == 9)
            hipLaunchKernelGGL((k_conv_x3<float, 64, 9>), grid, dim3(CONV_THREADS), lds, s, a);
        else
            hipLaunchKernelGGL((k_conv_x3<float, 64, 6>), grid, dim3(CONV_THREADS), lds, s, a);
    } else {
        if (P.fp32_split == 9)
            hipLaunchKernelGGL((k_conv_x3<float, 128, 9>), grid, dim3(CONV_THREADS), lds, s, a);
        else
            hipLaunchKernelGGL((k_conv_x3<float, 128, 6>), grid, dim3(CONV_THREADS), lds, s, a);
    }
}

// resident workgroups the split-K model assumes for the register-staged
// kernels (512: two per CU; 384-1024 measured neutral in round 3)
static const long long g_ks_slots = 512;

// split-K slice count for a launch of `tiles` output tiles and nk K-steps:
// minimise (block waves) x (K-steps per block + fixed cost) + reduction cost,
// with `slots` resident workgroups (2 on each of the 256 CUs; 1 for k_conv_x3)
static int choose_ksplit(long long tiles, int nk, long long M, int Cout, long long ws_bytes, long long slots = 512) {
    int best = 1;
    double best_cost = 1e30;
    for (int ks = 1; ks <= 8; ++ks) {
        if (ks > 1 && (nk / ks < 4 || (long long)ks * M * Cout * 4 > ws_bytes)) break;
        const long long waves = (tiles * ks + slots - 1) / slots;
        const double cost = (double)waves * ((nk + ks - 1) / ks + 4) + (ks > 1 ? 2.0 + ks : 0.0);
        if (cost < best_cost) {
            best_cost = cost;
            best = ks;
        }
    }
    return best;
}

extern "C" int64_t mdx_conv2d_workspace_bytes(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                              int pad) {
    const long long OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
    return 8ll * N * OH * OW * Cout * 4;
}

extern "C" int mdx_conv2d(const void *x, int N, int H, int W, int Cin, const void *w, const float *bias, int Cout,
                          int KH, int KW, int stride, int pad, const void *residual, int relu, int out_mode,
                          int in_dtype, int out_dtype, void *out, mdx_stream_t stream) {
    return mdx_conv2d_splitk(x, N, H, W, Cin, w, bias, Cout, KH, KW, stride, pad, residual, relu, out_mode, in_dtype,
                             out_dtype, out, 1, nullptr, 0, stream);
}

extern "C" int mdx_conv2d_splitk(const void *x, int N, int H, int W, int Cin, const void *w, const float *bias,
                                 int Cout, int KH, int KW, int stride, int pad, const void *residual, int relu,
                                 int out_mode, int in_dtype, int out_dtype, void *out, int ksplit, void *workspace,
                                 int64_t workspace_bytes, mdx_stream_t stream) {
    MDX_REQUIRE(x && w && out, "mdx_conv2d: null pointer");
    const mdx_policy &P = pol();
    MDX_REQUIRE(in_dtype == 0 || in_dtype == 1, "mdx_conv2d: in_dtype must be 0 (f32) or 1 (f16)");
    MDX_REQUIRE(out_dtype == 0 || out_dtype == 1, "mdx_conv2d: out_dtype must be 0 (f32) or 1 (f16)");
    const int VEC = in_dtype == 1 ? 8 : 4;
    MDX_REQUIRE(Cin % VEC == 0, "mdx_conv2d: Cin=%d must be a multiple of %d (pad channels)", Cin, VEC);
    MDX_REQUIRE(N > 0 && H > 0 && W > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
                "mdx_conv2d: bad shape");
    MDX_REQUIRE(out_mode == 0 || (out_mode == 1 && KH == 1 && KW == 1 && stride == 1 && pad == 0 && Cout % 4 == 0),
                "mdx_conv2d: out_mode 1 (deconv2x2) needs a 1x1/s1 GEMM with Cout = 4*Co");
    const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
    MDX_REQUIRE(OH > 0 && OW > 0, "mdx_conv2d: empty output");
    ConvArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.res = residual; a.out = out;
    a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
    a.OH = OH; a.OW = OW;
    const long long M = (long long)N * OH * OW;
    MDX_REQUIRE(M < (1ll << 31), "mdx_conv2d: M too large");
    a.M = (int)M;
    a.K = KH * KW * Cin;
    {
        const long long es = in_dtype == 1 ? 2 : 4;
        const long long xb = (long long)N * H * W * Cin * es, wb = (long long)Cout * a.K * es;
        MDX_REQUIRE(xb < (1ll << 31) && wb < (1ll << 31), "mdx_conv2d: operands above 2 GiB are not supported");
        a.xbytes = (int)xb;
        a.wbytes = (int)wb;
        const long long rb = residual ? M * Cout * (out_dtype == 1 ? 2 : 4) : 0;
        MDX_REQUIRE(rb < (1ll << 31), "mdx_conv2d: residual above 2 GiB is not supported");
        a.rbytes = (int)rb;
    }
    a.relu = relu;
    a.out_mode = out_mode;
    hipStream_t s = as_stream(stream);
    // fp32 narrow-output 1x1 layers (RPN / mask / box predictors)
    if (P.head_f32 && in_dtype == 0 && out_dtype == 0 && out_mode == 0 && KH == 1 && KW == 1 && stride == 1 &&
        pad == 0 && !residual && Cout <= 16 && Cin % 16 == 0 && Cin <= 1024 && (ksplit == 1 || ksplit == 0)) {
        a.tiles_n = 1;
        a.tiles_total = 1;
        a.ksplit = 1;
        const long long groups = (M + 15) / 16;
        const unsigned grid = (unsigned)std::min<long long>((groups + 3) / 4, 4096);
        switch (Cin / 16) {
#define MDX_HEAD_F32(KC_) \
    case KC_: hipLaunchKernelGGL(k_head_f32<KC_>, dim3(grid), dim3(256), 0, s, a); break;
            MDX_HEAD_F32(1) MDX_HEAD_F32(2) MDX_HEAD_F32(4) MDX_HEAD_F32(8) MDX_HEAD_F32(16) MDX_HEAD_F32(32)
            MDX_HEAD_F32(64)
#undef MDX_HEAD_F32
            default: goto general;  // other K: the general kernels
        }
        t_plan_kernel = MDX_CONV_KERNEL_HEAD1X1;
        t_plan_ksplit = 1;
        MDX_CHECK_LAUNCH("mdx_conv2d");
        return MDX_OK;
    }
general:
    // HBM-bound 1x1 layers: the streaming kernel
    if (P.stream1x1 && in_dtype == 1 && out_dtype == 0 && out_mode == 0 && KH == 1 && KW == 1 && stride == 1 &&
        pad == 0 && !residual && (Cin == 64 || Cin == 128 || Cin == 256) && Cout <= 16 && (ksplit == 1 || ksplit == 0)) {
        a.tiles_n = 1;
        a.tiles_total = (int)ceil_div(M, 128);
        a.ksplit = 1;
        if (Cin == 64)
            hipLaunchKernelGGL(k_conv1x1_head<2>, dim3(a.tiles_total), dim3(256), 0, s, a);
        else if (Cin == 128)
            hipLaunchKernelGGL(k_conv1x1_head<4>, dim3(a.tiles_total), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL(k_conv1x1_head<8>, dim3(a.tiles_total), dim3(256), 0, s, a);
        t_plan_kernel = MDX_CONV_KERNEL_HEAD1X1;
        t_plan_ksplit = 1;
        MDX_CHECK_LAUNCH("mdx_conv2d");
        return MDX_OK;
    }
    if (P.stream1x1 && in_dtype == 1 && out_dtype == 1 && out_mode == 0 && KH == 1 && KW == 1 && stride == 1 &&
        pad == 0 && (Cin == 64 || Cin == 128 || (Cin == 256 && (Cout == 64 || P.stream1x1 == 2))) && Cout % 64 == 0 &&
        (ksplit == 1 || ksplit == 0) && M >= P.stream1x1_min_m) {
        // (K = 256 with Cout > 64 stays on the 256x256 kernel: measured faster)
        a.tiles_n = Cout / 64;
        a.tiles_total = (int)(ceil_div(M, 128) * a.tiles_n);
        a.ksplit = 1;
        if (Cin == 64)
            hipLaunchKernelGGL(k_conv1x1_stream<2>, dim3(a.tiles_total), dim3(256), 0, s, a);
        else if (Cin == 128)
            hipLaunchKernelGGL(k_conv1x1_stream<4>, dim3(a.tiles_total), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL(k_conv1x1_stream<8>, dim3(a.tiles_total), dim3(256), 0, s, a);
        t_plan_kernel = MDX_CONV_KERNEL_STREAM1X1;
        t_plan_ksplit = 1;
        MDX_CHECK_LAUNCH("mdx_conv2d");
        return MDX_OK;
    }
    // fp16 layers with Cin % 64 == 0: the LDS-DMA pipelined kernels -- the
    // 128x128 tile (DMA pieces interleaved with the MFMAs) for layers with
    // many tiles, the 256x256 tile by policy, else the register-staged kernel
    // (with split-K) below, which serves the small grids better
    // fp32 operands (Cin % 32 == 0, fp32 out): the 256x256 kernel on 16x16x4 f32
    // MFMAs, same LDS image (64-B rows of 16 floats)
    const bool x3 = in_dtype == 0 && out_dtype == 0 && P.fp32_split;
    // (mode 4: as 2, also while the split-plane mode routes the other fp32
    // layers to k_conv_x3 -- a diagnostic for kernel-level A/B runs)
    const bool dma_f32 = in_dtype == 0 && out_dtype == 0 && Cin % 32 == 0 && P.dma_f32 && (!x3 || P.dma_f32 == 4);
    if (((in_dtype == 1 && Cin % 64 == 0) || dma_f32) && (ksplit == 1 || ksplit == 0) &&
        KH * KW * Cin > P.narrow_kmax) {
        const int subk = in_dtype == 1 ? 32 : 16;  // K elements per 64-B substep
        const long long t128 = ceil_div(M, 128) * ceil_div(Cout, 128);
        if (in_dtype == 0 && P.dma_f32 == 1 && Cout > 64 && (P.large_tiles == 2 || t128 >= 512)) {
            // fp32: the 128x128 LDS-DMA tile, two workgroups per CU (their
            // barriers interleave, so one wave's fragment reads overlap the
            // other's MFMA bursts)
            using G4 = GTile<4>;
            a.tiles_n = (int)ceil_div(Cout, G4::BN);
            a.tiles_total = (int)t128;
            a.ksplit = 1;
            a.ksteps = a.K / subk;
            hipLaunchKernelGGL((k_convg<float, float, 4, false>), dim3(a.tiles_total), dim3(G4::THREADS), G4::LDS, s,
                               a);
            t_plan_kernel = MDX_CONV_KERNEL_DMA128;
            t_plan_ksplit = 1;
            MDX_CHECK_LAUNCH("mdx_conv2d");
            return MDX_OK;
        }
        if (in_dtype == 1 && (P.dma128 == 2 || (P.dma128 == 1 && Cout > 64 && t128 >= P.dma128_min_tiles))) {
            using G4 = GTile<4>;
            a.tiles_n = (int)ceil_div(Cout, G4::BN);
            a.tiles_total = (int)t128;
            a.ksplit = 1;
            a.ksteps = a.K / 32;
            if (out_dtype == 1 && P.dma128_interleave)
                hipLaunchKernelGGL((k_convg<_Float16, _Float16, 4, true>), dim3(a.tiles_total), dim3(G4::THREADS), G4::LDS, s, a);
            else if (out_dtype == 1)
                hipLaunchKernelGGL((k_convg<_Float16, _Float16, 4, false>), dim3(a.tiles_total), dim3(G4::THREADS), G4::LDS, s,
                                   a);
            else
                hipLaunchKernelGGL((k_convg<_Float16, float, 4, false>), dim3(a.tiles_total), dim3(G4::THREADS), G4::LDS, s, a);
            t_plan_kernel = MDX_CONV_KERNEL_DMA128;
            t_plan_ksplit = 1;
            MDX_CHECK_LAUNCH("mdx_conv2d");
            return MDX_OK;
        }
        const long long t256 = ceil_div(M, G_BM) * ceil_div(Cout, G_BN);
        const bool big = Cout >= 192 && (in_dtype == 1 || P.dma_f32 == 3 ? t256 >= (P.f16_pingpong ? MDX_F16_PP_MIN_TILES : 384)
                                                                            : t256 >= 500 && a.K >= 1024);
        // fp16: the 256x128 tile (two workgroups per CU) in place of 256x256
        // (large-tile modes 3: whenever eligible, 4: the layers mode 1 takes)
        if (in_dtype == 1 && (P.large_tiles == 3 || (P.large_tiles == 4 && big))) {
            using G6 = GTile<6>;
            a.tiles_n = (int)ceil_div(Cout, G6::BN);
            a.tiles_total = (int)(ceil_div(M, G6::BM) * a.tiles_n);
            a.ksplit = 1;
            a.ksteps = a.K / subk;
            if (out_dtype == 1)
                hipLaunchKernelGGL((k_convg<_Float16, _Float16, 6, false>), dim3(a.tiles_total), dim3(G6::THREADS),
                                   G6::LDS, s, a);
            else
                hipLaunchKernelGGL((k_convg<_Float16, float, 6, false>), dim3(a.tiles_total), dim3(G6::THREADS),
                                   G6::LDS, s, a);
            t_plan_kernel = MDX_CONV_KERNEL_DMA256;
            t_plan_ksplit = 1;
            MDX_CHECK_LAUNCH("mdx_conv2d");
            return MDX_OK;
        }
        if (P.large_tiles == 2 || P.large_tiles == 3 || ((P.large_tiles == 1 || P.large_tiles == 4) && big)) {
            a.tiles_n = (int)ceil_div(Cout, G_BN);
            a.tiles_total = (int)t256;
            a.ksplit = 1;
            a.ksteps = a.K / subk;
            const dim3 grid256((unsigned)a.tiles_total);
            if (in_dtype == 1 && P.f16_pingpong) {  // fp16: the ping-pong kernel
                if (out_dtype == 1)
                    hipLaunchKernelGGL((k_conv16_pp<_Float16>), grid256, dim3(P16_THREADS), P16_LDS, s, a);
                else
                    hipLaunchKernelGGL((k_conv16_pp<float>), grid256, dim3(P16_THREADS), P16_LDS, s, a);
                t_plan_kernel = MDX_CONV_KERNEL_PP16;
                t_plan_ksplit = 1;
                MDX_CHECK_LAUNCH("mdx_conv2d");
                return MDX_OK;
            }
            // (the interleaved schedule spills at the 8-wave tile's 256-VGPR budget)
            if (in_dtype == 0)
                hipLaunchKernelGGL((k_convg<float, float, 8, false>), grid256, dim3(G_THREADS), G_LDS, s, a);
            else if (out_dtype == 1)
                hipLaunchKernelGGL((k_convg<_Float16, _Float16, 8, false>), grid256, dim3(G_THREADS), G_LDS, s, a);
            else
                hipLaunchKernelGGL((k_convg<_Float16, float, 8, false>), grid256, dim3(G_THREADS), G_LDS, s, a);
            t_plan_kernel = MDX_CONV_KERNEL_DMA256;
            t_plan_ksplit = 1;
            MDX_CHECK_LAUNCH("mdx_conv2d");
            return MDX_OK;
        }
    }
    // 64-wide N tile: no wasted MFMA columns for 64-channel layers; more
    // workgroups per CU for the small-K layers
    const bool narrow = Cout <= 64 || a.K <= P.narrow_kmax || (x3 && P.x3_narrow);
    const int bn = narrow ? 64 : BN;
    const int tiles_m = (int)ceil_div(M, BM), tiles_n = (int)ceil_div(Cout, bn);
    a.tiles_n = tiles_n;
    a.tiles_total = tiles_m * tiles_n;
    const int nk = (a.K + (in_dtype == 1 ? 64 : 32) - 1) / (in_dtype == 1 ? 64 : 32);
    if (ksplit <= 0)
        ksplit = (workspace && Cout % 8 == 0) ? choose_ksplit(a.tiles_total, nk, M, Cout, workspace_bytes, x3 ? 256 : g_ks_slots)
                                              : 1;
    MDX_REQUIRE(ksplit == 1 || (workspace && Cout % 8 == 0 && (long long)ksplit * M * Cout * 4 <= workspace_bytes),
                "mdx_conv2d: split-K needs Cout %% 8 == 0 and a workspace of ksplit*M*Cout*4 bytes");
    ksplit = ksplit > nk ? nk : ksplit;
    a.ksteps = (nk + ksplit - 1) / ksplit;
    a.ksplit = (nk + a.ksteps - 1) / a.ksteps;
    a.part = reinterpret_cast<float *>(workspace);
    a.epi_direct = P.direct_epilogue && out_dtype == 0;
    // stage buffers: one when the whole K is one step, else two; epilogue
    // image: half the tile in fp32
    const size_t lds_main = (a.ksteps == 1 ? 1 : 2) * ((size_t)BM * PITCH + (size_t)bn * PITCH);
    const size_t lds_epi = (size_t)(BM / 2) * (bn + 4) * 4;
    const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
    if (x3) {
        launch_x3(a, bn, dim3(a.tiles_total, a.ksplit), s);
        if (a.ksplit > 1)
            hipLaunchKernelGGL((k_conv_reduce<float>), dim3((unsigned)ceil_div(M * (Cout / 8), 256)), dim3(256), 0, s, a);
        t_plan_kernel = narrow ? MDX_CONV_KERNEL_X3_64 : MDX_CONV_KERNEL_X3_128;
        t_plan_ksplit = a.ksplit;
        MDX_CHECK_LAUNCH("mdx_conv2d");
        return MDX_OK;
    }
    const bool pw = P.pointwise && KH == 1 && KW == 1 && pad == 0;
    // (mode 3: the fp16 register-staged PW layers too; the fp16 model's big
    // layers stay on the LDS-DMA kernels)
    // (mode 4: as 3, plus the fp16 KxK layers the LDS-DMA kernels do not take)
    const bool sb = P.single_stage && ((in_dtype == 0 && out_dtype == 0) || (P.single_stage >= 3 && in_dtype == 1 && out_dtype == 1));
    const bool sbg = P.single_stage >= 2 && !pw &&
                     ((in_dtype == 0 && out_dtype == 0) || (P.single_stage >= 4 && in_dtype == 1 && out_dtype == 1));
#define MDX_LAUNCH_CONV(TI_, TO_)                                                                           \
    do {                                                                                                    \
        const dim3 grid(a.tiles_total, a.ksplit);                                                           \
        if (narrow && pw && sb)                                                                             \
            hipLaunchKernelGGL((k_conv_sb<TI_, TO_, 64>), grid, dim3(CONV_THREADS),          \
                               conv_lds(64, a.ksteps, true), s, a);                                         \
        else if (!narrow && pw && sb)                                                                       \
            hipLaunchKernelGGL((k_conv_sb<TI_, TO_, 128>), grid, dim3(CONV_THREADS),         \
                               conv_lds(128, a.ksteps, true), s, a);                                        \
        else if (narrow && sbg)                                                                             \
            hipLaunchKernelGGL((k_conv_sbg<TI_, TO_, 64>), grid, dim3(CONV_THREADS),                         \
                               conv_lds(64, a.ksteps, true), s, a);                                         \
        else if (!narrow && sbg)                                                                            \
            hipLaunchKernelGGL((k_conv_sbg<TI_, TO_, 128>), grid, dim3(CONV_THREADS),                        \
                               conv_lds(128, a.ksteps, true), s, a);                                        \
        else if (narrow && pw)                                                                              \
            hipLaunchKernelGGL((k_conv<TI_, TO_, 64, false, true>), grid, dim3(CONV_THREADS), lds, s, a);    \
        else if (narrow)                                                                                    \
            hipLaunchKernelGGL((k_conv<TI_, TO_, 64>), grid, dim3(CONV_THREADS), lds, s, a);                 \
        else if (pw)                                                                                        \
            hipLaunchKernelGGL((k_conv<TI_, TO_, 128, false, true>), grid, dim3(CONV_THREADS), lds, s, a);   \
        else                                                                                                \
            hipLaunchKernelGGL((k_conv<TI_, TO_, 128>), grid, dim3(CONV_THREADS), lds, s, a);                \
        if (a.ksplit > 1)                                                                                   \
            hipLaunchKernelGGL((k_conv_reduce<TO_>), dim3((unsigned)ceil_div(M * (Cout / 8), 256)), dim3(256), \
                               0, s, a);                                                                    \
    } while (0)
    if (in_dtype == 1 && out_dtype == 1)
        MDX_LAUNCH_CONV(_Float16, _Float16);
    else if (in_dtype == 1 && out_dtype == 0)
        MDX_LAUNCH_CONV(_Float16, float);
    else if (in_dtype == 0 && out_dtype == 0)
        MDX_LAUNCH_CONV(float, float);
    else
        MDX_LAUNCH_CONV(float, _Float16);
#undef MDX_LAUNCH_CONV
    t_plan_kernel = narrow ? (pw ? (sb ? MDX_CONV_KERNEL_SB64 : MDX_CONV_KERNEL_PW64)
                                 : (sbg ? MDX_CONV_KERNEL_SBG64 : MDX_CONV_KERNEL_REG64))
                           : (pw ? (sb ? MDX_CONV_KERNEL_SB128 : MDX_CONV_KERNEL_PW128)
                                 : (sbg ? MDX_CONV_KERNEL_SBG128 : MDX_CONV_KERNEL_REG128));
    t_plan_ksplit = a.ksplit;
    MDX_CHECK_LAUNCH("mdx_conv2d");
    return MDX_OK;
}

extern "C" int64_t mdx_x6_plane_bytes(int64_t rows, int K) {
    if (rows < 0 || K <= 0 || K % 16) return -1;
    return rows * (int64_t)K * 6;
}

extern "C" int mdx_split_x6(const float *x, int64_t rows, int K, int64_t ldx, void *out, mdx_stream_t stream) {
    MDX_REQUIRE(x && out, "mdx_split_x6: null pointer");
    MDX_REQUIRE(rows >= 0 && K > 0 && K % 16 == 0 && ldx >= K && ldx % 4 == 0,
                "mdx_split_x6: K %% 16 == 0, ldx >= K and ldx %% 4 == 0 required");
    MDX_REQUIRE((reinterpret_cast<uintptr_t>(x) % 16) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0,
                "mdx_split_x6: 16-B aligned buffers required");
    if (rows == 0) return MDX_OK;
    const long long items = rows * (long long)(K / 8);
    const unsigned grid = (unsigned)std::min<long long>((items + 255) / 256, 1 << 16);
    hipLaunchKernelGGL(k_split_x6, dim3(grid), dim3(256), 0, as_stream(stream), x, (long long)rows, K, (long long)ldx,
                       reinterpret_cast<char *>(out));
    MDX_CHECK_LAUNCH("mdx_split_x6");
    return MDX_OK;
}

extern "C" int mdx_gemm_x6(const void *a_planes, const void *b_planes, const float *bias, int M, int N, int K,
                           const float *residual, int relu, float *out, mdx_stream_t stream) {
    MDX_REQUIRE(a_planes && b_planes && out, "mdx_gemm_x6: null pointer");
    MDX_REQUIRE(M > 0 && N > 0 && K > 0 && K % 16 == 0, "mdx_gemm_x6: M, N > 0 and K %% 16 == 0 required");
    MDX_REQUIRE(!residual || (long long)M * N * 4 < (1ll << 31), "mdx_gemm_x6: residual above 2 GiB");
    ConvArgs a{};
    a.x = a_planes; a.w = b_planes; a.bias = bias; a.res = residual; a.out = out;
    a.H = M; a.W = 1; a.Cin = K; a.Cout = N; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
    a.OH = M; a.OW = 1; a.M = M; a.K = K;
    a.relu = relu; a.out_mode = 0;
    a.rbytes = residual ? (int)((long long)M * N * 4) : 0;
    a.tiles_n = (int)ceil_div(N, X6_BN);
    a.tiles_total = (int)(ceil_div(M, X6_BM) * a.tiles_n);
    a.ksplit = 1;
    a.ksteps = K / 16;
    hipLaunchKernelGGL(k_gemm_x6, dim3((unsigned)a.tiles_total), dim3(X6_THREADS), X6_LDS, as_stream(stream), a);
    t_plan_kernel = MDX_CONV_KERNEL_X6DMA;
    t_plan_ksplit = 1;
    MDX_CHECK_LAUNCH("mdx_gemm_x6");
    return MDX_OK;
}

// A bottleneck's conv3 (1x1 over x, N x H x W x Cin) and its projection
// shortcut (1x1 / stride2 over x2, N x H2 x W2 x Cin2) as ONE GEMM over the
// concatenated K = Cin + Cin2: out = act(x . W[:, :Cin] + x2_strided .
// W[:, Cin:] + bias), w packed [Cout][Cin + Cin2], bias = b3 + b_sc.  Saves
// the shortcut's output write and its re-read as the residual.
extern "C" int mdx_conv2d_dual(const void *x, int N, int H, int W, int Cin, const void *x2, int H2, int W2, int Cin2,
                               int stride2, const void *w, const float *bias, int Cout, int relu, int dtype, void *out,
                               void *workspace, int64_t workspace_bytes, mdx_stream_t stream) {
    MDX_REQUIRE(x && x2 && w && out, "mdx_conv2d_dual: null pointer");
    const mdx_policy &P = pol();
    MDX_REQUIRE(dtype == 0 || dtype == 1, "mdx_conv2d_dual: dtype must be 0 (f32) or 1 (f16)");
    const int BKd = dtype == 1 ? 64 : 32;
    MDX_REQUIRE(N > 0 && H > 0 && W > 0 && Cout > 0 && stride2 > 0 && Cin > 0 && Cin2 > 0,
                "mdx_conv2d_dual: bad shape");
    MDX_REQUIRE(Cin % BKd == 0 && Cin2 % BKd == 0,
                "mdx_conv2d_dual: Cin=%d and Cin2=%d must be multiples of %d", Cin, Cin2, BKd);
    MDX_REQUIRE((H - 1) * stride2 < H2 && (W - 1) * stride2 < W2, "mdx_conv2d_dual: x2 too small for the stride");
    const long long es = dtype == 1 ? 2 : 4;
    const long long M = (long long)N * H * W;
    const long long xb = M * Cin * es, x2b = (long long)N * H2 * W2 * Cin2 * es, wb = (long long)Cout * (Cin + Cin2) * es;
    MDX_REQUIRE(M < (1ll << 31) && xb < (1ll << 31) && x2b < (1ll << 31) && wb < (1ll << 31),
                "mdx_conv2d_dual: operands above 2 GiB are not supported");
    ConvArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.res = nullptr; a.out = out;
    a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
    a.OH = H; a.OW = W;
    a.M = (int)M;
    a.K = Cin + Cin2;
    a.xbytes = (int)xb;
    a.wbytes = (int)wb;
    a.relu = relu;
    a.out_mode = 0;
    a.x2 = x2; a.K1 = Cin; a.H2 = H2; a.W2 = W2; a.Cin2 = Cin2; a.stride2 = stride2; a.x2bytes = (int)x2b;
    const bool narrow = Cout <= 64 || a.K <= P.narrow_kmax;
    const int bn = narrow ? 64 : BN;
    a.tiles_n = (int)ceil_div(Cout, bn);
    a.tiles_total = (int)(ceil_div(M, BM) * a.tiles_n);
    const int nk = (a.K + BKd - 1) / BKd;
    int ksplit = (workspace && Cout % 8 == 0) ? choose_ksplit(a.tiles_total, nk, M, Cout, workspace_bytes, g_ks_slots) : 1;
    ksplit = ksplit > nk ? nk : ksplit;
    a.ksteps = (nk + ksplit - 1) / ksplit;
    a.ksplit = (nk + a.ksteps - 1) / a.ksteps;
    a.part = reinterpret_cast<float *>(workspace);
    a.epi_direct = P.direct_epilogue && dtype == 0;
    const size_t lds_main = (a.ksteps == 1 ? 1 : 2) * ((size_t)BM * PITCH + (size_t)bn * PITCH);
    const size_t lds_epi = (size_t)(BM / 2) * (bn + 4) * 4;
    const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
    hipStream_t s = as_stream(stream);
    const dim3 grid(a.tiles_total, a.ksplit);
    const bool sb = dtype == 0 && P.single_stage;
    if (dtype == 0) {
        if (narrow && sb)
            hipLaunchKernelGGL((k_conv_sb<float, float, 64, true>), grid, dim3(CONV_THREADS),
                               conv_lds(64, a.ksteps, true), s, a);
        else if (sb)
            hipLaunchKernelGGL((k_conv_sb<float, float, 128, true>), grid, dim3(CONV_THREADS),
                               conv_lds(128, a.ksteps, true), s, a);
        else if (narrow)
            hipLaunchKernelGGL((k_conv<float, float, 64, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        else
            hipLaunchKernelGGL((k_conv<float, float, 128, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        if (a.ksplit > 1)
            hipLaunchKernelGGL((k_conv_reduce<float>), dim3((unsigned)ceil_div(M * (Cout / 8), 256)), dim3(256), 0, s, a);
    } else {
        if (narrow)
            hipLaunchKernelGGL((k_conv<_Float16, _Float16, 64, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        else
            hipLaunchKernelGGL((k_conv<_Float16, _Float16, 128, true, true>), grid, dim3(CONV_THREADS), lds, s, a);
        if (a.ksplit > 1)
            hipLaunchKernelGGL((k_conv_reduce<_Float16>), dim3((unsigned)ceil_div(M * (Cout / 8), 256)), dim3(256), 0,
                               s, a);
    }
    t_plan_kernel = narrow ? (sb ? MDX_CONV_KERNEL_SBDUAL64 : MDX_CONV_KERNEL_DUAL64)
                           : (sb ? MDX_CONV_KERNEL_SBDUAL128 : MDX_CONV_KERNEL_DUAL128);
    t_plan_ksplit = a.ksplit;
    MDX_CHECK_LAUNCH("mdx_conv2d_dual");
    return MDX_OK;
}

extern "C" int mdx_conv2d_last_plan(int *kernel, int *ksplit) {
    MDX_REQUIRE(kernel && ksplit, "mdx_conv2d_last_plan: null pointer");
    *kernel = t_plan_kernel;
    *ksplit = t_plan_ksplit;
    return MDX_OK;
}

// ---------------------------------------------------------------------------
// Winograd F(m x m, 3x3) host side
// ---------------------------------------------------------------------------

extern "C" int mdx_winograd_weights(const float *w, int Cout, int Cin, int m, float *U) {
    MDX_REQUIRE(w && U && Cout > 0 && Cin > 0 && (m == 2 || m == 4 || m == 6), "mdx_winograd_weights: bad args");
    // U = G g G^T (in double, rounded once)
    static const double G2[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    static const double G4[6][3] = {{1.0 / 4, 0, 0},
                                    {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                    {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                    {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                    {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                    {0, 0, 1}};
    static const double G6[8][3] = {{1, 0, 0},
                                    {-2.0 / 9, -2.0 / 9, -2.0 / 9},
                                    {-2.0 / 9, 2.0 / 9, -2.0 / 9},
                                    {1.0 / 90, 1.0 / 45, 2.0 / 45},
                                    {1.0 / 90, -1.0 / 45, 2.0 / 45},
                                    {32.0 / 45, 16.0 / 45, 8.0 / 45},
                                    {32.0 / 45, -16.0 / 45, 8.0 / 45},
                                    {0, 0, 1}};
    const int A = m + 2;
    auto G = [&](int i, int j) { return m == 2 ? G2[i][j] : m == 4 ? G4[i][j] : G6[i][j]; };
    const long long plane = (long long)Cout * Cin;
    for (int o = 0; o < Cout; ++o)
        for (int i = 0; i < Cin; ++i) {
            const float *g = w + ((long long)o * Cin + i) * 9;
            double tg[8][3];
            for (int a = 0; a < A; ++a)
                for (int c = 0; c < 3; ++c) tg[a][c] = G(a, 0) * g[0 * 3 + c] + G(a, 1) * g[1 * 3 + c] + G(a, 2) * g[2 * 3 + c];
            for (int a = 0; a < A; ++a)
                for (int b = 0; b < A; ++b)
                    U[(long long)(A * a + b) * plane + (long long)o * Cin + i] =
                        (float)(tg[a][0] * G(b, 0) + tg[a][1] * G(b, 1) + tg[a][2] * G(b, 2));
        }
    return MDX_OK;
}

extern "C" int64_t mdx_winograd_workspace_bytes(int N, int H, int W, int Cin, int Cout, int m) {
    if (m != 2 && m != 4 && m != 6) return -1;
    const long long T = (long long)N * ((H + m - 1) / m) * ((W + m - 1) / m);
    // fp32 V + M, or (split-plane mode) V as bf16 planes (6 B per value) + M
    return (long long)(m + 2) * (m + 2) * T * (Cin * 6 + Cout * 4) + 256;
}

// policy 6: F(6,3) where its 8x8 tiles execute under 0.9x the tile products
// of F(4,3)'s 6x6 (the large maps; edge tiles of the small ones waste the
// gain), else F(4,3)
static const int g_wino6_pct = 90;
extern "C" int mdx_winograd_tile(int H, int W, int mode) {
    if (mode != 6) return mode;
    const long long p6 = 64ll * ((H + 5) / 6) * ((W + 5) / 6), p4 = 36ll * ((H + 3) / 4) * ((W + 3) / 4);
    return 100 * p6 < g_wino6_pct * p4 ? 6 : 4;
}

static thread_local WinoProbe *t_wino_probe = nullptr;
void mdx::wino_probe(WinoProbe *p) { t_wino_probe = p; }
WinoProbe *mdx::wino_probe_current() { return t_wino_probe; }
void mdx::set_last_plan(int kernel, int ksplit) {
    t_plan_kernel = kernel;
    t_plan_ksplit = ksplit;
}

// the model packs Winograd weight planes (and so runs the split-plane
// Winograd GEMMs on k_gemm_x6) only when MDX_WINO_X6 is set: the split-plane
// loop measured 4 % slower with them (1481 / 1494 vs 1543 / 1574 frames/s,
// profiles/r04_experiments.json), the plane input transform writing 6 B per
// value against 4
static const bool g_wino_x6_model = getenv("MDX_WINO_X6") != nullptr;
bool mdx::winograd_planes_enabled() { return g_wino_x6_model; }

static int winograd_impl(const float *x, int N, int H, int W, int Cin, const float *U, const void *Up,
                         const float *bias, int Cout, int relu, int m, float *out, void *workspace,
                         int64_t workspace_bytes, mdx_stream_t stream);

extern "C" int mdx_conv3x3_winograd(const float *x, int N, int H, int W, int Cin, const float *U, const float *bias,
                                    int Cout, int relu, int m, float *out, void *workspace, int64_t workspace_bytes,
                                    mdx_stream_t stream) {
    return winograd_impl(x, N, H, W, Cin, U, nullptr, bias, Cout, relu, m, out, workspace, workspace_bytes, stream);
}

extern "C" int mdx_conv3x3_winograd_x6(const float *x, int N, int H, int W, int Cin, const float *U,
                                       const void *U_planes, const float *bias, int Cout, int relu, int m, float *out,
                                       void *workspace, int64_t workspace_bytes, mdx_stream_t stream) {
    MDX_REQUIRE(U_planes, "mdx_conv3x3_winograd_x6: null U planes");
    return winograd_impl(x, N, H, W, Cin, U, U_planes, bias, Cout, relu, m, out, workspace, workspace_bytes, stream);
}

static int winograd_impl(const float *x, int N, int H, int W, int Cin, const float *U, const void *Up,
                         const float *bias, int Cout, int relu, int m, float *out, void *workspace,
                         int64_t workspace_bytes, mdx_stream_t stream) {
    MDX_REQUIRE(x && U && out && workspace, "mdx_conv3x3_winograd: null pointer");
    const mdx_policy &P = pol();
    MDX_REQUIRE(m == 2 || m == 4 || m == 6, "mdx_conv3x3_winograd: tile m must be 2, 4 or 6");
    MDX_REQUIRE(N > 0 && H > 0 && W > 0 && Cin % 4 == 0 && Cout % 8 == 0,
                "mdx_conv3x3_winograd: Cin %% 4 == 0 and Cout %% 8 == 0 required");
    MDX_REQUIRE(workspace_bytes >= mdx_winograd_workspace_bytes(N, H, W, Cin, Cout, m),
                "mdx_conv3x3_winograd: workspace too small");
    MDX_REQUIRE((reinterpret_cast<uintptr_t>(workspace) % 16) == 0, "mdx_conv3x3_winograd: 16-B aligned workspace");
    const int A = m + 2, NB = A * A;
    const int TH = (H + m - 1) / m, TW = (W + m - 1) / m;
    const long long T = (long long)N * TH * TW;
    MDX_REQUIRE(T < (1ll << 31) && T * Cin * 4 < (1ll << 31) && T * Cout * 4 < (1ll << 31) &&
                    (long long)Cout * Cin * 4 < (1ll << 31),
                "mdx_conv3x3_winograd: layer too large");
    hipStream_t s = as_stream(stream);
    // split-plane mode with the U planes: V written as planes, the NB GEMMs on
    // the 256 x 256 LDS-DMA plane kernel
    const bool planes = Up && P.fp32_split == 6 && Cin % 16 == 0 &&
                        T * Cin * 6 < (1ll << 31) && (long long)Cout * Cin * 6 < (1ll << 31);
    WinoProbe *probe = t_wino_probe;
    float *V = reinterpret_cast<float *>(workspace);
    float *Mx = planes ? reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + NB * T * Cin * 6)
                       : V + NB * T * Cin;
    auto mark = [&](int i) {
        if (probe) (void)hipEventRecord(probe->ev[i], s);
    };
    mark(0);
    // transforms: workgroup = (tile, block of up to 256 channels)
    auto tgrid = [&](int ch, unsigned &bd) {
        bd = (unsigned)std::min(256, (ch + 63) / 64 * 64);
        return dim3((unsigned)T, (unsigned)((ch + (int)bd - 1) / (int)bd));
    };
    if (planes) {
        unsigned bd;
        const dim3 grid = tgrid(Cin, bd);
        char *Vp = reinterpret_cast<char *>(workspace);
        if (m == 2)
            hipLaunchKernelGGL(k_wino_in_x6<2>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, Vp);
        else if (m == 4)
            hipLaunchKernelGGL(k_wino_in_x6<4>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, Vp);
        else
            hipLaunchKernelGGL(k_wino_in_x6<6>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, Vp);
    } else {
        unsigned bd;
        const dim3 grid = tgrid(Cin, bd);
        if (m == 2)
            hipLaunchKernelGGL(k_wino_in<2>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, V);
        else if (m == 4)
            hipLaunchKernelGGL(k_wino_in<4>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, V);
        else
            hipLaunchKernelGGL(k_wino_in<6>, grid, dim3(bd), 0, s, x, N, H, W, Cin, TH, TW, V);
    }
    mark(1);
    mark(2);
    int gemm_kernel;
    // NB GEMMs M[xi] (T x Cout) = V[xi] (T x Cin) U[xi]^T in one launch (grid.z)
    ConvArgs a{};
    a.x = V; a.w = U; a.bias = nullptr; a.res = nullptr; a.out = Mx;
    a.H = (int)T; a.W = 1; a.Cin = Cin; a.Cout = Cout; a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
    a.OH = (int)T; a.OW = 1; a.M = (int)T; a.K = Cin; a.relu = 0; a.out_mode = 0;
    a.xbytes = (int)(T * Cin * 4);
    a.wbytes = Cout * Cin * 4;
    a.rbytes = 0;
    a.bsx = T * Cin * 4;
    a.bsw = (long long)Cout * Cin * 4;
    a.bso = T * Cout * 4;
    a.epi_direct = P.direct_epilogue;
    const int bn = Cout <= 64 || (P.fp32_split && P.x3_narrow) ? 64 : BN;
    a.tiles_n = (int)ceil_div(Cout, bn);
    a.tiles_total = (int)(ceil_div(T, BM) * a.tiles_n);
    const int nk = (Cin + 31) / 32;
    a.ksplit = 1;
    a.ksteps = nk;
    const size_t lds_main = (nk == 1 ? 1 : 2) * ((size_t)BM * PITCH + (size_t)bn * PITCH);
    const size_t lds_epi = (size_t)(BM / 2) * (bn + 4) * 4;
    const size_t lds = lds_main > lds_epi ? lds_main : lds_epi;
    const dim3 grid((unsigned)a.tiles_total, 1, (unsigned)NB);
    // the wide GEMMs (Cout a multiple of 256) on the 256x256 LDS-DMA kernel
    // when the NB batch entries give it enough workgroups
    const long long t256 = ceil_div(T, G_BM) * (Cout / G_BN);
    const bool dma = !P.fp32_split && Cin % 32 == 0 && Cout % G_BN == 0 &&
                     (P.winograd_dma == 2 || (P.winograd_dma == 1 && t256 * NB >= P.winograd_dma_min_wgs));
    if (planes) {
        a.x = workspace;
        a.w = Up;
        a.xbytes = 0;
        a.wbytes = 0;
        a.bsx = T * Cin * 6;
        a.bsw = (long long)Cout * Cin * 6;
        a.tiles_n = (int)ceil_div(Cout, X6_BN);
        a.tiles_total = (int)(ceil_div(T, X6_BM) * a.tiles_n);
        hipLaunchKernelGGL(k_gemm_x6, dim3((unsigned)a.tiles_total, 1, (unsigned)NB), dim3(X6_THREADS), X6_LDS, s, a);
        gemm_kernel = MDX_CONV_KERNEL_X6DMA;
    } else if (dma) {
        a.tiles_n = Cout / G_BN;
        a.tiles_total = (int)t256;
        a.ksteps = Cin / 16;  // 16-float substeps
        hipLaunchKernelGGL((k_convg<float, float, 8, false>), dim3((unsigned)t256, 1, (unsigned)NB), dim3(G_THREADS),
                           G_LDS, s, a);
        gemm_kernel = MDX_CONV_KERNEL_DMA256;
    } else if (P.fp32_split) {
        launch_x3(a, bn, grid, s);
        gemm_kernel = bn == 64 ? MDX_CONV_KERNEL_X3_64 : MDX_CONV_KERNEL_X3_128;
    } else if (bn == 64) {
        if (P.pointwise && P.single_stage) {
            hipLaunchKernelGGL((k_conv_sb<float, float, 64>), grid, dim3(CONV_THREADS),
                               conv_lds(64, a.ksteps, true), s, a);
            gemm_kernel = MDX_CONV_KERNEL_SB64;
        } else if (P.pointwise) {
            hipLaunchKernelGGL((k_conv<float, float, 64, false, true>), grid, dim3(CONV_THREADS), lds, s, a);
            gemm_kernel = MDX_CONV_KERNEL_PW64;
        } else {
            hipLaunchKernelGGL((k_conv<float, float, 64>), grid, dim3(CONV_THREADS), lds, s, a);
            gemm_kernel = MDX_CONV_KERNEL_REG64;
        }
    } else {
        if (P.pointwise && P.single_stage) {
            hipLaunchKernelGGL((k_conv_sb<float, float, 128>), grid, dim3(CONV_THREADS),
                               conv_lds(128, a.ksteps, true), s, a);
            gemm_kernel = MDX_CONV_KERNEL_SB128;
        } else if (P.pointwise) {
            hipLaunchKernelGGL((k_conv<float, float, 128, false, true>), grid, dim3(CONV_THREADS), lds, s, a);
            gemm_kernel = MDX_CONV_KERNEL_PW128;
        } else {
            hipLaunchKernelGGL((k_conv<float, float, 128>), grid, dim3(CONV_THREADS), lds, s, a);
            gemm_kernel = MDX_CONV_KERNEL_REG128;
        }
    }
    mark(3);
    mark(4);
    {
        unsigned bd;
        const dim3 grid2 = tgrid(Cout, bd);
        if (m == 2)
            hipLaunchKernelGGL(k_wino_out<2>, grid2, dim3(bd), 0, s, Mx, N, H, W, Cout, TH, TW, bias, relu, out);
        else if (m == 4)
            hipLaunchKernelGGL(k_wino_out<4>, grid2, dim3(bd), 0, s, Mx, N, H, W, Cout, TH, TW, bias, relu, out);
        else
            hipLaunchKernelGGL(k_wino_out<6>, grid2, dim3(bd), 0, s, Mx, N, H, W, Cout, TH, TW, bias, relu, out);
    }
    mark(5);
    if (probe) probe->gemm_kernel = gemm_kernel;
    t_plan_kernel = MDX_CONV_KERNEL_WINOGRAD;
    t_plan_ksplit = 1;
    MDX_CHECK_LAUNCH("mdx_conv3x3_winograd");
    return MDX_OK;
}
