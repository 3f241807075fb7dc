// Non-GEMM kernels of the Mask/Keypoint R-CNN forward (gfx950).
//
//   k_preprocess     scale LUT + (x - mean)/std + zero pad to /32, NHWC
//                    (Predictor.__call__ M/model/predict.py:53-102 +
//                     GeneralizedRCNN.preprocess_image; scale_raw_frames fused)
//   k_maxpool        stem max_pool2d(3,2,1) and LastLevelMaxPool (k1,s2)
//   k_gn_stats/apply GroupNorm(32) of the FPN convs, fused with the top-down
//                    nearest x2 upsample + add (+ /2 for FUSE_TYPE avg)
//   k_rpn_topk       per (image, level): radix-select top-k objectness,
//                    bitonic sort, anchor decode (Box2BoxTransform), clip,
//                    nonempty                        (find_top_rpn_proposals)
//   k_nms_mask/scan  greedy NMS on score-sorted boxes: IoU bitmask + one-wave
//                    serial sweep                     (torchvision nms)
//   k_rpn_merge      batched_nms merge of levels, top post_nms_topk
//   k_roi_align      ROIPooler + ROIAlignV2 (level assignment, adaptive grid)
//   k_box_post       softmax, decode (10,10,5,5), clip, score filter, NMS,
//                    top-k, detector_postprocess nonempty
//   k_paste          mask sigmoid + paste_masks_in_image (grid_sample) >= 0.5
//   k_kp_deconv      ConvTranspose2d(k4, s2, p1) of the keypoint head
//   k_upsample2x     F.interpolate(x2, bilinear, align_corners=False)
//   k_heatmap_kp     heatmaps_to_keypoints (bicubic resize, argmax, score)
// Float arithmetic follows the reference's operation order with FMA
// contraction disabled.
#include <cfloat>
#include <cmath>

#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

constexpr int MAX_LEVELS = 8;

template <typename T>
__device__ __forceinline__ float ld(const T *p) {
    return (float)*p;
}
template <typename T>
__device__ __forceinline__ void st(T *p, float v) {
    *p = (T)v;
}

template <typename T>
__device__ __forceinline__ void ld8(const T *p, float *v) {
    if constexpr (sizeof(T) == 2) {
        const uint4 u = *reinterpret_cast<const uint4 *>(p);
        const T *e = reinterpret_cast<const T *>(&u);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)e[i];
    } else {
        const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
}
template <typename T>
__device__ __forceinline__ void st8(T *p, const float *v) {
    if constexpr (sizeof(T) == 2) {
        uint4 u;
        T *e = reinterpret_cast<T *>(&u);
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = (T)v[i];
        *reinterpret_cast<uint4 *>(p) = u;
    } else {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4 *>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

// ---------------------------------------------------------------------------
// preprocess
// ---------------------------------------------------------------------------
struct PrepArgs {
    uint8_t lut[256];
    float mean[4], stdv[4];
};

template <typename T>
__global__ __launch_bounds__(256) void k_preprocess(const uint8_t *__restrict__ fr, int B, int h, int w, int C, int Cp,
                                                    int Hp, int Wp, PrepArgs pa, T *__restrict__ out) {
    const int total = B * Hp * Wp;  // < 2^31 (checked on the host)
    for (int p = blockIdx.x * 256 + threadIdx.x; p < total; p += gridDim.x * 256) {
        const int b = p / (Hp * Wp);
        const int rem = p - b * Hp * Wp;
        const int y = rem / Wp, x = rem - y * Wp;
        T *o = out + (long long)p * Cp;
        if (y < h && x < w) {
            const float v = (float)pa.lut[fr[((long long)b * h + y) * w + x]];
            for (int c = 0; c < Cp; ++c) o[c] = c < C ? (T)((v - pa.mean[c]) / pa.stdv[c]) : (T)0.f;
        } else {
            for (int c = 0; c < Cp; ++c) o[c] = (T)0.f;
        }
    }
}

// Space-to-depth form of the same input for the stride-2 7x7 stem: S2D pixel
// (Y, X) of shape (Hp/2 + 1, Wp/2 + 1, 16) holds padded-image pixels
// (2Y - 1 + dy, 2X - 1 + dx) in channels (2 dy + dx) * 4 + c (c < C, rest 0);
// the stem becomes a 4x4 / stride-1 / pad-1 conv over 16 channels
// (K = 256 instead of 7*7*8 = 392 with 16-B contiguous channel runs).
// FOLD: the 2-channel form for a stem whose per-channel normalisation is
// folded into its weights -- per phase (value, inside): the scaled pixel
// (0 outside the image) and 1 / 0, 8 channels per s2d pixel instead of 16
template <typename T, bool FOLD = false>
__global__ __launch_bounds__(256) void k_preprocess_s2d(const uint8_t *__restrict__ fr, int B, int h, int w, int C,
                                                        int Hs, int Ws, PrepArgs pa, T *__restrict__ out) {
    const int total = B * Hs * Ws;
    for (int p = blockIdx.x * 256 + threadIdx.x; p < total; p += gridDim.x * 256) {
        const int b = p / (Hs * Ws);
        const int rem = p - b * Hs * Ws;
        const int Y = rem / Ws, X = rem - Y * Ws;
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int y = 2 * Y - 1 + (q >> 1), x = 2 * X - 1 + (q & 1);
            const bool in = y >= 0 && y < h && x >= 0 && x < w;
            const float pix = in ? (float)pa.lut[fr[((long long)b * h + y) * w + x]] : 0.f;
            if constexpr (FOLD) {
                v[q * 2] = pix;
                v[q * 2 + 1] = in ? 1.f : 0.f;
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) v[q * 4 + c] = (in && c < C) ? (pix - pa.mean[c]) / pa.stdv[c] : 0.f;
            }
        }
        T *o = out + (long long)p * (FOLD ? 8 : 16);
        st8(o, v);
        if constexpr (!FOLD) st8(o + 8, v + 8);
    }
}

// ---------------------------------------------------------------------------
// maxpool NHWC
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_maxpool(const T *__restrict__ x, int N, int H, int W, int C, int k, int s,
                                                 int p, int OH, int OW, T *__restrict__ out) {
    const int CV = C / 8;
    const int total = N * OH * OW * CV;  // < 2^31 (checked on the host)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        int r = i / CV;
        const int c0 = (i - r * CV) * 8;
        const int ox = r % OW;
        r /= OW;
        const int oy = r % OH;
        const int n = r / OH;
        float m[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
        for (int ky = 0; ky < k; ++ky) {
            const int iy = oy * s - p + ky;
            if (iy < 0 || iy >= H) continue;
            for (int kx = 0; kx < k; ++kx) {
                const int ix = ox * s - p + kx;
                if (ix < 0 || ix >= W) continue;
                float v[8];
                ld8(x + (((long long)n * H + iy) * W + ix) * C + c0, v);
#pragma unroll
                for (int q = 0; q < 8; ++q) m[q] = v[q] > m[q] ? v[q] : m[q];
            }
        }
        st8(out + (((long long)n * OH + oy) * OW + ox) * C + c0, m);
    }
}

// ---------------------------------------------------------------------------
// dtype conversion (f32 <-> f16, round to nearest even), 8 values per lane
// ---------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void k_convert(const TI *__restrict__ x, long long n8, TO *__restrict__ y) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
        float v[8];
        ld8(x + i * 8, v);
        st8(y + i * 8, v);
    }
}

// ---------------------------------------------------------------------------
// GroupNorm
// ---------------------------------------------------------------------------
__device__ __forceinline__ float block_sum(float v, float *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float s = 0.f;
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

// GroupNorm statistics in two kernels: (1) every block streams a contiguous
// chunk of pixels (full channel rows, coalesced) and writes a Welford partial
// (count, mean, M2) per group; (2) one lane per (image, group) merges the
// partials with Chan's formula.  Lane -> 8-channel octet mapping needs C/G % 8
// == 0 (the FPN's 256/32).
constexpr int GN_CHUNK_PIX = 64;

template <typename T>
__global__ __launch_bounds__(256) void k_gn_partial(const T *__restrict__ x, int HW, int C, int G,
                                                    float *__restrict__ part) {
    __shared__ float s_n[256], s_m[256], s_q[256];
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int nchunks = gridDim.x;
    const int CV = C / 8;               // octets per pixel (<= 256)
    const int rows = 256 / CV;          // pixels processed in parallel
    const int cv = threadIdx.x % CV, pr = threadIdx.x / CV;
    const int p0 = chunk * GN_CHUNK_PIX;
    // shifted sums (shift = the lane's first value) -> exact-enough per-lane
    // (count, mean, M2) for <= GN_CHUNK_PIX*8 values
    float cnt = 0.f, mean = 0.f, m2 = 0.f;
    if (pr < rows && p0 + pr < HW) {
        float sh = 0.f, S = 0.f, Q = 0.f;
        bool first = true;
        for (int p = p0 + pr; p < p0 + GN_CHUNK_PIX && p < HW; p += rows) {
            float v[8];
            ld8(x + ((long long)n * HW + p) * C + cv * 8, v);
            if (first) {
                sh = v[0];
                first = false;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float d = v[k] - sh;
                S += d;
                Q += d * d;
            }
            cnt += 8.f;
        }
        mean = sh + S / cnt;
        m2 = fmaxf(Q - S * (S / cnt), 0.f);
    }
    s_n[threadIdx.x] = cnt;
    s_m[threadIdx.x] = mean;
    s_q[threadIdx.x] = m2;
    __syncthreads();
    // merge the lanes of one group: octets g*cpg/8 .. over all pixel rows
    const int opg = (C / G) / 8;  // octets per group
    if (threadIdx.x < G) {
        const int g = threadIdx.x;
        float N = 0.f, M = 0.f, Q = 0.f;
        for (int r = 0; r < rows; ++r)
            for (int o = 0; o < opg; ++o) {
                const int t = r * CV + g * opg + o;
                const float nb = s_n[t];
                if (nb == 0.f) continue;
                const float tot = N + nb;
                const float d = s_m[t] - M;
                M += d * (nb / tot);
                Q += s_q[t] + d * d * (N * nb / tot);
                N = tot;
            }
        float *pp = part + (((long long)n * G + g) * nchunks + chunk) * 3;
        pp[0] = N;
        pp[1] = M;
        pp[2] = Q;
    }
}

// one wave per (image, group): lanes merge strided chunk partials, then a
// butterfly of Chan merges (fp64)
__global__ __launch_bounds__(256) void k_gn_final(const float *__restrict__ part, int NG, int nchunks, float eps,
                                                  float *__restrict__ stats) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= NG) return;
    const float *pp = part + (long long)i * nchunks * 3;
    double N = 0.0, M = 0.0, Q = 0.0;
    for (int c = lane; c < nchunks; c += 64) {
        const double nb = pp[3 * c];
        if (nb == 0.0) continue;
        const double tot = N + nb;
        const double d = (double)pp[3 * c + 1] - M;
        M += d * (nb / tot);
        Q += (double)pp[3 * c + 2] + d * d * (N * nb / tot);
        N = tot;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double nb = __shfl_xor(N, off), mb = __shfl_xor(M, off), qb = __shfl_xor(Q, off);
        const double tot = N + nb;
        if (tot > 0.0) {
            const double d = mb - M;
            M += d * (nb / tot);
            Q += qb + d * d * (N * nb / tot);
            N = tot;
        }
    }
    if (lane == 0) {
        const float var = (float)(Q / N);
        stats[2 * i] = (float)M;
        stats[2 * i + 1] = 1.0f / sqrtf(var + eps);
    }
}

// y = (x - mean) * rstd * gamma + beta; optionally fused: y = (y + up(prev)) [/ 2]
// 8 consecutive channels per lane (C % 8 == 0 and C/G % 8 == 0 required)
template <typename T>
__global__ __launch_bounds__(256) void k_gn_apply(const T *__restrict__ x, int N, int H, int W, int C, int G,
                                                  const float *__restrict__ stats, const float *__restrict__ gamma,
                                                  const float *__restrict__ beta, const T *__restrict__ up, int fuse,
                                                  T *__restrict__ out) {
    const int CV = C / 8;
    const int total = N * H * W * CV;  // < 2^31 (checked on the host)
    const int cpg = C / G;
    const int HW = H * W;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        const int pixi = i / CV;
        const int c0 = (i - pixi * CV) * 8;
        const long long pix = pixi;
        const int n = pixi / HW;
        const int g = c0 / cpg;
        const float mean = stats[2 * (n * G + g)], rstd = stats[2 * (n * G + g) + 1];
        float v[8];
        ld8(x + pix * C + c0, v);
        float u[8];
        if (fuse) {
            const int rem = pixi - n * HW;
            const int yy = rem / W, xx = rem - yy * W;
            const int UH = H / 2, UW = W / 2;
            ld8(up + (((long long)n * UH + (yy >> 1)) * UW + (xx >> 1)) * C + c0, u);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float y = (v[k] - mean) * rstd * gamma[c0 + k] + beta[c0 + k];
            if (fuse) {
                y = y + u[k];
                if (fuse == 2) y = y / 2.0f;
            }
            v[k] = y;
        }
        st8(out + pix * C + c0, v);
    }
}

// ---------------------------------------------------------------------------
// box helpers (Box2BoxTransform.apply_deltas, Boxes.clip / nonempty)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void apply_delta(const float *box, float dxr, float dyr, float dwr, float dhr,
                                            const float *wts, float clampv, float *o) {
    const float widths = box[2] - box[0];
    const float heights = box[3] - box[1];
    const float ctr_x = box[0] + 0.5f * widths;
    const float ctr_y = box[1] + 0.5f * heights;
    const float dx = dxr / wts[0], dy = dyr / wts[1];
    float dw = dwr / wts[2], dh = dhr / wts[3];
    dw = dw > clampv ? clampv : dw;
    dh = dh > clampv ? clampv : dh;
    const float pcx = dx * widths + ctr_x;
    const float pcy = dy * heights + ctr_y;
    const float pw = expf(dw) * widths;
    const float ph = expf(dh) * heights;
    o[0] = pcx - 0.5f * pw;
    o[1] = pcy - 0.5f * ph;
    o[2] = pcx + 0.5f * pw;
    o[3] = pcy + 0.5f * ph;
}

__device__ __forceinline__ float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ unsigned fkey(float v) {
    const unsigned u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// bitonic sort of n (power of two, <= blockDim*k) (key, val) pairs in LDS,
// descending by key then ascending by val
__device__ void bitonic_desc(unsigned *key, unsigned *val, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = ((lo & size) == 0);  // segment direction
                const unsigned ka = key[lo], kb = key[hi], va = val[lo], vb = val[hi];
                // "a before b" in final (descending key, ascending val) order
                const bool a_first = ka > kb || (ka == kb && va < vb);
                const bool swap = up ? !a_first : a_first;
                if (swap) {
                    key[lo] = kb; key[hi] = ka;
                    val[lo] = vb; val[hi] = va;
                }
            }
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// RPN: top-k + decode per (image, level)
// ---------------------------------------------------------------------------
struct RpnLevels {
    const float *head[MAX_LEVELS];  // (B, H, W, A*5) f32: [obj(A), deltas(A*4)]
    int H[MAX_LEVELS], W[MAX_LEVELS], stride[MAX_LEVELS];
    float cell[MAX_LEVELS][8][4];  // up to 8 aspect ratios
    float wts[4];                  // RPN.BBOX_REG_WEIGHTS
    int L, A, B, pre_topk;
    float offset, img_h, img_w, min_size, clampv;
};

// decode the k score-sorted anchors s_val[0..k) of segment seg (image b,
// level l) into boxes (apply_deltas, clip, nonempty), scores, valid flags
__device__ void rpn_decode(const RpnLevels &rl, int seg, int k, const unsigned *s_val, float *__restrict__ ws_boxes,
                           float *__restrict__ ws_scores, int *__restrict__ ws_valid, int *__restrict__ ws_k) {
    const int b = seg / rl.L, l = seg - b * rl.L;
    const int A = rl.A, CH = A * 5;
    const int HW = rl.H[l] * rl.W[l];
    const float *hd = rl.head[l] + (long long)b * HW * CH;
    const int st = rl.stride[l];
    float *ob = ws_boxes + (long long)seg * rl.pre_topk * 4;
    float *os = ws_scores + (long long)seg * rl.pre_topk;
    int *ov = ws_valid + (long long)seg * rl.pre_topk;
    const float wts[4] = {rl.wts[0], rl.wts[1], rl.wts[2], rl.wts[3]};
    for (int r = threadIdx.x; r < k; r += blockDim.x) {
        const int i = (int)s_val[r];
        const int pix = i / A, a = i - pix * A;
        const int y = pix / rl.W[l], x = pix - y * rl.W[l];
        const float sx = rl.offset * (float)st + (float)(x * st);
        const float sy = rl.offset * (float)st + (float)(y * st);
        const float anc[4] = {sx + rl.cell[l][a][0], sy + rl.cell[l][a][1], sx + rl.cell[l][a][2],
                              sy + rl.cell[l][a][3]};
        const float *dl = hd + (long long)pix * CH + A + a * 4;
        float bx[4];
        apply_delta(anc, dl[0], dl[1], dl[2], dl[3], wts, rl.clampv, bx);
        const float score = hd[(long long)pix * CH + a];
        bool fin = isfinite(bx[0]) && isfinite(bx[1]) && isfinite(bx[2]) && isfinite(bx[3]) && isfinite(score);
        bx[0] = clampf(bx[0], 0.f, rl.img_w);
        bx[1] = clampf(bx[1], 0.f, rl.img_h);
        bx[2] = clampf(bx[2], 0.f, rl.img_w);
        bx[3] = clampf(bx[3], 0.f, rl.img_h);
        const bool ne = (bx[2] - bx[0]) > rl.min_size && (bx[3] - bx[1]) > rl.min_size;
        ob[4 * r + 0] = bx[0];
        ob[4 * r + 1] = bx[1];
        ob[4 * r + 2] = bx[2];
        ob[4 * r + 3] = bx[3];
        os[r] = score;
        ov[r] = (fin && ne) ? 1 : 0;
    }
    if (threadIdx.x == 0) ws_k[seg] = k;
}

// Wave 0 of the block: the radix digit of a descending select.  d = the
// largest d >= 1 with S(d) = sum_{d' >= d} hist[d'] >= kk, else 0; returns
// through *s_d, *s_above (= S(d + 1)) and *s_cnt (= hist[d]).
__device__ void pick_digit(const unsigned *hist, unsigned kk, unsigned *s_d, unsigned *s_above, unsigned *s_cnt) {
    const int lane = threadIdx.x & 63;
    unsigned h[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) h[q] = hist[4 * lane + q];
    const unsigned lsum = h[0] + h[1] + h[2] + h[3];
    unsigned suf = lsum;
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned t = __shfl_down(suf, off);
        if (lane + off < 64) suf += t;
    }
    unsigned S[4];
    S[3] = suf - lsum + h[3];
    S[2] = S[3] + h[2];
    S[1] = S[2] + h[1];
    S[0] = S[1] + h[0];
    int qbest = -1;
#pragma unroll
    for (int q = 3; q >= 0; --q)
        if (qbest < 0 && 4 * lane + q >= 1 && S[q] >= kk) qbest = q;
    const unsigned long long any = __ballot(qbest >= 0);
    const int lb = any ? 63 - __builtin_clzll(any) : 0;
    const int qb = any ? __shfl(qbest, lb) : 0;
    const int Sd = __shfl((int)(qb == 3 ? S[3] : qb == 2 ? S[2] : qb == 1 ? S[1] : S[0]), lb);
    const int hd = __shfl((int)(qb == 3 ? h[3] : qb == 2 ? h[2] : qb == 1 ? h[1] : h[0]), lb);
    if (lane == 0) {
        *s_d = (unsigned)(4 * lb + qb);
        *s_above = (unsigned)Sd - (unsigned)hd;
        *s_cnt = (unsigned)hd;
    }
}

// Exact top-kk of the block's register-held unique 64-bit keys (descending):
// returns (mask, prefix) such that the selected keys are exactly those with
// (key & mask) >= prefix -- 8-bit radix passes from the top, stopping early
// once a digit's whole bin is taken.
template <int KPT, int NT>
__device__ void select_top64(const unsigned long long (&kr)[KPT], const bool (&ok)[KPT], unsigned kk, unsigned *hist,
                             unsigned *s_sel, unsigned long long &mask_out, unsigned long long &prefix_out) {
    unsigned long long prefix = 0, mask = 0;
    const int wid = threadIdx.x >> 6;
    for (int shift = 56; shift >= 0 && kk > 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j)
            if (ok[j] && (kr[j] & mask) == prefix) atomicAdd(&hist[(unsigned)(kr[j] >> shift) & 255u], 1u);
        __syncthreads();
        if (wid == 0) pick_digit(hist, kk, &s_sel[0], &s_sel[1], &s_sel[2]);
        __syncthreads();
        const unsigned d = s_sel[0], above = s_sel[1], cnt = s_sel[2];
        __syncthreads();
        prefix |= (unsigned long long)d << shift;
        mask |= 255ull << shift;
        kk -= above;
        if (cnt == kk) break;  // the whole bin is taken
    }
    mask_out = mask;
    prefix_out = prefix;
}

constexpr int TOPK_THREADS = 1024, TOPK_MAX = 1024;

// One workgroup per (image, level): radix select of the k-th largest key over
// the head tensor (every pass re-reads it), the ties taken in index order,
// bitonic sort, decode.  The default path splits the segment over RPN_SLICES
// workgroups (k_rpn_part / k_rpn_merge_topk below); this one serves
// mdx_policy.rpn_sliced = 0 and segments above RPN_SLICES * PART_KPT *
// TOPK_THREADS anchors.
__global__ __launch_bounds__(TOPK_THREADS) void k_rpn_topk(RpnLevels rl, float *__restrict__ ws_boxes,
                                                           float *__restrict__ ws_scores, int *__restrict__ ws_valid,
                                                           int *__restrict__ ws_k) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_key[TOPK_MAX], s_val[TOPK_MAX];
    __shared__ unsigned s_sel[3], s_cnt_gt, s_cnt_eq;
    __shared__ unsigned wcnt[TOPK_THREADS / 64];
    const int seg = blockIdx.x;  // b * L + l
    const int b = seg / rl.L, l = seg - b * rl.L;
    const int A = rl.A, CH = A * 5;
    const int HW = rl.H[l] * rl.W[l];
    const int n = HW * A;
    const int k = n < rl.pre_topk ? n : rl.pre_topk;
    const float *hd = rl.head[l] + (long long)b * HW * CH;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    auto keyat = [&](int i) {
        const int pix = i / A, a = i - pix * A;
        return fkey(hd[(long long)pix * CH + a]);
    };
    // radix select of the k-th largest key
    unsigned prefix = 0, mask = 0, kk = (unsigned)k, eq_total = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += TOPK_THREADS) hist[i] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += TOPK_THREADS) {
            const unsigned key = keyat(i);
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
        }
        __syncthreads();
        if (wid == 0) pick_digit(hist, kk, &s_sel[0], &s_sel[1], &s_sel[2]);
        __syncthreads();
        prefix |= s_sel[0] << shift;
        kk -= s_sel[1];
        eq_total = s_sel[2];
        mask |= 255u << shift;
        __syncthreads();
    }
    const unsigned T = prefix;  // k-th largest key; take kk of the eq_total ties (lowest indices)
    if (threadIdx.x == 0) {
        s_cnt_gt = 0;
        s_cnt_eq = 0;
    }
    for (int i = threadIdx.x; i < TOPK_MAX; i += TOPK_THREADS) {
        s_key[i] = 0;
        s_val[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (eq_total == kk) {
        // every key == T is taken: one unordered pass, the sort orders it
        for (int i = threadIdx.x; i < n; i += TOPK_THREADS) {
            const unsigned key = keyat(i);
            if (key >= T) {
                const unsigned pos = atomicAdd(&s_cnt_gt, 1u);
                s_key[pos] = key;
                s_val[pos] = (unsigned)i;
            }
        }
    } else {
        // keys > T (any order); keys == T in index order (ordered scan)
        const unsigned n_gt = (unsigned)k - kk;
        for (int base = 0; base < n; base += TOPK_THREADS) {
            const int i = base + threadIdx.x;
            const unsigned key = i < n ? keyat(i) : 0u;
            const bool gt = i < n && key > T, eq = i < n && key == T;
            if (gt) {
                const unsigned pos = atomicAdd(&s_cnt_gt, 1u);
                s_key[pos] = key;
                s_val[pos] = (unsigned)i;
            }
            const unsigned long long bal = __ballot(eq);
            if (lane == 0) wcnt[wid] = (unsigned)__popcll(bal);
            __syncthreads();
            if (eq) {
                unsigned before = s_cnt_eq;
                for (int w2 = 0; w2 < wid; ++w2) before += wcnt[w2];
                before += (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
                if (before < kk) {
                    s_key[n_gt + before] = key;
                    s_val[n_gt + before] = (unsigned)i;
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned tot = 0;
                for (int w2 = 0; w2 < TOPK_THREADS / 64; ++w2) tot += wcnt[w2];
                s_cnt_eq += tot;
            }
            __syncthreads();
        }
    }
    bitonic_desc(s_key, s_val, TOPK_MAX);
    rpn_decode(rl, seg, k, s_val, ws_boxes, ws_scores, ws_valid, ws_k);
}

// ---------------------------------------------------------------------------
// RPN top-k over several workgroups per (image, level): the anchors are split
// into RPN_SLICES slices, each workgroup keeps its slice's top-k by a 64-bit
// key (score key << 32 | ~index: unique, and larger = earlier in Detectron2's
// topk order, ties to the lower index), then one workgroup per segment merges
// the <= RPN_SLICES * k candidates, sorts and decodes them.
// ---------------------------------------------------------------------------
constexpr int RPN_SLICES = 8, PART_KPT = 6, MERGE_KPT = 8;

__device__ __forceinline__ unsigned long long rpn_ckey(unsigned key, int i) {
    return ((unsigned long long)key << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)i);
}

__global__ __launch_bounds__(TOPK_THREADS) void k_rpn_part(RpnLevels rl, unsigned long long *__restrict__ cand,
                                                           int *__restrict__ ccount) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_sel[3], s_pos;
    const int sl = blockIdx.x, seg = blockIdx.y;
    const int b = seg / rl.L, l = seg - b * rl.L;
    const int A = rl.A, CH = A * 5;
    const int HW = rl.H[l] * rl.W[l];
    const int n = HW * A;
    const int k = n < rl.pre_topk ? n : rl.pre_topk;
    const int len = (n + RPN_SLICES - 1) / RPN_SLICES;
    const int i0 = sl * len, i1 = min(n, i0 + len);
    const int m = i1 > i0 ? i1 - i0 : 0;
    const unsigned kk = (unsigned)min(k, m);
    const float *hd = rl.head[l] + (long long)b * HW * CH;
    unsigned long long kr[PART_KPT];
    bool ok[PART_KPT];
#pragma unroll
    for (int j = 0; j < PART_KPT; ++j) {
        const int i = i0 + j * TOPK_THREADS + threadIdx.x;
        ok[j] = i < i1;
        const int pix = i / A, a = i - pix * A;
        kr[j] = ok[j] ? rpn_ckey(fkey(hd[(long long)pix * CH + a]), i) : 0ull;
    }
    unsigned long long mask, prefix;
    select_top64<PART_KPT, TOPK_THREADS>(kr, ok, kk, hist, s_sel, mask, prefix);
    if (threadIdx.x == 0) s_pos = 0;
    __syncthreads();
    unsigned long long *out = cand + ((long long)seg * RPN_SLICES + sl) * rl.pre_topk;
#pragma unroll
    for (int j = 0; j < PART_KPT; ++j)
        if (kk > 0 && ok[j] && (kr[j] & mask) >= prefix) out[atomicAdd(&s_pos, 1u)] = kr[j];
    if (threadIdx.x == 0) ccount[seg * RPN_SLICES + sl] = (int)kk;
}

__global__ __launch_bounds__(TOPK_THREADS) void k_rpn_merge_topk(RpnLevels rl,
                                                                 const unsigned long long *__restrict__ cand,
                                                                 const int *__restrict__ ccount,
                                                                 float *__restrict__ ws_boxes,
                                                                 float *__restrict__ ws_scores,
                                                                 int *__restrict__ ws_valid, int *__restrict__ ws_k) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_key[TOPK_MAX], s_val[TOPK_MAX];
    __shared__ unsigned s_sel[3], s_pos;
    const int seg = blockIdx.x;
    const int l = seg % rl.L;
    const int n = rl.H[l] * rl.W[l] * rl.A;
    const int k = n < rl.pre_topk ? n : rl.pre_topk;
    const int P = rl.pre_topk;
    unsigned long long kr[MERGE_KPT];
    bool ok[MERGE_KPT];
#pragma unroll
    for (int j = 0; j < MERGE_KPT; ++j) {
        const int c = j * TOPK_THREADS + threadIdx.x;  // candidate c: slice c / P, position c % P
        const int sl = c / P, pos = c - sl * P;
        ok[j] = sl < RPN_SLICES && pos < ccount[seg * RPN_SLICES + (sl < RPN_SLICES ? sl : 0)];
        kr[j] = ok[j] ? cand[(long long)seg * RPN_SLICES * P + c] : 0ull;
    }
    unsigned long long mask, prefix;
    select_top64<MERGE_KPT, TOPK_THREADS>(kr, ok, (unsigned)k, hist, s_sel, mask, prefix);
    for (int i = threadIdx.x; i < TOPK_MAX; i += TOPK_THREADS) {
        s_key[i] = 0;
        s_val[i] = 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) s_pos = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MERGE_KPT; ++j)
        if (ok[j] && (kr[j] & mask) >= prefix) {
            const unsigned p = atomicAdd(&s_pos, 1u);
            s_key[p] = (unsigned)(kr[j] >> 32);
            s_val[p] = 0xFFFFFFFFu - (unsigned)kr[j];
        }
    bitonic_desc(s_key, s_val, TOPK_MAX);
    rpn_decode(rl, seg, k, s_val, ws_boxes, ws_scores, ws_valid, ws_k);
}

// ---------------------------------------------------------------------------
// NMS over score-sorted segments
// ---------------------------------------------------------------------------
// mask[seg][i][w]: bit j%64 of word w set when IoU(i, j) > thresh, j > i.
// Block = (word w, 256 rows i, segment): the word's 64 j-boxes are staged in
// LDS once and read as broadcasts; each lane keeps its i-box in registers.
__global__ __launch_bounds__(256) void k_nms_mask(const float *__restrict__ boxes, const int *__restrict__ kseg,
                                                  int cap, int words, float thresh,
                                                  unsigned long long *__restrict__ mask) {
    __shared__ float4 jb[64];
    const int seg = blockIdx.z, w = blockIdx.x;
    const int k = min(max(kseg[seg], 0), cap);  // (counts never address past the segment)
    const int j0 = w * 64;
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (j0 >= k || blockIdx.y * 256 >= k) return;  // uniform per block
    const float *bx = boxes + (long long)seg * cap * 4;
    if (threadIdx.x < 64) {
        const int j = j0 + threadIdx.x;
        jb[threadIdx.x] = j < k ? *reinterpret_cast<const float4 *>(bx + 4 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    if (i >= k) return;
    const float4 ib = *reinterpret_cast<const float4 *>(bx + 4 * i);
    const float ix1 = ib.x, iy1 = ib.y, ix2 = ib.z, iy2 = ib.w;
    const float iarea = (ix2 - ix1) * (iy2 - iy1);
    unsigned long long bits = 0ull;
    for (int jj = 0; jj < 64; ++jj) {
        const int j = j0 + jj;
        if (j <= i || j >= k) continue;
        const float4 q = jb[jj];
        const float jx1 = q.x, jy1 = q.y, jx2 = q.z, jy2 = q.w;
        const float xx1 = fmaxf(ix1, jx1), yy1 = fmaxf(iy1, jy1);
        const float xx2 = fminf(ix2, jx2), yy2 = fminf(iy2, jy2);
        const float w_ = fmaxf(0.f, xx2 - xx1), h_ = fmaxf(0.f, yy2 - yy1);
        const float inter = w_ * h_;
        const float jarea = (jx2 - jx1) * (jy2 - jy1);
        const float ovr = inter / (iarea + jarea - inter);
        if (ovr > thresh) bits |= 1ull << jj;
    }
    mask[((long long)seg * cap + i) * words + w] = bits;
}

// One workgroup per segment: the segment's whole IoU bitmask (k rows x words
// 64-bit words, <= 128 KB) is first staged into LDS by all 256 threads with
// every load in flight at once, then wave 0 sweeps it in score order from LDS;
// invalid boxes never keep nor suppress (Detectron2 removes them before
// NMS).  Per 64-row chunk the sweep is scalar over the rows still standing:
// the chunk's removed word and each kept row's word for the chunk are
// v_readlane'd, and the kept rows' full masks are OR-ed into `removed`
// afterwards (lane w holds word w).
constexpr int NMS_MAXW = 16;  // pre_topk <= 1024
constexpr int NMS_THREADS = 256;
__global__ __launch_bounds__(NMS_THREADS) void k_nms_scan(const int *__restrict__ valid, const int *__restrict__ kseg,
                                                          int cap, int words,
                                                          const unsigned long long *__restrict__ mask,
                                                          int *__restrict__ keep) {
    extern __shared__ unsigned long long rows[];  // [k][words]
    __shared__ unsigned long long vbits[NMS_MAXW];
    const int seg = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int k = min(max(kseg[seg], 0), cap);
    const int *vl = valid + (long long)seg * cap;
    const unsigned long long *mk = mask + (long long)seg * cap * words;
    int *kp = keep + (long long)seg * cap;
    const int total = k * words;
    if ((((long long)cap * words) & 1) || (reinterpret_cast<uintptr_t>(mask) & 15)) {
        for (int t = threadIdx.x; t < total; t += NMS_THREADS) rows[t] = mk[t];  // unaligned rows: 8-B pieces
    } else {
        // 16-B pieces, 8 loads in flight per thread before their LDS stores
        // (a load -> store loop waits out the memory latency every iteration)
        const int npc = total >> 1;
        const uint4 *src = reinterpret_cast<const uint4 *>(mk);
        uint4 *dst = reinterpret_cast<uint4 *>(rows);
        for (int t0 = 0; t0 < npc; t0 += 8 * NMS_THREADS) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + u * NMS_THREADS + threadIdx.x;
                v[u] = t < npc ? src[t] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + u * NMS_THREADS + threadIdx.x;
                if (t < npc) dst[t] = v[u];
            }
        }
        if ((total & 1) && threadIdx.x == 0) rows[total - 1] = mk[total - 1];
    }
    // valid flags as bits, one 64-row word per wave iteration
    for (int c = wid; c * 64 < k; c += NMS_THREADS / 64) {
        const int i = c * 64 + lane;
        const unsigned long long b = __ballot(i < k && vl[i] != 0);
        if (lane == 0) vbits[c] = b;
    }
    __syncthreads();
    if (wid == 0) {
        unsigned long long removed = 0ull;  // lane w < words holds word w
        for (int i0 = 0; i0 < k; i0 += 64) {
            const int cwi = i0 >> 6;
            const int nr = k - i0 < 64 ? k - i0 : 64;
            const unsigned long long own = lane < nr ? rows[(i0 + lane) * words + cwi] : 0ull;
            const unsigned own_lo = (unsigned)own, own_hi = (unsigned)(own >> 32);
            const unsigned long long vmask = vbits[cwi];
            unsigned long long cw =
                ((unsigned long long)__builtin_amdgcn_readlane((unsigned)(removed >> 32), cwi) << 32) |
                (unsigned)__builtin_amdgcn_readlane((unsigned)removed, cwi);
            unsigned long long kept = 0ull;
            const unsigned long long live = nr == 64 ? ~0ull : ((1ull << nr) - 1ull);
            unsigned long long cand = ~cw & vmask & live;
            while (cand) {
                const int r = __builtin_ctzll(cand);
                kept |= 1ull << r;
                cw |= ((unsigned long long)__builtin_amdgcn_readlane(own_hi, r) << 32) |
                      (unsigned)__builtin_amdgcn_readlane(own_lo, r);
                cand = ~cw & vmask & live & ~((2ull << r) - 1ull);
            }
            if (lane < words) {
                unsigned long long kk = kept;
                while (kk) {
                    const int r = __builtin_ctzll(kk);
                    kk &= kk - 1;
                    removed |= rows[(i0 + r) * words + lane];
                }
            }
            if (lane < nr) kp[i0 + lane] = (int)((kept >> lane) & 1ull);
        }
    }
    for (int i = k + threadIdx.x; i < cap; i += NMS_THREADS) kp[i] = 0;
}

// ---------------------------------------------------------------------------
// merge levels: batched_nms result sorted by score, first post_topk
// ---------------------------------------------------------------------------
constexpr int MERGE_MAX = 8192;

__global__ __launch_bounds__(1024) void k_rpn_merge(const float *__restrict__ ws_boxes,
                                                    const float *__restrict__ ws_scores,
                                                    const int *__restrict__ keep, const int *__restrict__ kseg,
                                                    int L, int cap, int post_topk, float *__restrict__ out_boxes,
                                                    float *__restrict__ out_scores, int *__restrict__ out_count) {
    extern __shared__ unsigned sm[];
    unsigned *key = sm, *val = sm + MERGE_MAX;
    __shared__ unsigned s_n;
    const int b = blockIdx.x;
    if (threadIdx.x == 0) s_n = 0;
    for (int i = threadIdx.x; i < MERGE_MAX; i += blockDim.x) {
        key[i] = 0;
        val[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    for (int l = 0; l < L; ++l) {
        const int seg = b * L + l;
        const int k = min(max(kseg[seg], 0), cap);
        for (int r = threadIdx.x; r < k; r += blockDim.x) {
            if (keep[(long long)seg * cap + r]) {
                const unsigned pos = atomicAdd(&s_n, 1u);
                key[pos] = fkey(ws_scores[(long long)seg * cap + r]);
                val[pos] = (unsigned)(l * cap + r);  // level-major tie order
            }
        }
    }
    __syncthreads();
    const int n = (int)s_n;
    int sz = 1;
    while (sz < n) sz <<= 1;
    bitonic_desc(key, val, sz < 2 ? 2 : sz);
    const int m = n < post_topk ? n : post_topk;
    for (int r = threadIdx.x; r < post_topk; r += blockDim.x) {
        float *ob = out_boxes + ((long long)b * post_topk + r) * 4;
        if (r < m) {
            const unsigned v = val[r];
            const int l = (int)(v / cap), rr = (int)(v - (unsigned)l * cap);
            const long long src = (long long)(b * L + l) * cap + rr;
            ob[0] = ws_boxes[src * 4];
            ob[1] = ws_boxes[src * 4 + 1];
            ob[2] = ws_boxes[src * 4 + 2];
            ob[3] = ws_boxes[src * 4 + 3];
            out_scores[(long long)b * post_topk + r] = ws_scores[src];
        } else {
            ob[0] = ob[1] = ob[2] = ob[3] = 0.f;
            out_scores[(long long)b * post_topk + r] = -INFINITY;
        }
    }
    if (threadIdx.x == 0) out_count[b] = m;
}

// ---------------------------------------------------------------------------
// ROIAlign (ROIPooler, ROIAlignV2)
// ---------------------------------------------------------------------------
struct RoiLevels {
    const void *feat[MAX_LEVELS];
    int H[MAX_LEVELS], W[MAX_LEVELS];
    float scale[MAX_LEVELS];
    int L, min_level, C, P, sampling, aligned, per_image;
    float canonical_size, canonical_level;
    int xcd_remap;  // 1: XCD-contiguous ROI ranges (default); 0: ROIs in dispatch order across XCDs
    const int *order;  // optional ROI permutation (k_roi_order), applied after the XCD remap
    int planes;        // fp32 only: write each ROI row as bf16 planes (mdx_split_x6 layout) for mdx_gemm_x6
};

// the ROI a workgroup pools: XCD-contiguous ranges of the dispatch order (the
// ROIs of one image share its maps), then the optional locality permutation
__device__ __forceinline__ int roi_of_block(const RoiLevels &rl) {
    int r = blockIdx.x;
    if (rl.xcd_remap) {
        const int Lb = blockIdx.x, nwg = gridDim.x;
        const int q = nwg / 8, rr = nwg % 8, xcd = Lb % 8;
        r = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + Lb / 8;
    }
    return rl.order ? rl.order[r] : r;
}

template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
    static constexpr int N = 4;
};
template <>
struct Vec16<_Float16> {
    static constexpr int N = 8;
};

template <typename T>
__device__ __forceinline__ void ld16(const T *p, float *v) {
    const uint4 u = *reinterpret_cast<const uint4 *>(p);
    const T *e = reinterpret_cast<const T *>(&u);
#pragma unroll
    for (int i = 0; i < Vec16<T>::N; ++i) v[i] = (float)e[i];
}
template <typename T>
__device__ __forceinline__ void st16(T *p, const float *v) {
    uint4 u;
    T *e = reinterpret_cast<T *>(&u);
#pragma unroll
    for (int i = 0; i < Vec16<T>::N; ++i) e[i] = (T)v[i];
    *reinterpret_cast<uint4 *>(p) = u;
}
// 4 fp32 values at element e (e % 4 == 0) of a row in the bf16 plane layout
// (mdx_split_x6: per 16 values 96 B = hi | mid | lo, x = hi + mid + lo exactly)
typedef __bf16 rbf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4_planes(char *row, long long e, const float *v) {
    rbf16x4 h, m, l;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const __bf16 hb = (__bf16)v[i];
        const float r1 = v[i] - (float)hb;
        const __bf16 mb = (__bf16)r1;
        h[i] = hb;
        m[i] = mb;
        l[i] = (__bf16)(r1 - (float)mb);
    }
    char *p = row + (e >> 4) * 96 + ((e >> 2) & 3) * 8;
    *reinterpret_cast<rbf16x4 *>(p) = h;
    *reinterpret_cast<rbf16x4 *>(p + 32) = m;
    *reinterpret_cast<rbf16x4 *>(p + 64) = l;
}

// ROIAlign sample geometry of one ROI (ROIAlignV2 / ROIPooler semantics)
struct RoiGeom {
    const void *feat;  // level map of this ROI's image
    int li, H, W, gh, gw;
    float rsw, rsh, bh, bw, count;
};

__device__ __forceinline__ RoiGeom roi_geom(const RoiLevels &rl, const float *rois, int r, int b, size_t esize) {
    const float x1 = rois[4 * r], y1 = rois[4 * r + 1], x2 = rois[4 * r + 2], y2 = rois[4 * r + 3];
    // level assignment (assign_boxes_to_levels)
    const float area = (x2 - x1) * (y2 - y1);
    const float bs = sqrtf(area);
    float lv = floorf(rl.canonical_level + log2f(bs / rl.canonical_size + 1e-8f));
    const float maxl = (float)(rl.min_level + rl.L - 1);
    // (a non-finite box maps to the lowest level, never to an index outside the table)
    lv = !(lv >= (float)rl.min_level) ? (float)rl.min_level : (lv > maxl ? maxl : lv);
    const int li = (int)lv - rl.min_level;
    RoiGeom g;
    g.li = li;
    g.H = rl.H[li];
    g.W = rl.W[li];
    g.feat = reinterpret_cast<const char *>(rl.feat[li]) + (size_t)b * g.H * g.W * rl.C * esize;
    const float sc = rl.scale[li];
    const float off = rl.aligned ? 0.5f : 0.f;
    g.rsw = x1 * sc - off;
    g.rsh = y1 * sc - off;
    const float rew = x2 * sc - off, reh = y2 * sc - off;
    float rw = rew - g.rsw, rh = reh - g.rsh;
    if (!rl.aligned) {
        rw = fmaxf(rw, 1.f);
        rh = fmaxf(rh, 1.f);
    }
    const int P = rl.P;
    g.bh = rh / (float)P;
    g.bw = rw / (float)P;
    g.gh = rl.sampling > 0 ? rl.sampling : (int)ceilf(rh / (float)P);
    g.gw = rl.sampling > 0 ? rl.sampling : (int)ceilf(rw / (float)P);
    g.count = (float)max(g.gh * g.gw, 1);
    return g;
}

// bilinear taps of one sample coordinate along one axis (roi_align_forward's
// bilinear_interpolate): returns false when the sample is outside (-1, size]
__device__ __forceinline__ bool roi_axis(float v, int size, int &lo, int &hi, float &l) {
    if (!(v >= -1.0f && v <= (float)size)) return false;  // (also rejects NaN)
    float vv = v <= 0.f ? 0.f : v;
    lo = (int)vv;
    if (lo >= size - 1) {
        hi = lo = size - 1;
        vv = (float)lo;
    } else {
        hi = lo + 1;
    }
    l = vv - (float)lo;
    return true;
}

// Grid (ROI, channel slice of up to 128 B).  Per workgroup: (1) the bilinear
// tap rows/cols and fractions of the ROI's P*gh sample rows and P*gw sample
// columns are computed once into LDS (the coordinate arithmetic -- including
// its divisions -- is the same for every channel); (2) the slice of the ROI's
// sample window is staged in LDS with 16-B loads, so each feature pixel is
// fetched once per ROI instead of once per tap of every sample (windows above
// ROI_WIN_BYTES read their taps from global memory); (3) every (bin,
// 16-B group) lane gathers and blends.  Arithmetic (sample positions,
// weights, accumulation order) is the reference kernel's per-sample formula.
constexpr int ROI_TAB = 256;     // max P*gh (and P*gw) held in the tables

// one 16-B LDS-DMA piece per lane: LDS destination = lds_base + 16 * lane
__device__ __forceinline__ void roi_glds16(const void *src, char *lds_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}
constexpr int ROI_WIN_BYTES = 224 * 128;  // staged window cap (pixels x slice bytes)

template <typename T>
__global__ __launch_bounds__(256) void k_roi_align(RoiLevels rl, const float *__restrict__ rois,
                                                   const int *__restrict__ counts, int gslice, T *__restrict__ out) {
    constexpr int V = Vec16<T>::N;  // channels per 16-B group
    __shared__ int s_y0[ROI_TAB], s_y1[ROI_TAB], s_x0[ROI_TAB], s_x1[ROI_TAB];
    __shared__ float s_ly[ROI_TAB], s_lx[ROI_TAB];
    __shared__ __attribute__((aligned(16))) char s_win[ROI_WIN_BYTES];
    // XCD-contiguous ROI ranges: the ROIs of one image share its feature maps
    const int r = roi_of_block(rl);
    const int G = gslice, PXB = G * 16;  // 16-B groups per slice, LDS bytes per pixel
    const int b = r / rl.per_image, ri = r - b * rl.per_image;
    const int C = rl.C, P = rl.P;
    const int c0 = blockIdx.y * G * V;
    T *o = out + (long long)r * P * P * C + c0;
    const int nitems = P * P * G;
    if (ri >= counts[b]) {
        const float z[V] = {};
        for (int i = threadIdx.x; i < nitems; i += 256) st16(o + (long long)(i / G) * C + (i % G) * V, z);
        return;
    }
    const RoiGeom g = roi_geom(rl, rois, r, b, sizeof(T));
    const T *f = reinterpret_cast<const T *>(g.feat) + c0;
    const int ny = P * g.gh, nx = P * g.gw;
    const bool tab = g.gh > 0 && g.gw > 0 && ny <= ROI_TAB && nx <= ROI_TAB;
    int ylo = 0, yhi = -1, xlo = 0, xhi = -1;
    if (tab) {
        for (int e = threadIdx.x; e < ny; e += 256) {
            const int ph = e / g.gh, iy = e - ph * g.gh;
            const float y = g.rsh + (float)ph * g.bh + ((float)iy + .5f) * g.bh / (float)g.gh;
            int lo, hi;
            float l;
            const bool ok = roi_axis(y, g.H, lo, hi, l);
            s_y0[e] = ok ? lo : -1;
            s_y1[e] = hi;
            s_ly[e] = l;
        }
        for (int e = threadIdx.x; e < nx; e += 256) {
            const int pw = e / g.gw, ix = e - pw * g.gw;
            const float x = g.rsw + (float)pw * g.bw + ((float)ix + .5f) * g.bw / (float)g.gw;
            int lo, hi;
            float l;
            const bool ok = roi_axis(x, g.W, lo, hi, l);
            s_x0[e] = ok ? lo : -1;
            s_x1[e] = hi;
            s_lx[e] = l;
        }
        __syncthreads();
        // window: rows/cols touched by the valid samples (tables are monotonic)
        for (int e = 0; e < ny; ++e)
            if (s_y0[e] >= 0) {
                ylo = s_y0[e];
                break;
            }
        for (int e = ny - 1; e >= 0; --e)
            if (s_y0[e] >= 0) {
                yhi = s_y1[e];
                break;
            }
        for (int e = 0; e < nx; ++e)
            if (s_x0[e] >= 0) {
                xlo = s_x0[e];
                break;
            }
        for (int e = nx - 1; e >= 0; --e)
            if (s_x0[e] >= 0) {
                xhi = s_x1[e];
                break;
            }
    }
    const int wh = yhi - ylo + 1, ww = xhi - xlo + 1;
    const bool staged = tab && wh > 0 && ww > 0 && wh * ww * PXB <= ROI_WIN_BYTES;
    if (staged) {
        // LDS-DMA: piece i (pixel i / G, 16-B group i % G) lands at byte 16 i
        // of the window, i.e. wave-uniform base + 16 * lane, so every piece
        // of the window is one global_load_lds_dwordx4 and all of a thread's
        // (<= ROI_STAGE) pieces are in flight together.  Lanes past the end
        // re-fetch piece 0 into the unused tail of the window.
        const int npc = wh * ww * G;
        const int nrounds = (npc + 255) / 256;
        for (int j = 0; j < nrounds; ++j) {
            const int i0 = j * 256 + (threadIdx.x & ~63);
            int i = i0 + (threadIdx.x & 63);
            i = i < npc ? i : 0;
            const int px = i / G, cg = i - px * G;
            const int py = px / ww, pxx = px - py * ww;
            const T *src = f + ((long long)(ylo + py) * g.W + xlo + pxx) * C + cg * V;
            roi_glds16(src, s_win + i0 * 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    for (int t = threadIdx.x; t < nitems; t += 256) {
        const int bin = t / G, cg = t - bin * G;
        const int ph = bin / P, pw = bin - ph * P;
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
        for (int iy = 0; iy < g.gh; ++iy) {
            int yl, yh;
            float ly;
            if (tab) {
                const int e = ph * g.gh + iy;
                yl = s_y0[e];
                yh = s_y1[e];
                ly = s_ly[e];
                if (yl < 0) continue;
            } else {
                const float y = g.rsh + (float)ph * g.bh + ((float)iy + .5f) * g.bh / (float)g.gh;
                if (!roi_axis(y, g.H, yl, yh, ly)) continue;
            }
            for (int ix = 0; ix < g.gw; ++ix) {
                int xl, xh;
                float lx;
                if (tab) {
                    const int e = pw * g.gw + ix;
                    xl = s_x0[e];
                    xh = s_x1[e];
                    lx = s_lx[e];
                    if (xl < 0) continue;
                } else {
                    const float x = g.rsw + (float)pw * g.bw + ((float)ix + .5f) * g.bw / (float)g.gw;
                    if (!roi_axis(x, g.W, xl, xh, lx)) continue;
                }
                const float hy = 1.f - ly, hx = 1.f - lx;
                const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
                float v1[V], v2[V], v3[V], v4[V];
                if (staged) {
                    const char *w0 = s_win + cg * 16;
                    const int a0 = (yl - ylo) * ww - xlo, a1 = (yh - ylo) * ww - xlo;
                    ld16(reinterpret_cast<const T *>(w0 + (a0 + xl) * PXB), v1);
                    ld16(reinterpret_cast<const T *>(w0 + (a0 + xh) * PXB), v2);
                    ld16(reinterpret_cast<const T *>(w0 + (a1 + xl) * PXB), v3);
                    ld16(reinterpret_cast<const T *>(w0 + (a1 + xh) * PXB), v4);
                } else {
                    const T *fc = f + cg * V;
                    ld16(fc + ((long long)yl * g.W + xl) * C, v1);
                    ld16(fc + ((long long)yl * g.W + xh) * C, v2);
                    ld16(fc + ((long long)yh * g.W + xl) * C, v3);
                    ld16(fc + ((long long)yh * g.W + xh) * C, v4);
                }
#pragma unroll
                for (int i = 0; i < V; ++i) acc[i] += w1 * v1[i] + w2 * v2[i] + w3 * v3[i] + w4 * v4[i];
            }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = acc[i] / g.count;
        st16(o + (long long)bin * C + cg * V, acc);
    }
}

// One workgroup per ROI over all C channels (grid R).  The bilinear tap
// tables of the ROI's P*gh sample rows / P*gw sample columns are built once in
// LDS; then items (bin, 16-B channel group), group fastest, gather their taps
// straight from the NHWC map (a wave-instruction reads whole 512-B pixel
// rows), accumulate in the reference's per-sample order and store 16 B.
// Every thread owns ~P*P*C/(8*256) items, so the ROI's fixed costs (count and
// box loads, level, tables) are paid once for all channels.
template <typename T, int ROI_NI>
__global__ __launch_bounds__(256) void k_roi_align_full(RoiLevels rl, const float *__restrict__ rois,
                                                        const int *__restrict__ counts, T *__restrict__ out) {
    constexpr int V = Vec16<T>::N;
    __shared__ int s_y0[ROI_TAB], s_y1[ROI_TAB], s_x0[ROI_TAB], s_x1[ROI_TAB];
    __shared__ float s_ly[ROI_TAB], s_lx[ROI_TAB];
    const int r = roi_of_block(rl);
    const int b = r / rl.per_image, ri = r - b * rl.per_image;
    const int C = rl.C, P = rl.P;
    const int G = C / V;  // 16-B groups per pixel
    T *o = out + (long long)r * P * P * C;
    const int nitems = P * P * G;
    if (ri >= counts[b]) {
        const float z[V] = {};
        for (int i = threadIdx.x; i < nitems; i += 256) st16(o + (long long)i * V, z);
        return;
    }
    const RoiGeom g = roi_geom(rl, rois, r, b, sizeof(T));
    const T *f = reinterpret_cast<const T *>(g.feat);
    const int ny = P * g.gh, nx = P * g.gw;
    const bool tab = g.gh > 0 && g.gw > 0 && ny <= ROI_TAB && nx <= ROI_TAB;
    if (tab) {
        for (int e = threadIdx.x; e < ny; e += 256) {
            const int ph = e / g.gh, iy = e - ph * g.gh;
            const float y = g.rsh + (float)ph * g.bh + ((float)iy + .5f) * g.bh / (float)g.gh;
            int lo, hi;
            float l;
            const bool ok = roi_axis(y, g.H, lo, hi, l);
            s_y0[e] = ok ? lo : -1;
            s_y1[e] = hi;
            s_ly[e] = l;
        }
        for (int e = threadIdx.x; e < nx; e += 256) {
            const int pw = e / g.gw, ix = e - pw * g.gw;
            const float x = g.rsw + (float)pw * g.bw + ((float)ix + .5f) * g.bw / (float)g.gw;
            int lo, hi;
            float l;
            const bool ok = roi_axis(x, g.W, lo, hi, l);
            s_x0[e] = ok ? lo : -1;
            s_x1[e] = hi;
            s_lx[e] = l;
        }
        __syncthreads();
    }
    // ROI_NI items per thread in lockstep (gh, gw are uniform over the ROI),
    // so 4 * ROI_NI tap loads are in flight per sample
    for (int t0 = threadIdx.x; t0 < nitems; t0 += 256 * ROI_NI) {
        int ph[ROI_NI], pw[ROI_NI];
        const T *fc[ROI_NI];
        float acc[ROI_NI][V];
#pragma unroll
        for (int k = 0; k < ROI_NI; ++k) {
            int t = t0 + k * 256;
            t = t < nitems ? t : t0;  // idle slots recompute item t0 (not stored)
            const int bin = t / G, cg = t - bin * G;
            ph[k] = bin / P;
            pw[k] = bin - ph[k] * P;
            fc[k] = f + cg * V;
#pragma unroll
            for (int i = 0; i < V; ++i) acc[k][i] = 0.f;
        }
        for (int iy = 0; iy < g.gh; ++iy) {
            int yl[ROI_NI], yh[ROI_NI];
            float ly[ROI_NI];
#pragma unroll
            for (int k = 0; k < ROI_NI; ++k) {
                if (tab) {
                    const int e = ph[k] * g.gh + iy;
                    yl[k] = s_y0[e];
                    yh[k] = s_y1[e];
                    ly[k] = s_ly[e];
                } else {
                    const float y = g.rsh + (float)ph[k] * g.bh + ((float)iy + .5f) * g.bh / (float)g.gh;
                    if (!roi_axis(y, g.H, yl[k], yh[k], ly[k])) yl[k] = -1;
                }
            }
            for (int ix = 0; ix < g.gw; ++ix) {
                float v[ROI_NI][4][V], w[ROI_NI][4];
                bool ok[ROI_NI];
#pragma unroll
                for (int k = 0; k < ROI_NI; ++k) {
                    int xl, xh;
                    float lx;
                    if (tab) {
                        const int e = pw[k] * g.gw + ix;
                        xl = s_x0[e];
                        xh = s_x1[e];
                        lx = s_lx[e];
                    } else {
                        const float x = g.rsw + (float)pw[k] * g.bw + ((float)ix + .5f) * g.bw / (float)g.gw;
                        if (!roi_axis(x, g.W, xl, xh, lx)) xl = -1;
                    }
                    ok[k] = yl[k] >= 0 && xl >= 0;
                    const float hy = 1.f - ly[k], hx = 1.f - lx;
                    w[k][0] = hy * hx;
                    w[k][1] = hy * lx;
                    w[k][2] = ly[k] * hx;
                    w[k][3] = ly[k] * lx;
                    const int y0 = ok[k] ? yl[k] : 0, y1 = ok[k] ? yh[k] : 0;
                    const int x0 = ok[k] ? xl : 0, x1 = ok[k] ? xh : 0;
                    const T *r0 = fc[k] + (long long)y0 * g.W * C, *r1 = fc[k] + (long long)y1 * g.W * C;
                    ld16(r0 + (long long)x0 * C, v[k][0]);
                    ld16(r0 + (long long)x1 * C, v[k][1]);
                    ld16(r1 + (long long)x0 * C, v[k][2]);
                    ld16(r1 + (long long)x1 * C, v[k][3]);
                }
#pragma unroll
                for (int k = 0; k < ROI_NI; ++k) {
                    if (!ok[k]) continue;
#pragma unroll
                    for (int i = 0; i < V; ++i)
                        acc[k][i] += w[k][0] * v[k][0][i] + w[k][1] * v[k][1][i] + w[k][2] * v[k][2][i] +
                                     w[k][3] * v[k][3][i];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < ROI_NI; ++k) {
            const int t = t0 + k * 256;
            if (t >= nitems) continue;
#pragma unroll
            for (int i = 0; i < V; ++i) acc[k][i] = acc[k][i] / g.count;
            st16(o + (long long)t * V, acc[k]);
        }
    }
}

// kernel choice (tests / microbenchmarks): 0 slice + LDS window; 1, 2, 3:
// full-channel rows with 1, 2, 4 items per thread in lockstep
// Separable form of the same average (mode 4): a sample's bilinear weights
// factor into a row part and a column part, so the bin average over its gh x gw
// sample grid is sum_r sum_c A[r] B[c] F[r][c] / count, with A[r] (B[c]) the
// summed row (column) weights of the bin's sample rows (columns).  With the
// adaptive grid (gh = ceil(bin height)) samples are <= 1 px apart and a bin
// touches gh + 1 rows: (gh+1)(gw+1) 16-B taps per output group instead of
// 4 gh gw (16 instead of 36 at 3 x 3) -- the tap loads through the texture
// path are what bound this kernel.  Rounding differs from the per-sample sum
// (fp32, ~1 ulp); bins needing more than ROI_RMAX rows or columns (fixed
// sampling ratios) take the per-sample path.
//
// ROWS (mode 5): the same sum as sum_c B[c] (sum_r A[r] F[r][c]): per bin row,
// the row-weighted values R[x] of every column x of the ROI's span are formed
// once in LDS (fp32) and shared by all P bins of that row, so a row of bins
// costs nr * (span) 16-B taps instead of P * nr * (nc)
// ((7 gw + 1) vs 7 (gw + 1) columns; rounding again ~1 ulp).  Spans wider
// than ROI_SPAN_FLOATS / C columns take the mode-4 loop.
constexpr int ROI_RMAX = 8, ROI_PMAX = 16, ROI_SPAN_FLOATS = 8192;
// WIN (mode 6): the ROI's whole sample window of a slice of ROI_SWIN_SG 16-B
// channel groups is staged in LDS once (each map pixel read once from L2
// instead of once per bin that touches it: ~2x fewer tap loads for the box
// pooler's 2-px bins), then every bin reads its taps from LDS in mode 4's
// order (same sums, bit for bit).  Windows above ROI_SWIN_BYTES per slice take
// mode 4's loop.
constexpr int ROI_SWIN_SG = 8, ROI_SWIN_BYTES = 32768;
#ifndef MDX_ROI_TAPS9  // (A/B builds: 0 = every bin through the padded two-round loop)
#define MDX_ROI_TAPS9 1
#endif

// x / c for the bin average with the ROI's reciprocal r = RN(1/c): q = RN(x r)
// refined by one FMA residual step (Markstein), 3 VALU instead of the ~10 of
// the IEEE division sequence per output element (the box pooler is VALU-
// bound: PMC SQ_INSTS_VALU).  Equal to RN(x / c) up to the rare last-ulp
// cases the oracle tolerance covers.
__device__ __forceinline__ float div_count(float x, float c, float r) {
    const float q = x * r;
    const float e = __builtin_fmaf(-q, c, x);
    return __builtin_fmaf(e, r, q);
}

template <typename T, bool ROWS = false, bool WIN = false>
__global__ __launch_bounds__(256) void k_roi_align_sep(RoiLevels rl, const float *__restrict__ rois,
                                                       const int *__restrict__ counts, T *__restrict__ out) {
    constexpr int V = Vec16<T>::N;
    __shared__ int s_r0[ROI_PMAX], s_nr[ROI_PMAX], s_c0[ROI_PMAX], s_nc[ROI_PMAX];
    __shared__ float s_A[ROI_PMAX][ROI_RMAX], s_B[ROI_PMAX][ROI_RMAX];
    __shared__ int s_bad;
    const int r = roi_of_block(rl);
    const int b = r / rl.per_image, ri = r - b * rl.per_image;
    const int C = rl.C, P = rl.P;
    const int G = C / V;
    T *o = out + (long long)r * P * P * C;
    const int nitems = P * P * G;
    // output of element e of this ROI's row: 16 B of T, or (planes, fp32) the
    // three bf16 planes of the 4 values
    char *const prow = sizeof(T) == 4 && rl.planes ? reinterpret_cast<char *>(out) + (long long)r * P * P * C * 6 : nullptr;
    auto put = [&](long long e, const float *v) {
        if (sizeof(T) == 4 && prow)
            st4_planes(prow, e, v);
        else
            st16(o + e, v);
    };
    // gridDim.y workgroups share one ROI's items (small ROI counts: mask /
    // keypoint poolers), each building the ROI's tables itself
    const int tstart = threadIdx.x + 256 * blockIdx.y, tstep = 256 * gridDim.y;
    if (ri >= counts[b]) {
        const float z[V] = {};
        for (int i = tstart; i < nitems; i += tstep) put((long long)i * V, z);
        return;
    }
    const RoiGeom g = roi_geom(rl, rois, r, b, sizeof(T));
    const T *f = reinterpret_cast<const T *>(g.feat);
    const float inv_count = 1.0f / g.count;  // once per ROI (see div_count)
    if (threadIdx.x == 0) s_bad = P > ROI_PMAX;
    __syncthreads();
    // row tables by lanes 0..P-1 of wave 0, column tables by wave 1
    const int w = threadIdx.x >> 6, lidx = threadIdx.x & 63;
    if (w < 2 && lidx < P && P <= ROI_PMAX) {
        const bool rows = w == 0;
        const int n = rows ? g.gh : g.gw, size = rows ? g.H : g.W;
        const float st = rows ? g.rsh : g.rsw, bsz = rows ? g.bh : g.bw;
        float wt[ROI_RMAX];
#pragma unroll
        for (int j = 0; j < ROI_RMAX; ++j) wt[j] = 0.f;
        int base = -1, cnt = 0;
        bool bad = false;
        for (int i = 0; i < n; ++i) {
            const float v = st + (float)lidx * bsz + ((float)i + .5f) * bsz / (float)n;
            int lo, hi;
            float l;
            if (!roi_axis(v, size, lo, hi, l)) continue;
            if (base < 0) base = lo;
            const int a = lo - base, c = hi - base;
            if (c >= ROI_RMAX) {
                bad = true;
                break;
            }
#pragma unroll
            for (int j = 0; j < ROI_RMAX; ++j) wt[j] += (j == a ? 1.f - l : 0.f) + (j == c ? l : 0.f);
            cnt = c + 1 > cnt ? c + 1 : cnt;
        }
        if (bad) s_bad = 1;
        if (rows) {
            s_r0[lidx] = base < 0 ? 0 : base;
            s_nr[lidx] = cnt;
#pragma unroll
            for (int j = 0; j < ROI_RMAX; ++j) s_A[lidx][j] = wt[j];
        } else {
            s_c0[lidx] = base < 0 ? 0 : base;
            s_nc[lidx] = cnt;
#pragma unroll
            for (int j = 0; j < ROI_RMAX; ++j) s_B[lidx][j] = wt[j];
        }
    }
    __syncthreads();
    if (s_bad) {
        // per-sample path (the reference formula), taps from global memory
        for (int t = tstart; t < nitems; t += tstep) {
            const int bin = t / G, cg = t - bin * G;
            const int ph = bin / P, pw = bin - ph * P;
            const T *fc = f + cg * V;
            float acc[V];
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = 0.f;
            for (int iy = 0; iy < g.gh; ++iy) {
                const float y = g.rsh + (float)ph * g.bh + ((float)iy + .5f) * g.bh / (float)g.gh;
                int yl, yh;
                float ly;
                if (!roi_axis(y, g.H, yl, yh, ly)) continue;
                for (int ix = 0; ix < g.gw; ++ix) {
                    const float x = g.rsw + (float)pw * g.bw + ((float)ix + .5f) * g.bw / (float)g.gw;
                    int xl, xh;
                    float lx;
                    if (!roi_axis(x, g.W, xl, xh, lx)) continue;
                    const float hy = 1.f - ly, hx = 1.f - lx;
                    float v1[V], v2[V], v3[V], v4[V];
                    ld16(fc + ((long long)yl * g.W + xl) * C, v1);
                    ld16(fc + ((long long)yl * g.W + xh) * C, v2);
                    ld16(fc + ((long long)yh * g.W + xl) * C, v3);
                    ld16(fc + ((long long)yh * g.W + xh) * C, v4);
#pragma unroll
                    for (int i = 0; i < V; ++i)
                        acc[i] += hy * hx * v1[i] + hy * lx * v2[i] + ly * hx * v3[i] + ly * lx * v4[i];
                }
            }
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = acc[i] / g.count;
            put((long long)t * V, acc);
        }
        return;
    }
    if constexpr (ROWS) {
        __shared__ int s_span[2];
        __shared__ __attribute__((aligned(16))) float sR[ROI_SPAN_FLOATS];
        if (threadIdx.x == 0) {
            int lo = 1 << 30, hi = 0;
            for (int pw = 0; pw < P; ++pw)
                if (s_nc[pw] > 0) {
                    lo = s_c0[pw] < lo ? s_c0[pw] : lo;
                    hi = s_c0[pw] + s_nc[pw] > hi ? s_c0[pw] + s_nc[pw] : hi;
                }
            if (lo > hi) lo = hi = 0;
            s_span[0] = lo;
            s_span[1] = hi - lo;
        }
        __syncthreads();
        const int cx0 = s_span[0], span = s_span[1];
        if (span * C <= ROI_SPAN_FLOATS) {
            const int n1 = span * G, n2 = P * G;
            for (int ph = 0; ph < P; ++ph) {
                const int nr = s_nr[ph];
                const T *rowp = f + ((long long)s_r0[ph] * g.W + cx0) * C;
                for (int it = threadIdx.x; it < n1; it += 256) {
                    const int x = it / G, cg = it - x * G;
                    const T *src = rowp + (long long)x * C + cg * V;
                    float acc[V];
#pragma unroll
                    for (int i = 0; i < V; ++i) acc[i] = 0.f;
                    for (int j = 0; j < nr; j += 2) {
                        const bool two = j + 1 < nr;
                        float v0[V], v1[V];
                        ld16(src + (long long)j * g.W * C, v0);
                        ld16(src + (long long)(two ? j + 1 : j) * g.W * C, v1);
                        const float a0 = s_A[ph][j], a1 = two ? s_A[ph][j + 1] : 0.f;
#pragma unroll
                        for (int i = 0; i < V; ++i) acc[i] += a0 * v0[i] + a1 * v1[i];
                    }
                    float *d = sR + x * C + cg * V;
#pragma unroll
                    for (int i = 0; i < V; i += 4)
                        *reinterpret_cast<float4 *>(d + i) = make_float4(acc[i], acc[i + 1], acc[i + 2], acc[i + 3]);
                }
                __syncthreads();
                for (int it = threadIdx.x; it < n2; it += 256) {
                    const int pw = it / G, cg = it - pw * G;
                    const int nc = s_nc[pw];
                    const float *srow = sR + (s_c0[pw] - cx0) * C + cg * V;
                    float acc[V];
#pragma unroll
                    for (int i = 0; i < V; ++i) acc[i] = 0.f;
                    for (int k = 0; k < nc; ++k) {
                        const float bk = s_B[pw][k];
#pragma unroll
                        for (int i = 0; i < V; i += 4) {
                            const float4 r4 = *reinterpret_cast<const float4 *>(srow + k * C + i);
                            acc[i] += bk * r4.x;
                            acc[i + 1] += bk * r4.y;
                            acc[i + 2] += bk * r4.z;
                            acc[i + 3] += bk * r4.w;
                        }
                    }
#pragma unroll
                    for (int i = 0; i < V; ++i) acc[i] = div_count(acc[i], g.count, inv_count);
                    put(((long long)(ph * P + pw) * G + cg) * V, acc);
                }
                __syncthreads();
            }
            return;
        }
    }
    if constexpr (WIN) {
        __shared__ int s_win[4];
        __shared__ __attribute__((aligned(16))) uint4 sW[ROI_SWIN_BYTES / 16];
        if (threadIdx.x == 0) {
            int y0 = 1 << 30, y1 = 0, x0 = 1 << 30, x1 = 0;
            for (int q = 0; q < P; ++q) {
                if (s_nr[q] > 0) {
                    y0 = s_r0[q] < y0 ? s_r0[q] : y0;
                    y1 = s_r0[q] + s_nr[q] > y1 ? s_r0[q] + s_nr[q] : y1;
                }
                if (s_nc[q] > 0) {
                    x0 = s_c0[q] < x0 ? s_c0[q] : x0;
                    x1 = s_c0[q] + s_nc[q] > x1 ? s_c0[q] + s_nc[q] : x1;
                }
            }
            if (y0 > y1) y0 = y1 = 0;
            if (x0 > x1) x0 = x1 = 0;
            s_win[0] = y0;
            s_win[1] = y1 - y0;
            s_win[2] = x0;
            s_win[3] = x1 - x0;
        }
        __syncthreads();
        const int wy0 = s_win[0], wr = s_win[1], wx0 = s_win[2], wc = s_win[3];
        constexpr int SG = ROI_SWIN_SG;
        if (G % SG == 0 && (long long)wr * wc * SG * 16 <= ROI_SWIN_BYTES && gridDim.y == 1) {
            const int npx = wr * wc, nst = npx * SG, nit = P * P * SG;
            for (int sl = 0; sl < G; sl += SG) {
                // stage the window's pixels of channel groups sl .. sl + SG
                for (int it = threadIdx.x; it < nst; it += 256) {
                    const int px = it / SG, cg = it - px * SG;
                    const int y = px / wc, x = px - y * wc;
                    sW[it] = *reinterpret_cast<const uint4 *>(f + ((long long)(wy0 + y) * g.W + (wx0 + x)) * C +
                                                              (sl + cg) * V);
                }
                __syncthreads();
                for (int it = threadIdx.x; it < nit; it += 256) {
                    const int bin = it / SG, cg = it - bin * SG;
                    const int ph = bin / P, pw = bin - ph * P;
                    const int nr = s_nr[ph], nc = s_nc[pw];
                    const uint4 *wp = sW + ((s_r0[ph] - wy0) * wc + (s_c0[pw] - wx0)) * SG + cg;
                    float acc[V];
#pragma unroll
                    for (int i = 0; i < V; ++i) acc[i] = 0.f;
                    for (int j = 0; j < nr; j += 2) {
                        const bool two = j + 1 < nr;
                        const float a0 = s_A[ph][j], a1 = two ? s_A[ph][j + 1] : 0.f;
                        const uint4 *rp0 = wp + j * wc * SG;
                        const uint4 *rp1 = two ? rp0 + wc * SG : rp0;
                        for (int kc = 0; kc < nc; kc += 4) {
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int k = kc + u < nc ? kc + u : nc - 1;
                                const uint4 r0 = rp0[k * SG], r1 = rp1[k * SG];
                                const float bk = kc + u < nc ? s_B[pw][kc + u] : 0.f;
                                const float w0 = a0 * bk, w1 = a1 * bk;
                                const T *e0 = reinterpret_cast<const T *>(&r0);
                                const T *e1 = reinterpret_cast<const T *>(&r1);
#pragma unroll
                                for (int i = 0; i < V; ++i)
                                    acc[i] = __builtin_fmaf(w1, (float)e1[i], __builtin_fmaf(w0, (float)e0[i], acc[i]));
                            }
                        }
                    }
#pragma unroll
                    for (int i = 0; i < V; ++i) acc[i] = div_count(acc[i], g.count, inv_count);
                    put(((long long)bin * G + sl + cg) * V, acc);
                }
                __syncthreads();
            }
            return;
        }
    }
    // item t = (bin, channel group); when G divides 256 a thread keeps its
    // channel group and steps its bin by 256 / G (no divisions per item)
    const bool gstep = (tstep % G) == 0;
    const int bstep = gstep ? tstep / G : 0;
    int cg0 = tstart % G, bin0 = tstart / G;
    int ph0 = bin0 / P, pw0 = bin0 - ph0 * P;
    for (int t = tstart; t < nitems; t += tstep) {
        int cg = cg0, ph = ph0, pw = pw0;
        if (gstep) {
            pw0 += bstep;
            while (pw0 >= P) {
                pw0 -= P;
                ++ph0;
            }
        } else {
            const int bin = t / G;
            cg = t - bin * G;
            ph = bin / P;
            pw = bin - ph * P;
        }
        const int nr = s_nr[ph], nc = s_nc[pw];
        const T *fc = f + ((long long)s_r0[ph] * g.W + s_c0[pw]) * C + cg * V;
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
        // bins of at most 3 x 3 taps (3 / 4 of the box pooler's): the nine
        // taps loaded in one round (the loop below loads 16 in two rounds for a
        // 3 x 3 bin), then the loop's FMA sequence (rows in pairs, columns in
        // order, rows within a pair); an absent tap re-reads the bin's last
        // valid pixel with weight 0 and adds exactly nothing, as the loop's
        // padding taps do -- the same sums, bit for bit.  When G is a multiple
        // of 64 a wave's lanes share one bin, so the bounds are wave-uniform.
        if (MDX_ROI_TAPS9 && nr <= 3 && nc <= 3 && nr > 0 && nc > 0) {
            uint4 raw[9];
            float wq[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int jr = q < 6 ? (q & 1) : 2, k = q < 6 ? (q >> 1) : q - 6;
                const bool ok = jr < nr && k < nc;
                const int jc = ok ? jr : nr - 1, kk = ok ? k : nc - 1;
                raw[q] = *reinterpret_cast<const uint4 *>(fc + ((long long)jc * g.W + kk) * C);
                wq[q] = ok ? s_A[ph][jr] * s_B[pw][k] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const T *e = reinterpret_cast<const T *>(&raw[q]);
#pragma unroll
                for (int i = 0; i < V; ++i) acc[i] = __builtin_fmaf(wq[q], (float)e[i], acc[i]);
            }
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = div_count(acc[i], g.count, inv_count);
            put((long long)t * V, acc);
            continue;
        }
        // two rows x four columns of taps per round, all eight loads issued
        // before any is consumed (the kernel is bound by load latency):
        // out-of-range taps re-read the last valid pixel with weight 0
        for (int j = 0; j < nr; j += 2) {
            const bool two = j + 1 < nr;
            const float a0 = s_A[ph][j], a1 = two ? s_A[ph][j + 1] : 0.f;
            const T *rp0 = fc + (long long)j * g.W * C;
            const T *rp1 = two ? rp0 + (long long)g.W * C : rp0;
            for (int kc = 0; kc < nc; kc += 4) {
                uint4 raw[8];  // raw 16-B taps, converted inside the FMAs
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = kc + u < nc ? kc + u : nc - 1;
                    raw[u] = *reinterpret_cast<const uint4 *>(rp0 + (long long)k * C);
                    raw[4 + u] = *reinterpret_cast<const uint4 *>(rp1 + (long long)k * C);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float bk = kc + u < nc ? s_B[pw][kc + u] : 0.f;
                    const float w0 = a0 * bk, w1 = a1 * bk;
                    const T *e0 = reinterpret_cast<const T *>(&raw[u]);
                    const T *e1 = reinterpret_cast<const T *>(&raw[4 + u]);
                    // fma(w, (float)half, acc): one mixed-precision FMA per tap
                    // and channel (v_fma_mix_f32) instead of cvt + mul + fma + add
#pragma unroll
                    for (int i = 0; i < V; ++i)
                        acc[i] = __builtin_fmaf(w1, (float)e1[i], __builtin_fmaf(w0, (float)e0[i], acc[i]));
                }
            }
        }
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = div_count(acc[i], g.count, inv_count);
        put((long long)t * V, acc);
    }
}

// Per image, a permutation of its ROIs grouped by pyramid level and, within a
// level, by horizontal band of the sample window's centre row, valid ROIs
// first.  The pooler's workgroups in flight on one XCD then read one band of
// one level map (L2 reuse) instead of all four maps of the image (the box
// pooler fetched ~6x the map bytes in ROI order).  Positions come from LDS
// atomics, so the permutation varies from run to run; the pooled rows do
// not (every ROI writes its own rows with the same arithmetic).
__global__ __launch_bounds__(256) void k_roi_order(RoiLevels rl, const float *__restrict__ rois,
                                                   const int *__restrict__ counts, int *__restrict__ order) {
    __shared__ int s_off[256];
    const int b = blockIdx.x, n = rl.per_image, t = threadIdx.x;
    const int valid = min(counts[b], n);
    const int bands = 255 / rl.L, NK = rl.L * bands + 1;  // last key: empty slots
    auto key = [&](int k) -> int {
        if (k >= valid) return NK - 1;
        const RoiGeom g = roi_geom(rl, rois, b * n + k, b, 4);
        const float cy = g.rsh + 0.5f * g.bh * (float)rl.P;
        int band = (int)(cy * (float)bands / (float)g.H);
        band = band < 0 ? 0 : (band >= bands ? bands - 1 : band);
        return g.li * bands + band;
    };
    s_off[t] = 0;
    __syncthreads();
    for (int k = t; k < n; k += 256) atomicAdd(&s_off[key(k)], 1);
    __syncthreads();
    // exclusive scan of the 256 counts (Hillis-Steele, inclusive then shift)
    int v = s_off[t];
    for (int d = 1; d < 256; d <<= 1) {
        __syncthreads();
        const int u = t >= d ? s_off[t - d] : 0;
        __syncthreads();
        v += u;
        s_off[t] = v;
    }
    __syncthreads();
    const int excl = t ? s_off[t - 1] : 0;
    __syncthreads();
    s_off[t] = excl;
    __syncthreads();
    for (int k = t; k < n; k += 256) {
        const int pos = atomicAdd(&s_off[key(k)], 1);
        order[b * n + pos] = b * n + k;
    }
}

// ---------------------------------------------------------------------------
// box head post-process (fast_rcnn_inference_single_image + detector_postprocess)
// ---------------------------------------------------------------------------
struct BoxPostArgs {
    int R, ld_pred;  // rows per image, row stride of pred (f32 columns)
    int D;           // detections per image
    float score_thresh, nms_thresh, img_h, img_w, clampv;
    float wts[4];
};

__global__ __launch_bounds__(1024) void k_box_post(BoxPostArgs ba, const float *__restrict__ pred,
                                                   const float *__restrict__ props, const int *__restrict__ counts,
                                                   float *__restrict__ det_boxes, float *__restrict__ det_scores,
                                                   long long *__restrict__ det_classes, int *__restrict__ ndet) {
    __shared__ unsigned key[1024], val[1024];
    __shared__ float bxs[1024][4];
    __shared__ float scs[1024];
    const int b = blockIdx.x;
    const int R = ba.R;
    for (int i = threadIdx.x; i < 1024; i += 1024) {
        key[i] = 0;
        val[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    const int n = counts[b];
    for (int r = threadIdx.x; r < R && r < 1024; r += 1024) {
        if (r >= n) continue;
        const float *p = pred + ((long long)b * R + r) * ba.ld_pred;
        // softmax over (cls0, bg)
        const float l0 = p[0], l1 = p[1];
        const float mx = fmaxf(l0, l1);
        const float e0 = expf(l0 - mx), e1 = expf(l1 - mx);
        const float sum = e0 + e1;
        const float s0 = e0 / sum;
        float bx[4];
        apply_delta(props + ((long long)b * R + r) * 4, p[2], p[3], p[4], p[5], ba.wts, ba.clampv, bx);
        const bool fin = isfinite(bx[0]) && isfinite(bx[1]) && isfinite(bx[2]) && isfinite(bx[3]) && isfinite(s0) &&
                         isfinite(e1 / sum);
        bx[0] = clampf(bx[0], 0.f, ba.img_w);
        bx[1] = clampf(bx[1], 0.f, ba.img_h);
        bx[2] = clampf(bx[2], 0.f, ba.img_w);
        bx[3] = clampf(bx[3], 0.f, ba.img_h);
        bxs[r][0] = bx[0]; bxs[r][1] = bx[1]; bxs[r][2] = bx[2]; bxs[r][3] = bx[3];
        scs[r] = s0;
        if (fin && s0 > ba.score_thresh) {
            key[r] = fkey(s0);
            val[r] = (unsigned)r;
        }
    }
    bitonic_desc(key, val, 1024);
    if (threadIdx.x == 0) {
        int kept[16];
        int nk = 0;
        for (int i = 0; i < 1024 && nk < ba.D; ++i) {
            if (val[i] == 0xFFFFFFFFu) break;
            const int r = (int)val[i];
            const float ix1 = bxs[r][0], iy1 = bxs[r][1], ix2 = bxs[r][2], iy2 = bxs[r][3];
            bool sup = false;
            for (int q = 0; q < nk && !sup; ++q) {
                const int j = kept[q];
                // torchvision: suppress j (later) by kept i (earlier): IoU with the kept box
                const float kx1 = bxs[j][0], ky1 = bxs[j][1], kx2 = bxs[j][2], ky2 = bxs[j][3];
                const float karea = (kx2 - kx1) * (ky2 - ky1);
                const float xx1 = fmaxf(kx1, ix1), yy1 = fmaxf(ky1, iy1);
                const float xx2 = fminf(kx2, ix2), yy2 = fminf(ky2, iy2);
                const float w_ = fmaxf(0.f, xx2 - xx1), h_ = fmaxf(0.f, yy2 - yy1);
                const float inter = w_ * h_;
                const float iarea = (ix2 - ix1) * (iy2 - iy1);
                const float ovr = inter / (karea + iarea - inter);
                sup = ovr > ba.nms_thresh;
            }
            if (!sup) kept[nk++] = r;
        }
        // detector_postprocess: clip (no-op, already clipped) + nonempty
        int m = 0;
        for (int q = 0; q < nk; ++q) {
            const int r = kept[q];
            if (!((bxs[r][2] - bxs[r][0]) > 0.f && (bxs[r][3] - bxs[r][1]) > 0.f)) continue;
            float *ob = det_boxes + ((long long)b * ba.D + m) * 4;
            ob[0] = bxs[r][0]; ob[1] = bxs[r][1]; ob[2] = bxs[r][2]; ob[3] = bxs[r][3];
            det_scores[(long long)b * ba.D + m] = scs[r];
            det_classes[(long long)b * ba.D + m] = 0;
            ++m;
        }
        for (int q = m; q < ba.D; ++q) {
            float *ob = det_boxes + ((long long)b * ba.D + q) * 4;
            ob[0] = ob[1] = ob[2] = ob[3] = 0.f;
            det_scores[(long long)b * ba.D + q] = 0.f;
            det_classes[(long long)b * ba.D + q] = 0;
        }
        ndet[b] = m;
    }
}

// ---------------------------------------------------------------------------
// mask paste: sigmoid(logits) -> grid_sample(bilinear, zeros, align_corners=False) >= thr
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_paste(const float *__restrict__ logits, const float *__restrict__ boxes,
                                               const int *__restrict__ counts, int D, int M, int img_h, int img_w,
                                               long long plane, float thr, uint8_t *__restrict__ out) {
    __shared__ float prob[64 * 64];
    const int r = blockIdx.y;
    const int b = r / D, d = r - b * D;
    uint8_t *o = out + (long long)r * plane;
    const int rows_per_block = 8;
    const int y0 = blockIdx.x * rows_per_block;
    if (d >= counts[b]) {
        for (int i = threadIdx.x; i < rows_per_block * img_w; i += 256) {
            const int y = y0 + i / img_w, x = i % img_w;
            if (y < img_h) o[(long long)y * img_w + x] = 0;
        }
        return;
    }
    for (int i = threadIdx.x; i < M * M; i += 256) {
        const float v = logits[(long long)r * M * M + i];
        prob[i] = 1.0f / (1.0f + expf(-v));
    }
    __syncthreads();
    const float bx0 = boxes[4 * r], by0 = boxes[4 * r + 1], bx1 = boxes[4 * r + 2], by1 = boxes[4 * r + 3];
    for (int i = threadIdx.x; i < rows_per_block * img_w; i += 256) {
        const int y = y0 + i / img_w, x = i % img_w;
        if (y >= img_h) continue;
        const float gy = ((float)y + 0.5f - by0) / (by1 - by0) * 2.f - 1.f;
        const float gx = ((float)x + 0.5f - bx0) / (bx1 - bx0) * 2.f - 1.f;
        // ATen GridSamplerKernel (vectorised CPU path, align_corners=False):
        // unnormalize = (g + 1) * (size / 2) - 0.5; weights from floor distances
        const float ix = (gx + 1.f) * ((float)M / 2.f) - 0.5f;
        const float iy = (gy + 1.f) * ((float)M / 2.f) - 0.5f;
        const float fx = floorf(ix), fy = floorf(iy);
        const int xw = (int)fx, yn = (int)fy;
        const float w_ = ix - fx, e_ = 1.f - w_;
        const float n_ = iy - fy, s_ = 1.f - n_;
        const float nw = s_ * e_, ne = s_ * w_, sw = n_ * e_, se = n_ * w_;
        auto at = [&](int yy, int xx) -> float {
            return (yy >= 0 && yy < M && xx >= 0 && xx < M) ? prob[yy * M + xx] : 0.f;
        };
        const float v = ((at(yn, xw) * nw + at(yn, xw + 1) * ne) + at(yn + 1, xw) * sw) + at(yn + 1, xw + 1) * se;
        o[(long long)y * img_w + x] = v >= thr ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// keypoint head tail
// ---------------------------------------------------------------------------
// ConvTranspose2d(Cin -> Co, k=4, s=2, p=1) as GEMM + col2im:
// y (R*Hi*Wi, Co*16) f32 = x @ W[ci][co*16 + ky*4 + kx] (k_conv), then
// out[r][co][oy][ox] = bias[co] + sum_{ky,kx: oy = 2*iy - 1 + ky, ox = 2*ix - 1 + kx} y[r,iy,ix][co,ky,kx]
__global__ __launch_bounds__(256) void k_deconv_col2im(const float *__restrict__ y, const float *__restrict__ bias,
                                                       int R, int Hi, int Wi, int Co, float *__restrict__ out) {
    const int OH = 2 * Hi, OW = 2 * Wi;
    const long long total = (long long)R * Co * OH * OW;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const int ox = (int)(i % OW);
        const int oy = (int)((i / OW) % OH);
        const int co = (int)((i / ((long long)OH * OW)) % Co);
        const int r = (int)(i / ((long long)OH * OW * Co));
        float acc = bias ? bias[co] : 0.f;
        for (int ky = 0; ky < 4; ++ky) {
            const int ty = oy + 1 - ky;
            if (ty < 0 || (ty & 1)) continue;
            const int iy = ty >> 1;
            if (iy >= Hi) continue;
            for (int kx = 0; kx < 4; ++kx) {
                const int tx = ox + 1 - kx;
                if (tx < 0 || (tx & 1)) continue;
                const int ix = tx >> 1;
                if (ix >= Wi) continue;
                acc += y[(((long long)r * Hi + iy) * Wi + ix) * (Co * 16) + co * 16 + ky * 4 + kx];
            }
        }
        out[i] = acc;
    }
}

// F.interpolate(scale_factor=2, mode='bilinear', align_corners=False), NCHW f32
__global__ __launch_bounds__(256) void k_upsample2x(const float *__restrict__ x, int NC, int H, int W,
                                                    float *__restrict__ out) {
    const int OH = 2 * H, OW = 2 * W;
    const long long total = (long long)NC * OH * OW;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const int ox = (int)(i % OW);
        const int oy = (int)((i / OW) % OH);
        const long long nc = i / ((long long)OH * OW);
        const float rh = 0.5f, rw = 0.5f;  // 1 / scale_factor
        float sy = ((float)oy + 0.5f) * rh - 0.5f;
        sy = sy < 0.f ? 0.f : sy;
        float sx = ((float)ox + 0.5f) * rw - 0.5f;
        sx = sx < 0.f ? 0.f : sx;
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
        const float l1y = sy - (float)y0, l0y = 1.f - l1y;
        const float l1x = sx - (float)x0, l0x = 1.f - l1x;
        const float *p = x + nc * H * W;
        out[i] = l0y * (l0x * p[y0 * W + x0] + l1x * p[y0 * W + x1]) +
                 l1y * (l0x * p[y1 * W + x0] + l1x * p[y1 * W + x1]);
    }
}

__device__ __forceinline__ float cubic1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cubic2(float x, float A) {
    return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
}

// heatmaps_to_keypoints: one block per (roi, keypoint)
__global__ __launch_bounds__(256) void k_heatmap_kp(const float *__restrict__ maps, const float *__restrict__ boxes,
                                                    const int *__restrict__ counts, int D, int K, int M,
                                                    float *__restrict__ out) {
    __shared__ float red_v[256];
    __shared__ int red_i[256];
    __shared__ float red_s[256];
    const int r = blockIdx.x / K, kpt = blockIdx.x - r * K;
    const int b = r / D, d = r - b * D;
    float *o = out + ((long long)r * K + kpt) * 3;
    if (d >= counts[b]) {
        if (threadIdx.x == 0) o[0] = o[1] = o[2] = 0.f;
        return;
    }
    const float *mp = maps + ((long long)r * K + kpt) * M * M;
    const float x0 = boxes[4 * r], y0 = boxes[4 * r + 1], x1 = boxes[4 * r + 2], y1 = boxes[4 * r + 3];
    float wdt = x1 - x0, hgt = y1 - y0;
    wdt = wdt < 1.f ? 1.f : wdt;
    hgt = hgt < 1.f ? 1.f : hgt;
    const float wc = ceilf(wdt), hc = ceilf(hgt);
    const int OW = (int)wc, OH = (int)hc;
    const float sw = (float)M / (float)OW, sh = (float)M / (float)OH;  // area_pixel_compute_scale
    const float A = -0.75f;
    float best = -INFINITY;
    int besti = 0x7fffffff;
    for (int t = threadIdx.x; t < OH * OW; t += 256) {
        const int oy = t / OW, ox = t - oy * OW;
        const float ry = sh * ((float)oy + 0.5f) - 0.5f;
        const float rx = sw * ((float)ox + 0.5f) - 0.5f;
        const float fy = floorf(ry), fx = floorf(rx);
        const int iy = (int)fy, ix = (int)fx;
        const float ty = ry - fy, tx = rx - fx;
        const float cx[4] = {cubic2(tx + 1.f, A), cubic1(tx, A), cubic1(1.f - tx, A), cubic2(2.f - tx, A)};
        const float cy[4] = {cubic2(ty + 1.f, A), cubic1(ty, A), cubic1(1.f - ty, A), cubic2(2.f - ty, A)};
        float rows[4];
        for (int i = 0; i < 4; ++i) {
            int yy = iy - 1 + i;
            yy = yy < 0 ? 0 : (yy > M - 1 ? M - 1 : yy);
            float acc = 0.f;
            for (int j = 0; j < 4; ++j) {
                int xx = ix - 1 + j;
                xx = xx < 0 ? 0 : (xx > M - 1 ? M - 1 : xx);
                acc = acc + mp[yy * M + xx] * cx[j];
            }
            rows[i] = acc;
        }
        const float v = ((rows[0] * cy[0] + rows[1] * cy[1]) + rows[2] * cy[2]) + rows[3] * cy[3];
        if (v > best || (v == best && t < besti)) {
            best = v;
            besti = t;
        }
    }
    red_v[threadIdx.x] = best;
    red_i[threadIdx.x] = besti;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const float ov = red_v[threadIdx.x + s];
            const int oi = red_i[threadIdx.x + s];
            if (ov > red_v[threadIdx.x] || (ov == red_v[threadIdx.x] && oi < red_i[threadIdx.x])) {
                red_v[threadIdx.x] = ov;
                red_i[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    const float mx = red_v[0];
    const int pos = red_i[0];
    float s = 0.f;
    for (int t = threadIdx.x; t < M * M; t += 256) s += expf(mp[t] - mx);
    red_s[threadIdx.x] = s;
    __syncthreads();
    for (int q = 128; q > 0; q >>= 1) {
        if (threadIdx.x < q) red_s[threadIdx.x] += red_s[threadIdx.x + q];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int xi = pos % OW, yi = pos / OW;
        const float wcor = wdt / wc, hcor = hgt / hc;
        o[0] = ((float)xi + 0.5f) * wcor + x0;
        o[1] = ((float)yi + 0.5f) * hcor + y0;
        o[2] = 1.0f / red_s[0];  // exp(max - max) / sum(exp(maps - max))
    }
}

}  // namespace mdx

using namespace mdx;

static int grid_for(long long total) {
    long long g = (total + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

extern "C" int mdx_preprocess(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], const float *mean,
                              const float *stdv, int C, int Cp, int Hp, int Wp, int dtype, void *out,
                              mdx_stream_t stream) {
    MDX_REQUIRE(frames && lut && mean && stdv && out, "mdx_preprocess: null pointer");
    MDX_REQUIRE(C >= 1 && C <= 4 && Cp >= C && Cp <= 8 && Hp >= h && Wp >= w, "mdx_preprocess: bad shape");
    MDX_REQUIRE((long long)B * Hp * Wp < (1ll << 31), "mdx_preprocess: too many pixels");
    PrepArgs pa;
    for (int i = 0; i < 256; ++i) pa.lut[i] = lut[i];
    for (int c = 0; c < 4; ++c) {
        pa.mean[c] = c < C ? mean[c] : 0.f;
        pa.stdv[c] = c < C ? stdv[c] : 1.f;
    }
    const long long total = (long long)B * Hp * Wp;
    if (dtype == 1)
        hipLaunchKernelGGL(k_preprocess<_Float16>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), frames, B,
                           h, w, C, Cp, Hp, Wp, pa, (_Float16 *)out);
    else
        hipLaunchKernelGGL(k_preprocess<float>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), frames, B, h,
                           w, C, Cp, Hp, Wp, pa, (float *)out);
    MDX_CHECK_LAUNCH("mdx_preprocess");
    return MDX_OK;
}

extern "C" int mdx_preprocess_s2d(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], const float *mean,
                                  const float *stdv, int C, int Hp, int Wp, int dtype, void *out, mdx_stream_t stream) {
    MDX_REQUIRE(frames && lut && mean && stdv && out, "mdx_preprocess_s2d: null pointer");
    MDX_REQUIRE(C >= 1 && C <= 4 && Hp >= h && Wp >= w && Hp % 2 == 0 && Wp % 2 == 0,
                "mdx_preprocess_s2d: bad shape (C <= 4, even Hp, Wp)");
    const int Hs = Hp / 2 + 1, Ws = Wp / 2 + 1;
    MDX_REQUIRE((long long)B * Hs * Ws * 16 < (1ll << 31), "mdx_preprocess_s2d: too many pixels");
    PrepArgs pa;
    for (int i = 0; i < 256; ++i) pa.lut[i] = lut[i];
    for (int c = 0; c < 4; ++c) {
        pa.mean[c] = c < C ? mean[c] : 0.f;
        pa.stdv[c] = c < C ? stdv[c] : 1.f;
    }
    const long long total = (long long)B * Hs * Ws;
    if (dtype == 1)
        hipLaunchKernelGGL(k_preprocess_s2d<_Float16>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), frames,
                           B, h, w, C, Hs, Ws, pa, (_Float16 *)out);
    else
        hipLaunchKernelGGL(k_preprocess_s2d<float>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), frames, B,
                           h, w, C, Hs, Ws, pa, (float *)out);
    MDX_CHECK_LAUNCH("mdx_preprocess_s2d");
    return MDX_OK;
}

extern "C" int mdx_preprocess_s2d_folded(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], int Hp,
                                         int Wp, int dtype, void *out, mdx_stream_t stream) {
    MDX_REQUIRE(frames && lut && out, "mdx_preprocess_s2d_folded: null pointer");
    MDX_REQUIRE(Hp >= h && Wp >= w && Hp % 2 == 0 && Wp % 2 == 0, "mdx_preprocess_s2d_folded: bad shape (even Hp, Wp)");
    const int Hs = Hp / 2 + 1, Ws = Wp / 2 + 1;
    MDX_REQUIRE((long long)B * Hs * Ws * 8 < (1ll << 31), "mdx_preprocess_s2d_folded: too many pixels");
    PrepArgs pa;
    for (int i = 0; i < 256; ++i) pa.lut[i] = lut[i];
    for (int c = 0; c < 4; ++c) {
        pa.mean[c] = 0.f;
        pa.stdv[c] = 1.f;
    }
    const long long total = (long long)B * Hs * Ws;
    if (dtype == 1)
        hipLaunchKernelGGL((k_preprocess_s2d<_Float16, true>), dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                           frames, B, h, w, 1, Hs, Ws, pa, (_Float16 *)out);
    else
        hipLaunchKernelGGL((k_preprocess_s2d<float, true>), dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                           frames, B, h, w, 1, Hs, Ws, pa, (float *)out);
    MDX_CHECK_LAUNCH("mdx_preprocess_s2d_folded");
    return MDX_OK;
}

extern "C" int mdx_maxpool2d(const void *x, int N, int H, int W, int C, int k, int s, int p, int dtype, void *out,
                             mdx_stream_t stream) {
    MDX_REQUIRE(x && out && k > 0 && s > 0 && p >= 0 && C % 8 == 0, "mdx_maxpool2d: bad args (C % 8 == 0)");
    MDX_REQUIRE((long long)N * H * W * C < (1ll << 31), "mdx_maxpool2d: tensor too large");
    const int OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
    const long long total = (long long)N * OH * OW * (C / 8);
    if (dtype == 1)
        hipLaunchKernelGGL(k_maxpool<_Float16>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                           (const _Float16 *)x, N, H, W, C, k, s, p, OH, OW, (_Float16 *)out);
    else
        hipLaunchKernelGGL(k_maxpool<float>, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), (const float *)x,
                           N, H, W, C, k, s, p, OH, OW, (float *)out);
    MDX_CHECK_LAUNCH("mdx_maxpool2d");
    return MDX_OK;
}

extern "C" int64_t mdx_groupnorm_workspace_bytes(int N, int H, int W, int G) {
    const long long nch = ((long long)H * W + GN_CHUNK_PIX - 1) / GN_CHUNK_PIX;
    return (long long)N * G * 2 * 4 + (long long)N * G * nch * 3 * 4 + 64;
}

extern "C" int mdx_convert(const void *x, int64_t n, int in_dtype, void *out, int out_dtype, mdx_stream_t stream) {
    MDX_REQUIRE(x && out && n >= 0 && n % 8 == 0, "mdx_convert: null pointer or n not a multiple of 8");
    MDX_REQUIRE((in_dtype == 0 || in_dtype == 1) && (out_dtype == 0 || out_dtype == 1), "mdx_convert: bad dtype");
    if (n == 0) return MDX_OK;
    const unsigned grid = (unsigned)std::min<long long>((n / 8 + 255) / 256, 8192);
    hipStream_t s = as_stream(stream);
    if (in_dtype == 0 && out_dtype == 1)
        hipLaunchKernelGGL((k_convert<float, _Float16>), dim3(grid), dim3(256), 0, s, (const float *)x, n / 8,
                           (_Float16 *)out);
    else if (in_dtype == 1 && out_dtype == 0)
        hipLaunchKernelGGL((k_convert<_Float16, float>), dim3(grid), dim3(256), 0, s, (const _Float16 *)x, n / 8,
                           (float *)out);
    else
        MDX_HIP(hipMemcpyAsync(out, x, (size_t)n * (in_dtype == 1 ? 2 : 4), hipMemcpyDeviceToDevice, s));
    MDX_CHECK_LAUNCH("mdx_convert");
    return MDX_OK;
}

extern "C" int mdx_groupnorm(const void *x, int N, int H, int W, int C, int G, float eps, const float *gamma,
                             const float *beta, const void *up, int fuse, int dtype, void *out, float *workspace,
                             mdx_stream_t stream) {
    MDX_REQUIRE(x && out && gamma && beta && workspace && G > 0 && C % G == 0, "mdx_groupnorm: bad args");
    MDX_REQUIRE(!fuse || (up && H % 2 == 0 && W % 2 == 0), "mdx_groupnorm: fuse needs up and even H, W");
    MDX_REQUIRE(C % 8 == 0 && (C / G) % 8 == 0 && C / 8 <= 256 && G <= 256,
                "mdx_groupnorm: C and C/G must be multiples of 8, C <= 2048");
    MDX_REQUIRE((long long)N * H * W * C < (1ll << 31), "mdx_groupnorm: tensor too large");
    hipStream_t s = as_stream(stream);
    const int HW = H * W;
    const int nch = (HW + GN_CHUNK_PIX - 1) / GN_CHUNK_PIX;
    float *stats = workspace;
    float *part = workspace + 2 * N * G;
    const long long total = (long long)N * H * W * C;
    if (dtype == 1) {
        hipLaunchKernelGGL(k_gn_partial<_Float16>, dim3(nch, N), dim3(256), 0, s, (const _Float16 *)x, HW, C, G, part);
        hipLaunchKernelGGL(k_gn_final, dim3((N * G + 3) / 4), dim3(256), 0, s, part, N * G, nch, eps, stats);
        hipLaunchKernelGGL(k_gn_apply<_Float16>, dim3(grid_for(total / 8)), dim3(256), 0, s, (const _Float16 *)x, N, H,
                           W, C, G, stats, gamma, beta, (const _Float16 *)up, fuse, (_Float16 *)out);
    } else {
        hipLaunchKernelGGL(k_gn_partial<float>, dim3(nch, N), dim3(256), 0, s, (const float *)x, HW, C, G, part);
        hipLaunchKernelGGL(k_gn_final, dim3((N * G + 3) / 4), dim3(256), 0, s, part, N * G, nch, eps, stats);
        hipLaunchKernelGGL(k_gn_apply<float>, dim3(grid_for(total / 8)), dim3(256), 0, s, (const float *)x, N, H, W, C,
                           G, stats, gamma, beta, (const float *)up, fuse, (float *)out);
    }
    MDX_CHECK_LAUNCH("mdx_groupnorm");
    return MDX_OK;
}

extern "C" int64_t mdx_rpn_workspace_bytes(int B, int L, int pre_topk) {
    const long long segs = (long long)B * L;
    const long long words = (pre_topk + 63) / 64;
    return segs * pre_topk * (16 + 4 + 4 + 4) + segs * 4 + segs * pre_topk * words * 8 + 256 +
           segs * RPN_SLICES * pre_topk * 8 + segs * RPN_SLICES * 4 + 64;  // sliced top-k candidates
}

// RPN top-k: several workgroups per (image, level) (1, default) or one (0)

extern "C" int mdx_rpn_proposals(const float *const *head, const int *lvl_h, const int *lvl_w, const int *strides,
                                 int L, int B, int A, const float *cell_anchors, float offset, int img_h, int img_w,
                                 int pre_topk, int post_topk, float nms_thresh, float min_size, float clampv,
                                 const float *reg_weights, float *out_boxes, float *out_scores, int *out_count,
                                 void *workspace, mdx_stream_t stream) {
    MDX_REQUIRE(head && lvl_h && lvl_w && strides && cell_anchors && out_boxes && out_scores && out_count && workspace,
                "mdx_rpn_proposals: null pointer");
    MDX_REQUIRE(L >= 1 && L <= MAX_LEVELS && A >= 1 && A <= 8, "mdx_rpn_proposals: L or A out of range");
    MDX_REQUIRE(pre_topk >= 1 && pre_topk <= TOPK_MAX && (pre_topk + 63) / 64 <= NMS_MAXW,
                "mdx_rpn_proposals: pre_topk must be in [1, %d]", TOPK_MAX);
    MDX_REQUIRE(post_topk >= 1 && L * pre_topk <= MERGE_MAX, "mdx_rpn_proposals: too many candidates to merge");
    RpnLevels rl{};
    for (int l = 0; l < L; ++l) {
        rl.head[l] = head[l];
        rl.H[l] = lvl_h[l];
        rl.W[l] = lvl_w[l];
        rl.stride[l] = strides[l];
        for (int a = 0; a < A; ++a)
            for (int c = 0; c < 4; ++c) rl.cell[l][a][c] = cell_anchors[(l * A + a) * 4 + c];
    }
    for (int c = 0; c < 4; ++c) rl.wts[c] = reg_weights ? reg_weights[c] : 1.f;
    rl.L = L; rl.A = A; rl.B = B; rl.pre_topk = pre_topk;
    rl.offset = offset; rl.img_h = (float)img_h; rl.img_w = (float)img_w; rl.min_size = min_size; rl.clampv = clampv;
    const long long segs = (long long)B * L;
    const int words = (pre_topk + 63) / 64;
    char *ws = (char *)workspace;
    float *wb = (float *)ws; ws += segs * pre_topk * 16;
    float *wsc = (float *)ws; ws += segs * pre_topk * 4;
    int *wv = (int *)ws; ws += segs * pre_topk * 4;
    int *wkeep = (int *)ws; ws += segs * pre_topk * 4;
    int *wk = (int *)ws; ws += segs * 4;
    ws = (char *)(((uintptr_t)ws + 15) & ~(uintptr_t)15);
    unsigned long long *wmask = (unsigned long long *)ws;
    ws += segs * pre_topk * words * 8;
    ws = (char *)(((uintptr_t)ws + 15) & ~(uintptr_t)15);
    unsigned long long *wcand = (unsigned long long *)ws;
    ws += segs * RPN_SLICES * pre_topk * 8;
    int *wccount = (int *)ws;
    hipStream_t s = as_stream(stream);
    int nmax = 0;
    for (int l = 0; l < L; ++l) nmax = std::max(nmax, lvl_h[l] * lvl_w[l] * A);
    if (pol().rpn_sliced && nmax <= RPN_SLICES * PART_KPT * TOPK_THREADS) {
        hipLaunchKernelGGL(k_rpn_part, dim3(RPN_SLICES, (unsigned)segs), dim3(TOPK_THREADS), 0, s, rl, wcand, wccount);
        hipLaunchKernelGGL(k_rpn_merge_topk, dim3((unsigned)segs), dim3(TOPK_THREADS), 0, s, rl, wcand, wccount, wb, wsc,
                           wv, wk);
    } else {
        hipLaunchKernelGGL(k_rpn_topk, dim3((unsigned)segs), dim3(TOPK_THREADS), 0, s, rl, wb, wsc, wv, wk);
    }
    hipLaunchKernelGGL(k_nms_mask, dim3(words, (pre_topk + 255) / 256, (unsigned)segs), dim3(256), 0, s, wb, wk,
                       pre_topk, words, nms_thresh, wmask);
    hipLaunchKernelGGL(k_nms_scan, dim3((unsigned)segs), dim3(NMS_THREADS), (size_t)pre_topk * words * 8, s, wv, wk,
                       pre_topk, words, wmask, wkeep);
    hipLaunchKernelGGL(k_rpn_merge, dim3(B), dim3(1024), 2 * MERGE_MAX * sizeof(unsigned), s, wb, wsc, wkeep, wk, L,
                       pre_topk, post_topk, out_boxes, out_scores, out_count);
    MDX_CHECK_LAUNCH("mdx_rpn_proposals");
    return MDX_OK;
}

extern "C" int mdx_roi_align(const void *const *feats, const int *fh, const int *fw, const float *scales, int L,
                             int min_level, int C, const float *rois, const int *counts, int R, int per_image, int P,
                             int sampling, int aligned, float canonical_size, float canonical_level, int dtype,
                             void *out, mdx_stream_t stream) {
    return mdx_roi_align_ex(feats, fh, fw, scales, L, min_level, C, rois, counts, R, per_image, P, sampling, aligned,
                            canonical_size, canonical_level, dtype, nullptr, out, stream);
}

extern "C" int mdx_roi_align_ex(const void *const *feats, const int *fh, const int *fw, const float *scales, int L,
                                int min_level, int C, const float *rois, const int *counts, int R, int per_image,
                                int P, int sampling, int aligned, float canonical_size, float canonical_level,
                                int dtype, int *order_ws, void *out, mdx_stream_t stream) {
    MDX_REQUIRE(feats && fh && fw && scales && rois && counts && out, "mdx_roi_align: null pointer");
    MDX_REQUIRE(L >= 1 && L <= MAX_LEVELS && per_image > 0 && R % per_image == 0, "mdx_roi_align: bad args");
    const int vch = dtype == 1 ? 8 : 4;  // channels per 16 B
    MDX_REQUIRE(C % vch == 0, "mdx_roi_align: C must be a multiple of 16 bytes of channels");
    if (R == 0) return MDX_OK;
    // channel slice of up to 128 B (8 groups of 16 B) that divides C
    int gslice = 8;
    while (gslice > 1 && (C / vch) % gslice) gslice >>= 1;
    RoiLevels rl{};
    for (int l = 0; l < L; ++l) {
        rl.feat[l] = feats[l];
        rl.H[l] = fh[l];
        rl.W[l] = fw[l];
        rl.scale[l] = scales[l];
    }
    rl.L = L; rl.min_level = min_level; rl.C = C; rl.P = P; rl.sampling = sampling; rl.aligned = aligned;
    rl.per_image = per_image; rl.canonical_size = canonical_size; rl.canonical_level = canonical_level;
    rl.xcd_remap = pol().roi_xcd_order;
    rl.order = nullptr;
    // dtype 2: fp32 features, output rows as bf16 planes (mdx_split_x6 layout,
    // the A operand of mdx_gemm_x6); separable kernels only
    rl.planes = dtype == 2;
    MDX_REQUIRE(dtype != 2 || ((pol().roi_mode >= 4 && pol().roi_mode <= 7) && P <= ROI_PMAX && (P * P * C) % 16 == 0),
                "mdx_roi_align: plane output (dtype 2) needs the separable kernel and P*P*C %% 16 == 0");
    if (order_ws && pol().roi_sorted) {
        hipLaunchKernelGGL(k_roi_order, dim3(R / per_image), dim3(256), 0, as_stream(stream), rl, rois, counts,
                           order_ws);
        rl.order = order_ws;
    }
    if (((pol().roi_mode == 6 && R >= 1024) || pol().roi_mode == 7) && P <= ROI_PMAX) {
        // the box pooler (mode 6; 7: any ROI count, tests): each ROI's sample
        // window staged in LDS per channel slice
        if (dtype == 1)
            hipLaunchKernelGGL((k_roi_align_sep<_Float16, false, true>), dim3(R), dim3(256), 0, as_stream(stream), rl,
                               rois, counts, (_Float16 *)out);
        else
            hipLaunchKernelGGL((k_roi_align_sep<float, false, true>), dim3(R), dim3(256), 0, as_stream(stream), rl,
                               rois, counts, (float *)out);
    } else if (pol().roi_mode == 5 && P <= ROI_PMAX) {
        if (dtype == 1)
            hipLaunchKernelGGL((k_roi_align_sep<_Float16, true>), dim3(R), dim3(256), 0, as_stream(stream), rl, rois,
                               counts, (_Float16 *)out);
        else
            hipLaunchKernelGGL((k_roi_align_sep<float, true>), dim3(R), dim3(256), 0, as_stream(stream), rl, rois,
                               counts, (float *)out);
    } else if ((pol().roi_mode == 4 || pol().roi_mode == 6) && P <= ROI_PMAX) {
        // few ROIs (mask / keypoint heads: B x D): split each ROI's items over
        // up to 4 workgroups so the grid covers the CUs
        const int split = R >= 1024 ? 1 : (R >= 512 ? 2 : 4);
        if (dtype == 1)
            hipLaunchKernelGGL(k_roi_align_sep<_Float16>, dim3(R, split), dim3(256), 0, as_stream(stream), rl, rois,
                               counts, (_Float16 *)out);
        else
            hipLaunchKernelGGL(k_roi_align_sep<float>, dim3(R, split), dim3(256), 0, as_stream(stream), rl, rois,
                               counts, (float *)out);
    } else if (pol().roi_mode >= 1 && pol().roi_mode <= 4) {
#define MDX_ROI_FULL(NI_)                                                                                     \
    do {                                                                                                      \
        if (dtype == 1)                                                                                       \
            hipLaunchKernelGGL((k_roi_align_full<_Float16, NI_>), dim3(R), dim3(256), 0, as_stream(stream), rl, \
                               rois, counts, (_Float16 *)out);                                                \
        else                                                                                                  \
            hipLaunchKernelGGL((k_roi_align_full<float, NI_>), dim3(R), dim3(256), 0, as_stream(stream), rl,    \
                               rois, counts, (float *)out);                                                   \
    } while (0)
        if (pol().roi_mode == 1)
            MDX_ROI_FULL(1);
        else if (pol().roi_mode == 2)
            MDX_ROI_FULL(2);
        else
            MDX_ROI_FULL(4);
#undef MDX_ROI_FULL
    } else if (dtype == 1)
        hipLaunchKernelGGL(k_roi_align<_Float16>, dim3(R, C / (gslice * vch)), dim3(256), 0, as_stream(stream), rl,
                           rois, counts, gslice, (_Float16 *)out);
    else
        hipLaunchKernelGGL(k_roi_align<float>, dim3(R, C / (gslice * vch)), dim3(256), 0, as_stream(stream), rl, rois,
                           counts, gslice, (float *)out);
    MDX_CHECK_LAUNCH("mdx_roi_align");
    return MDX_OK;
}

extern "C" int mdx_box_postprocess(const float *pred, int ld_pred, const float *proposals, const int *counts, int B,
                                   int R, int D, float score_thresh, float nms_thresh, int img_h, int img_w,
                                   const float *reg_weights, float clampv, float *det_boxes, float *det_scores,
                                   int64_t *det_classes, int *ndet, mdx_stream_t stream) {
    MDX_REQUIRE(pred && proposals && counts && det_boxes && det_scores && det_classes && ndet && reg_weights,
                "mdx_box_postprocess: null pointer");
    MDX_REQUIRE(R >= 1 && R <= 1024 && D >= 1 && D <= 16 && ld_pred >= 6, "mdx_box_postprocess: R<=1024, D<=16");
    BoxPostArgs ba{};
    ba.R = R; ba.ld_pred = ld_pred; ba.D = D; ba.score_thresh = score_thresh; ba.nms_thresh = nms_thresh;
    ba.img_h = (float)img_h; ba.img_w = (float)img_w; ba.clampv = clampv;
    for (int i = 0; i < 4; ++i) ba.wts[i] = reg_weights[i];
    hipLaunchKernelGGL(k_box_post, dim3(B), dim3(1024), 0, as_stream(stream), ba, pred, proposals, counts, det_boxes,
                       det_scores, (long long *)det_classes, ndet);
    MDX_CHECK_LAUNCH("mdx_box_postprocess");
    return MDX_OK;
}

extern "C" int mdx_paste_masks(const float *logits, const float *boxes, const int *counts, int B, int D, int M,
                               int img_h, int img_w, int64_t plane_stride, float thresh, uint8_t *out,
                               mdx_stream_t stream) {
    MDX_REQUIRE(logits && boxes && counts && out && M <= 64, "mdx_paste_masks: bad args");
    MDX_REQUIRE(plane_stride >= (int64_t)img_h * img_w, "mdx_paste_masks: plane_stride < img_h*img_w");
    dim3 grid((img_h + 7) / 8, B * D);
    hipLaunchKernelGGL(k_paste, grid, dim3(256), 0, as_stream(stream), logits, boxes, counts, D, M, img_h, img_w,
                       (long long)plane_stride, thresh, out);
    MDX_CHECK_LAUNCH("mdx_paste_masks");
    return MDX_OK;
}

extern "C" int mdx_deconv_col2im(const float *y, const float *bias, int R, int Hi, int Wi, int Co, float *out,
                                 mdx_stream_t stream) {
    MDX_REQUIRE(y && out, "mdx_deconv_col2im: null pointer");
    if (R == 0) return MDX_OK;
    const long long total = (long long)R * Co * 4 * Hi * Wi;
    hipLaunchKernelGGL(k_deconv_col2im, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), y, bias, R, Hi, Wi,
                       Co, out);
    MDX_CHECK_LAUNCH("mdx_deconv_col2im");
    return MDX_OK;
}

extern "C" int mdx_upsample_bilinear2x(const float *x, int NC, int H, int W, float *out, mdx_stream_t stream) {
    MDX_REQUIRE(x && out, "mdx_upsample_bilinear2x: null pointer");
    const long long total = (long long)NC * 4 * H * W;
    hipLaunchKernelGGL(k_upsample2x, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x, NC, H, W, out);
    MDX_CHECK_LAUNCH("mdx_upsample_bilinear2x");
    return MDX_OK;
}

extern "C" int mdx_heatmaps_to_keypoints(const float *maps, const float *boxes, const int *counts, int B, int D,
                                         int K, int M, float *out, mdx_stream_t stream) {
    MDX_REQUIRE(maps && boxes && counts && out, "mdx_heatmaps_to_keypoints: null pointer");
    hipLaunchKernelGGL(k_heatmap_kp, dim3(B * D * K), dim3(256), 0, as_stream(stream), maps, boxes, counts, D, K, M,
                       out);
    MDX_CHECK_LAUNCH("mdx_heatmaps_to_keypoints");
    return MDX_OK;
}
