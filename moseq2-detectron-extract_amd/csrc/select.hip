// Instance selection after inference (gfx950):
//   ProcessFeaturesStep.__nms_mask_instances   M/pipeline/process_features_step.py:63-113
//   mask_and_keypoints_from_model_output (instance 0)  M/proc/proc.py:657-685
//
// One workgroup per frame.  Areas and pairwise intersections of the <= D
// pasted masks are popcount reductions over the frame; the reference's
// sequential pick loop (including its quirk: every row index with ANY later
// IoU > thr is deleted, plus `last`) then runs on one lane.  The selected
// instance 0's mask and keypoints are written out for the frame-feature stage.
#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

constexpr int SEL_MAXD = 8, SEL_THREADS = 1024;

// DM: compile-time bound on the detections per frame, so the per-lane mask
// words and pair counters are indexed statically and stay in registers
template <int DM>
__global__ __launch_bounds__(SEL_THREADS) void k_mask_nms_select(const uint8_t *__restrict__ masks,
                                                                 const float *__restrict__ scores,
                                                                 const int *__restrict__ ndet,
                                                                 const float *__restrict__ kpts, int D, int K,
                                                                 long long hw, long long plane, float thr,
                                                                 int *__restrict__ keep_idx, int *__restrict__ nkeep,
                                                                 uint8_t *__restrict__ sel_mask,
                                                                 double *__restrict__ sel_kpts) {
    __shared__ unsigned long long s_cnt[SEL_MAXD * SEL_MAXD];
    __shared__ int s_sel;
    const int b = blockIdx.x;
    const int n = min(max(ndet[b], 0), min(D, DM));  // (a count never addresses past the planes)
    const uint8_t *mb = masks + (long long)b * D * plane;
    for (int i = threadIdx.x; i < SEL_MAXD * SEL_MAXD; i += SEL_THREADS) s_cnt[i] = 0;
    __syncthreads();
    if (n > 1) {
        // cnt[i][j] (j >= i): |m_i & m_j| ; cnt[i][i] = area_i.  Mask bytes are
        // 0/1, so the popcount of the AND of 16-byte words counts pixels.
        constexpr int NP = DM * (DM + 1) / 2;
        unsigned loc[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) loc[q] = 0;
        const long long nv = (plane % 16 == 0) ? hw / 16 : 0;
        for (long long v = threadIdx.x; v < nv; v += SEL_THREADS) {
            uint4 w[DM];
#pragma unroll
            for (int i = 0; i < DM; ++i)
                w[i] = i < n ? reinterpret_cast<const uint4 *>(mb + (long long)i * plane)[v] : make_uint4(0, 0, 0, 0);
            int q = 0;
#pragma unroll
            for (int i = 0; i < DM; ++i)
#pragma unroll
                for (int j = i; j < DM; ++j, ++q)
                    loc[q] += __popc(w[i].x & w[j].x) + __popc(w[i].y & w[j].y) + __popc(w[i].z & w[j].z) +
                              __popc(w[i].w & w[j].w);
        }
        for (long long p = nv * 16 + threadIdx.x; p < hw; p += SEL_THREADS) {
            unsigned m[DM];
#pragma unroll
            for (int i = 0; i < DM; ++i) m[i] = i < n ? (mb[(long long)i * plane + p] != 0) : 0u;
            int q = 0;
#pragma unroll
            for (int i = 0; i < DM; ++i)
#pragma unroll
                for (int j = i; j < DM; ++j, ++q) loc[q] += m[i] & m[j];
        }
        // wave reduction, then one LDS atomic per wave and pair
        int q = 0;
#pragma unroll
        for (int i = 0; i < DM; ++i)
#pragma unroll
            for (int j = i; j < DM; ++j, ++q) {
                unsigned v = loc[q];
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
                if ((threadIdx.x & 63) == 0 && i < n && j < n) atomicAdd(&s_cnt[i * SEL_MAXD + j], (unsigned long long)v);
            }
    }
    __syncthreads();
    // the serial decision of thread 0 keeps its run-time indexed arrays in LDS
    // (as private arrays they would live in scratch memory)
    __shared__ int pick[SEL_MAXD], cand[SEL_MAXD], idxs[SEL_MAXD];
    __shared__ bool del[SEL_MAXD];
    if (threadIdx.x == 0) {
        int np = 0;
        if (n <= 1) {
            for (int i = 0; i < n; ++i) pick[np++] = i;
        } else {
            // drop instances with an empty mask
            int nc = 0;
            for (int i = 0; i < n; ++i)
                if (s_cnt[i * SEL_MAXD + i] > 0) cand[nc++] = i;
            // idxs = argsort(scores) ascending (stable for these sizes)
            for (int i = 0; i < nc; ++i) idxs[i] = cand[i];
            for (int i = 1; i < nc; ++i) {
                const int v = idxs[i];
                int j = i - 1;
                while (j >= 0 && scores[b * D + idxs[j]] > scores[b * D + v]) {
                    idxs[j + 1] = idxs[j];
                    --j;
                }
                idxs[j + 1] = v;
            }
            int len = nc;
            while (len > 0) {
                const int last = len - 1;
                pick[np++] = idxs[last];
                for (int r = 0; r < len; ++r) del[r] = (r == last);
                for (int r = 0; r < len; ++r) {
                    for (int c = r + 1; c < len; ++c) {
                        const int a = idxs[r], bb = idxs[c];
                        const int lo = a < bb ? a : bb, hi = a < bb ? bb : a;
                        const long long inter = (long long)s_cnt[lo * SEL_MAXD + hi];
                        const long long uni = (long long)s_cnt[a * SEL_MAXD + a] + (long long)s_cnt[bb * SEL_MAXD + bb] -
                                              inter;
                        const float iou = (float)inter / (float)uni;
                        if (iou > thr) del[r] = true;
                    }
                }
                int nl = 0;
                for (int r = 0; r < len; ++r)
                    if (!del[r]) idxs[nl++] = idxs[r];
                len = nl;
            }
        }
        for (int i = 0; i < D; ++i) keep_idx[b * D + i] = i < np ? pick[i] : -1;
        nkeep[b] = np;
        s_sel = np > 0 ? pick[0] : -1;
        const double nan = __builtin_nan("");
        for (int k = 0; k < K; ++k)
            for (int c = 0; c < 3; ++c)
                sel_kpts[((long long)b * K + k) * 3 + c] =
                    np > 0 ? (double)kpts[(((long long)b * D + pick[0]) * K + k) * 3 + c] : nan;
    }
    __syncthreads();
    const int s = s_sel;
    uint8_t *o = sel_mask + (long long)b * hw;
    const uint8_t *src = s >= 0 ? mb + (long long)s * plane : nullptr;
    long long p0 = 0;
    if (((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        const long long nv = hw / 16;
        for (long long v = threadIdx.x; v < nv; v += SEL_THREADS)
            reinterpret_cast<uint4 *>(o)[v] = src ? reinterpret_cast<const uint4 *>(src)[v] : make_uint4(0, 0, 0, 0);
        p0 = nv * 16;
    }
    for (long long p = p0 + threadIdx.x; p < hw; p += SEL_THREADS) o[p] = src ? src[p] : (uint8_t)0;
}

// Centres of the kept detections for the instance tracker
// (ProcessFeaturesStep.__instances_to_detections, process_features_step.py:
// 116-130): scipy.ndimage.center_of_mass of each kept mask = (sum rows / area,
// sum cols / area) -- integer sums, so the fp64 quotients are exact -- and the
// box centre (x, y) when the mask is empty (the reference's fallback, in its
// (x, y) order).  One workgroup per (frame, kept slot).  Mask bytes are 0/1:
// a 16-B word at plane offset p holds pixels p..p+15, i.e. row p / w from
// column p % w, wrapping onto the next row at most once when w >= 16, so its
// three sums come from per-dword popcounts and byte-index sums, without a
// per-pixel division.
constexpr int CEN_THREADS = 512, CEN_UNROLL = 4;

__device__ __forceinline__ unsigned byte_index_sum(unsigned d, unsigned base) {
    // sum over the 0/1 bytes of d of (base + byte index)
    const unsigned b0 = d & 1u, b1 = (d >> 8) & 1u, b2 = (d >> 16) & 1u, b3 = d >> 24;
    return base * (b0 + b1 + b2 + b3) + b1 + 2u * b2 + 3u * b3;
}

__global__ __launch_bounds__(CEN_THREADS) void k_mask_centers(const uint8_t *__restrict__ masks, long long plane,
                                                             const int *__restrict__ keep_idx,
                                                             const int *__restrict__ nkeep,
                                                             const float *__restrict__ boxes, int D, int h, int w,
                                                             double *__restrict__ centers) {
    __shared__ unsigned long long s_acc[3][CEN_THREADS / 64];
    const int b = blockIdx.x / D, slot = blockIdx.x % D;
    double *out = centers + ((long long)b * D + slot) * 2;
    const int j = keep_idx[b * D + slot];
    if (slot >= nkeep[b] || j < 0 || j >= D) {
        if (threadIdx.x == 0) out[0] = out[1] = __builtin_nan("");
        return;
    }
    const uint8_t *m = masks + ((long long)b * D + j) * plane;
    const long long hw = (long long)h * w;
    unsigned long long area = 0, sy = 0, sx = 0;
    long long p0 = 0;
    if (w >= 16 && (reinterpret_cast<uintptr_t>(m) & 15) == 0) {
        const int nv = (int)(hw / 16);
        const uint4 *mv = reinterpret_cast<const uint4 *>(m);
        for (int v0 = threadIdx.x; v0 < nv; v0 += CEN_THREADS * CEN_UNROLL) {
            uint4 q[CEN_UNROLL];
#pragma unroll
            for (int u = 0; u < CEN_UNROLL; ++u) {
                const int v = v0 + u * CEN_THREADS;
                q[u] = v < nv ? mv[v] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < CEN_UNROLL; ++u) {
                const int v = v0 + u * CEN_THREADS;
                const unsigned d[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
                unsigned cnt = 0, ks = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    cnt += __popc(d[t]);
                    ks += byte_index_sum(d[t], 4u * t);
                }
                const long long pp = 16LL * v;
                const unsigned y0 = (unsigned)(pp / w), x0 = (unsigned)(pp - (long long)y0 * w);
                unsigned hi = 0;  // pixels of the word that wrapped onto row y0 + 1
                if (x0 + 15u >= (unsigned)w) {
                    const unsigned kk = (unsigned)w - x0;  // first wrapped byte, 1..15
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int sh = (int)kk - 4 * t;
                        const unsigned msk = sh <= 0 ? 0xffffffffu : (sh >= 4 ? 0u : (0xffffffffu << (8 * sh)));
                        hi += __popc(d[t] & msk);
                    }
                }
                area += cnt;
                sx += (unsigned long long)x0 * cnt + ks - (unsigned long long)w * hi;
                sy += (unsigned long long)y0 * cnt + hi;
            }
        }
        p0 = (long long)nv * 16;
    }
    for (long long p = p0 + threadIdx.x; p < hw; p += CEN_THREADS) {  // tail / unaligned
        const unsigned v = m[p] != 0;
        const long long y = p / w;
        area += v;
        sy += v * (unsigned long long)y;
        sx += v * (unsigned long long)(p - y * w);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        area += __shfl_xor(area, off);
        sy += __shfl_xor(sy, off);
        sx += __shfl_xor(sx, off);
    }
    if (lane == 0) {
        s_acc[0][wave] = area;
        s_acc[1][wave] = sy;
        s_acc[2][wave] = sx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, ty = 0, tx = 0;
        for (int q = 0; q < CEN_THREADS / 64; ++q) {
            a += s_acc[0][q];
            ty += s_acc[1][q];
            tx += s_acc[2][q];
        }
        if (a > 0) {
            out[0] = (double)ty / (double)a;
            out[1] = (double)tx / (double)a;
        } else {  // Boxes.get_centers(): float32 (x0 + x1) / 2, (y0 + y1) / 2
            const float *bx = boxes + ((long long)b * D + j) * 4;
            out[0] = (double)((bx[0] + bx[2]) * 0.5f);
            out[1] = (double)((bx[1] + bx[3]) * 0.5f);
        }
    }
}

// Plane gather for the instance-selection fix-up: dst plane dst_idx[i] <-
// the hw bytes at src[i] (a device address; 0 = zero plane).  One launch for
// every changed frame of a chunk instead of a copy per frame.
constexpr int GATH_THREADS = 256;

__global__ __launch_bounds__(GATH_THREADS) void k_gather_planes(const unsigned long long *__restrict__ src,
                                                               const int *__restrict__ dst_idx,
                                                               uint8_t *__restrict__ dst, long long hw) {
    const int i = blockIdx.y;
    const uint8_t *s = reinterpret_cast<const uint8_t *>(src[i]);
    uint8_t *d = dst + (long long)dst_idx[i] * hw;
    const long long step = (long long)gridDim.x * GATH_THREADS;
    for (long long p = (long long)blockIdx.x * GATH_THREADS + threadIdx.x; p < hw; p += step)
        d[p] = s ? s[p] : (uint8_t)0;
}

}  // namespace mdx

using namespace mdx;

extern "C" int mdx_mask_nms_select(const uint8_t *masks, int64_t plane_stride, const float *scores,
                                   const int *ndet, const float *kpts, int B, int D, int K, int h, int w,
                                   float iou_thresh, int *keep_idx, int *nkeep, uint8_t *sel_mask, double *sel_kpts,
                                   mdx_stream_t stream) {
    MDX_REQUIRE(masks && scores && ndet && kpts && keep_idx && nkeep && sel_mask && sel_kpts,
                "mdx_mask_nms_select: null pointer");
    MDX_REQUIRE(D >= 1 && D <= SEL_MAXD, "mdx_mask_nms_select: D must be in [1, %d]", SEL_MAXD);
    const long long hw = (long long)h * w;
    MDX_REQUIRE(plane_stride >= hw, "mdx_mask_nms_select: plane_stride < h*w");
    MDX_REQUIRE(plane_stride % 16 != 0 || ((uintptr_t)masks % 16) == 0, "mdx_mask_nms_select: unaligned masks");
    if (B == 0) return MDX_OK;
    if (D <= 4)
        hipLaunchKernelGGL(k_mask_nms_select<4>, dim3(B), dim3(SEL_THREADS), 0, as_stream(stream), masks, scores, ndet,
                           kpts, D, K, hw, (long long)plane_stride, iou_thresh, keep_idx, nkeep, sel_mask, sel_kpts);
    else
        hipLaunchKernelGGL(k_mask_nms_select<SEL_MAXD>, dim3(B), dim3(SEL_THREADS), 0, as_stream(stream), masks, scores,
                           ndet, kpts, D, K, hw, (long long)plane_stride, iou_thresh, keep_idx, nkeep, sel_mask,
                           sel_kpts);
    MDX_CHECK_LAUNCH("mdx_mask_nms_select");
    return MDX_OK;
}

extern "C" int mdx_mask_centers(const uint8_t *masks, int64_t plane_stride, const int *keep_idx, const int *nkeep,
                                const float *boxes, int B, int D, int h, int w, double *centers,
                                mdx_stream_t stream) {
    MDX_REQUIRE(masks && keep_idx && nkeep && boxes && centers, "mdx_mask_centers: null pointer");
    MDX_REQUIRE(D >= 1 && D <= SEL_MAXD && h > 0 && w > 0, "mdx_mask_centers: bad shape");
    MDX_REQUIRE(plane_stride >= (int64_t)h * w, "mdx_mask_centers: plane_stride < h*w");
    if (B == 0) return MDX_OK;
    hipLaunchKernelGGL(k_mask_centers, dim3(B * D), dim3(CEN_THREADS), 0, as_stream(stream), masks,
                       (long long)plane_stride, keep_idx, nkeep, boxes, D, h, w, centers);
    MDX_CHECK_LAUNCH("mdx_mask_centers");
    return MDX_OK;
}

extern "C" int mdx_gather_planes(const uint64_t *src_ptrs, const int *dst_idx, uint8_t *dst, int64_t plane_bytes,
                                 int n, mdx_stream_t stream) {
    MDX_REQUIRE(src_ptrs && dst_idx && dst, "mdx_gather_planes: null pointer");
    MDX_REQUIRE(plane_bytes > 0 && n >= 0 && n <= 65535, "mdx_gather_planes: bad size");
    if (n == 0) return MDX_OK;
    const long long per = (plane_bytes + GATH_THREADS - 1) / GATH_THREADS;
    const int bx = (int)(per < 64 ? per : 64);
    hipLaunchKernelGGL(k_gather_planes, dim3(bx, n), dim3(GATH_THREADS), 0, as_stream(stream),
                       reinterpret_cast<const unsigned long long *>(src_ptrs), dst_idx, dst, (long long)plane_bytes);
    MDX_CHECK_LAUNCH("mdx_gather_planes");
    return MDX_OK;
}
