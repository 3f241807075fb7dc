// fill_invalid_pixels -> cv2.inpaint(frame, invalid, 3, cv2.INPAINT_NS)
// (M/proc/proc.py:189-210; OpenCV imgproc/inpaint.cpp icvNSInpaintFMM as
// restated in oracle/frameops.c orc_inpaint_ns_one).
//
// Parallel decomposition that is EXACT w.r.t. the serial fast-marching order:
// computing an unknown pixel reads state only within Chebyshev distance
// `range + 1` of it (window taps +-range, gradients +-1, FMM neighbours +-1),
// and writes only the pixel itself.  Unknown pixels are therefore grouped into
// clusters (connected under Chebyshev distance <= R = max(range + 1, 2)); two
// clusters never read each other's changing state, nor share a narrow-band
// pixel.  OpenCV's priority list pops by (T, insertion order); restricted to
// one cluster that order is the order a cluster-local list produces (its
// initial narrow band is pushed in raster order with T = 0, every later push
// has T >= 0.5), so each cluster can be marched independently and the result
// is bit-identical to the serial algorithm.  A cluster of one pixel has a
// closed form: the pixel is filled once, from its window of known pixels, when
// the first of its band neighbours is popped (unless it lies on the image's
// first row or column, which the serial loop never fills).
//
// Workspace: sparse per-frame slots.  A frame's state image ("plane", one
// int16 per padded pixel) is zero = KNOWN everywhere at rest; a call writes
// only the entries of its multi-pixel clusters and their narrow band and
// resets exactly those entries when it is done, so nothing is filled per call.
// The per-unknown tables (pixel list, labels, T, member lists, FIFO/heap
// scratch) hold `cap` pixels per frame (inp_layout); a frame with more unknown
// pixels is done in the one dense slot (int32 plane, tables for every pixel)
// by a single workgroup after the others.
//
//   k_inp_setup   (one workgroup per frame): the frame's unknown pixels as a
//                 bit image in LDS (ranks by word prefix + popcount), cluster
//                 labels by min-label propagation + pointer jumping over the
//                 bits, one-pixel clusters filled in place (their window's
//                 states read from the bits), the multi-pixel clusters' member
//                 lists and plane entries written for the march
//   k_inp_march   (one wave per multi-pixel cluster): local FIFO(band) +
//                 heap(T, seq) FMM with the NS weights (window taps one per
//                 lane, summed in the serial order), pixel values in place
//   k_inp_dense   (one workgroup): the frames over `cap`, one after another,
//                 on the global plane
#include <atomic>
#include <cmath>

#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

constexpr int INP_SETUP_THREADS = 512, INP_DENSE_THREADS = 1024;
constexpr int INP_LDS_MAX = 150 * 1024;  // bit image + word ranks + labels of one frame
#ifndef MDX_INP_MARCH_BLOCKS
#define MDX_INP_MARCH_BLOCKS 64
#endif
#ifndef MDX_INP_MARCH_WAVES
#define MDX_INP_MARCH_WAVES 1
#endif
constexpr int INP_MARCH_BLOCKS = MDX_INP_MARCH_BLOCKS, MARCH_WAVES = MDX_INP_MARCH_WAVES;
constexpr int DENSE_WAVES = INP_DENSE_THREADS / 64, MAX_TAPS = 15 * 15;
constexpr int INP_HDR = 16;        // ints of a slot header
constexpr int INP_GLOBAL = 256;    // bytes of the workspace header
constexpr int INP_MAGIC = 0x4d445049;
constexpr int INP_CAP_MAX = 32764;  // int16 plane: k + 1 and -(k + 2) fit

// plane values (a pixel's state in the serial algorithm's terms):
//   0         KNOWN, never in the band (T = 1e6)
//   -1        the initial narrow band (T = 0)
//   k + 1     unknown pixel k of the slot's list, not yet filled (T = t[k] = 1e6)
//   -(k + 2)  unknown pixel k, filled (T = t[k])
struct SlotOff {
    long long bits, plane, ins, lab, t, ord, cnt, start, fill, scr, bytes;
};

__host__ __device__ inline SlotOff slot_off(long long nw, long long np, int cap, int idx_bytes) {
    SlotOff o;
    long long b = INP_HDR * 4;
    o.bits = b;  // the unknown pixels' bit image (k_prep / k_inp_bits)
    b += (nw * 4 + 15) / 16 * 16;
    o.plane = b;
    b += (np * idx_bytes + 15) / 16 * 16;
    const long long a = (long long)(cap + 4) / 4 * 16;  // one table: cap + 1 ints, 16-B padded
    o.ins = b; b += a;
    o.lab = b; b += a;
    o.t = b; b += a;
    o.ord = b; b += a;
    o.cnt = b; b += a;
    o.start = b; b += a;
    o.fill = b; b += a;
    o.scr = b; b += 7 * a;  // per cluster: band FIFO (<= 4 m) + heap (<= m entries of 3)
    o.bytes = b;
    return o;
}

struct InpLayout {
    int H, W, PH, PW, cap, hw;
    long long np;
    SlotOff s, d;           // a frame's sparse slot (int16 plane), the dense slot (int32 plane)
    long long o_dense, o_slots;
    // k_inp_setup's LDS: bit image (nw words, wpr per padded row), uint16
    // rank of each word's first bit, int16 label per unknown pixel
    int wpr, nw, lds_pref, lds_lab, lds_bytes, lds_ok;
    __host__ __device__ uint32_t *bits(char *ws) const { return reinterpret_cast<uint32_t *>(ws + o_slots + s.bits); }
    __host__ __device__ long long bits_fstride() const { return s.bytes / 4; }  // words
};

static inline InpLayout inp_layout(int H, int W) {
    InpLayout L;
    L.H = H;
    L.W = W;
    L.PH = H + 2;
    L.PW = W + 2;
    L.hw = H * W;
    L.np = (long long)L.PH * L.PW;
    int cap = (L.hw / 24 + 3) / 4 * 4;  // 4.2 % of the frame
    cap = cap < 256 ? 256 : (cap > INP_CAP_MAX ? INP_CAP_MAX : cap);
    if (cap > (L.hw + 3) / 4 * 4) cap = (L.hw + 3) / 4 * 4;
    L.cap = cap;
    L.wpr = (L.PW + 31) / 32;
    const long long nw = (long long)L.PH * L.wpr;
    L.nw = (int)(nw < (1 << 30) ? nw : (1 << 30));
    L.s = slot_off(nw, L.np, L.cap, 2);
    L.d = slot_off(0, L.np, L.hw, 4);
    L.o_dense = INP_GLOBAL;
    L.o_slots = INP_GLOBAL + L.d.bytes;
    L.lds_pref = L.nw * 4;
    L.lds_lab = L.lds_pref + (L.nw * 2 + 15) / 16 * 16;
    const long long lds = (long long)L.lds_lab + (L.cap * 2 + 15) / 16 * 16;
    L.lds_ok = lds <= INP_LDS_MAX;
    L.lds_bytes = L.lds_ok ? (int)lds : 0;
    return L;
}

template <typename Idx>
struct Slot {
    int *hdr, *ins, *lab, *ord, *cnt, *start, *fill, *scr;
    float *t;
    Idx *plane;
};

template <typename Idx>
__device__ __forceinline__ Slot<Idx> slot_view(char *base, const SlotOff &o) {
    Slot<Idx> S;
    S.hdr = reinterpret_cast<int *>(base);
    S.plane = reinterpret_cast<Idx *>(base + o.plane);
    S.ins = reinterpret_cast<int *>(base + o.ins);
    S.lab = reinterpret_cast<int *>(base + o.lab);
    S.t = reinterpret_cast<float *>(base + o.t);
    S.ord = reinterpret_cast<int *>(base + o.ord);
    S.cnt = reinterpret_cast<int *>(base + o.cnt);
    S.start = reinterpret_cast<int *>(base + o.start);
    S.fill = reinterpret_cast<int *>(base + o.fill);
    S.scr = reinterpret_cast<int *>(base + o.scr);
    return S;
}

__device__ __forceinline__ char *frame_slot(char *ws, const InpLayout &L, long long f) {
    return ws + L.o_slots + f * L.s.bytes;
}

__device__ __forceinline__ bool ws_ok(const char *ws, const InpLayout &L) {
    const int *g = reinterpret_cast<const int *>(ws);
    return g[0] == INP_MAGIC && g[1] == L.H && g[2] == L.W;
}

// the invalid mask ORed into each frame's bit image (zero at rest; the
// layout k_prep writes); grid (ceil(H * W / 256), n)
__global__ __launch_bounds__(256) void k_inp_bits(const uint8_t *__restrict__ invalid, char *ws, InpLayout L) {
    if (!ws_ok(ws, L)) return;
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (p >= L.hw || !invalid[f * L.hw + p]) return;
    const int y = (int)(p / L.W), x = (int)(p - (long long)y * L.W);
    atomicOr(L.bits(ws) + f * L.bits_fstride() + (long long)(y + 1) * L.wpr + ((x + 1) >> 5), 1u << ((x + 1) & 31));
}

__global__ void k_inp_header(int *ws, int H, int W) {
    if (threadIdx.x == 0) {
        ws[0] = INP_MAGIC;
        ws[1] = H;
        ws[2] = W;
    }
}

template <typename Idx>
__device__ __forceinline__ float t_of(const Slot<Idx> &S, int p) {
    const int v = S.plane[p];
    return v == 0 ? 1.0e6f : (v == -1 ? 0.0f : S.t[v > 0 ? v - 1 : -v - 2]);
}

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

template <typename Idx>
__device__ __forceinline__ float fm_solve(int i1, int j1, int i2, int j2, const Slot<Idx> &S, int PW) {
    double sol;
    const double a11 = t_of(S, i1 * PW + j1), a22 = t_of(S, i2 * PW + j2);
    const double m12 = a11 < a22 ? a11 : a22;
    const bool in1 = S.plane[i1 * PW + j1] > 0, in2 = S.plane[i2 * PW + j2] > 0;
    if (!in1) {
        if (!in2) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt((double)(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else
            sol = 1 + a11;
    } else if (!in2)
        sol = 1 + a22;
    else
        sol = 1 + m12;
    return (float)sol;
}

__device__ __forceinline__ float min4f(float a, float b, float c, float d) {
    const float x = a < b ? a : b, y = c < d ? c : d;
    return x < y ? x : y;
}

template <int NT>
__device__ __forceinline__ int block_scan_excl(int v, int *sh, int &total) {
    // exclusive prefix sum over an NT-thread block (sh: >= NT ints)
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int o = 1; o < NT; o <<= 1) {
        const int a = tid >= o ? sh[tid - o] : 0;
        __syncthreads();
        sh[tid] += a;
        __syncthreads();
    }
    const int incl = sh[tid];
    total = sh[NT - 1];
    __syncthreads();
    return incl - v;
}

template <int NT>
__device__ __forceinline__ int block_sum(int v, int *sh) {
    int total;
    block_scan_excl<NT>(v, sh, total);
    return total;
}

// back to rest (KNOWN) after the pixel is done: the pixel and its band
template <typename Idx>
__device__ __forceinline__ void rest_pixel(const Slot<Idx> &S, int j, int PW) {
    S.plane[j] = 0;
    const int nb[4] = {j - PW, j - 1, j + 1, j + PW};
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (S.plane[nb[q]] == -1) S.plane[nb[q]] = 0;
}

// frames whose label propagation ended unconverged (see setup_body)
__device__ unsigned int g_inp_errors = 0;

// A march's view of the frame: "is (k, l) an unknown pixel not yet filled"
// (padded coordinates) and the current value of unpadded pixel (r, c).  The
// global plane and frame; the bit image in LDS (one-pixel clusters: nothing in
// their window changes); a cluster's window staged in LDS (WinState).
template <typename Idx>
struct PlaneState {
    const Idx *plane;
    int PW;
    const uint8_t *out;
    int W;
    __device__ __forceinline__ bool unknown(int k, int l) const { return plane[k * PW + l] > 0; }
    __device__ __forceinline__ int px(int r, int c) const { return out[r * W + c]; }
};
struct BitState {
    const uint32_t *bits;
    int wpr;
    const uint8_t *out;
    int W;
    __device__ __forceinline__ bool unknown(int k, int l) const { return (bits[k * wpr + (l >> 5)] >> (l & 31)) & 1u; }
    __device__ __forceinline__ int px(int r, int c) const { return out[r * W + c]; }
};

// One NS window tap (k, l) around the pixel (i, j) being filled: returns the
// weight w and the product w * I exactly as the serial loop forms them (0, 0
// for a tap the loop skips, an exact no-op in its running sums).
template <typename U>
__device__ __forceinline__ void ns_tap(int k, int l, int i, int j, int range, int PH, int PW, const U &u,
                                       float &w_out, float &wi_out) {
    w_out = 0.f;
    wi_out = 0.f;
    const int km = k - 1 + (k == 1), kp = k - 1 - (k == PH - 2);
    const int lm = l - 1 + (l == 1), lp = l - 1 - (l == PW - 2);
    if (!(k > 0 && l > 0 && k < PH - 1 && l < PW - 1)) return;
    if (u.unknown(k, l)) return;
    if ((l - j) * (l - j) + (k - i) * (k - i) > range * range) return;
    const float ry = (float)(k - i), rx = (float)(l - j);
    const float lr = rx * rx + ry * ry;
    const float dst = (float)(1. / (lr * sqrt((double)lr)));
    const bool up_ok = !u.unknown(k - 1, l), dn_ok = !u.unknown(k + 1, l);
    const bool lf_ok = !u.unknown(k, l - 1), rt_ok = !u.unknown(k, l + 1);
    float gx, gy;
    if (dn_ok) {
        if (up_ok)
            gx = (float)(abs(u.px(kp + 1, lm) - u.px(kp, lm)) + abs(u.px(kp, lm) - u.px(km - 1, lm)));
        else
            gx = (float)(abs(u.px(kp + 1, lm) - u.px(kp, lm))) * 2.0f;
    } else {
        if (up_ok)
            gx = (float)(abs(u.px(kp, lm) - u.px(km - 1, lm))) * 2.0f;
        else
            gx = 0;
    }
    if (rt_ok) {
        if (lf_ok)
            gy = -(float)(abs(u.px(km, lp + 1) - u.px(km, lm)) + abs(u.px(km, lm) - u.px(km, lm - 1)));
        else
            gy = -(float)(abs(u.px(km, lp + 1) - u.px(km, lm))) * 2.0f;
    } else {
        if (lf_ok)
            gy = -(float)(abs(u.px(km, lm) - u.px(km, lm - 1))) * 2.0f;
        else
            gy = 0;
    }
    const float dot = rx * gx + ry * gy;
    const float lg = gx * gx + gy * gy;
    float dir = fabsf(dot / sqrtf(lr * lg));
    if (!(dir > 0.01f)) dir = 0.000001f;
    const float w = dst * dir;
    w_out = w;
    wi_out = w * (float)u.px(km, lm);
}

__device__ __forceinline__ uint8_t ns_value(float Ia, float sw) {
    const double v = (double)Ia / sw;
    const int r = __double2int_rn(v);
    return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

// The window of the pixel (i, j) being filled, one tap per lane (up to 4 taps
// a lane for range 7) into the wave's LDS rows tw / twi, summed by lane 0 in
// the serial loop's (k, l) order: the serial loop's float sums (valid in lane
// 0 only).
template <typename U>
__device__ __forceinline__ void wave_tap_sum(const U &u, int i, int j, int range, int PH, int PW, float *tw,
                                             float *twi, float &Ia, float &sw) {
    const int lane = threadIdx.x & 63;
    const int wside = 2 * range + 1, ntaps = wside * wside;
    for (int tp = lane; tp < ntaps; tp += 64)
        ns_tap(i - range + tp / wside, j - range + tp % wside, i, j, range, PH, PW, u, tw[tp], twi[tp]);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    Ia = 0.0f;
    sw = 1.0e-20f;
    if (lane == 0)
        for (int tp = 0; tp < ntaps; ++tp) {
            Ia += twi[tp];
            sw += tw[tp];
        }
}

// a one-pixel cluster at padded (i, j), by one thread: the taps summed in the
// serial order
template <typename U>
__device__ void fill_single(const U &u, int i, int j, uint8_t *out, int H, int W, int range) {
    const int PH = H + 2, PW = W + 2;
    if (i > 1 && j > 1) {  // the serial loop never fills the first row / column
        const int wside = 2 * range + 1, ntaps = wside * wside;
        float Ia = 0.0f, sw = 1.0e-20f;
        for (int tp = 0; tp < ntaps; ++tp) {
            float w, wi;
            ns_tap(i - range + tp / wside, j - range + tp % wside, i, j, range, PH, PW, u, w, wi);
            Ia += wi;
            sw += w;
        }
        out[(i - 1) * W + (j - 1)] = ns_value(Ia, sw);
    }
}

// Per-frame setup on an NT-thread workgroup, the slot's unknown list built
// (nin > 0 entries): narrow band, cluster labels, member lists; one-pixel
// clusters filled and put back to rest; the multi-pixel clusters listed in
// S.fill[0, S.hdr[2]).  Returns their number, or -1 (the frame left
// un-inpainted and its plane at rest) when the labels did not converge.
template <typename Idx, int NT>
__device__ int setup_body(const Slot<Idx> &S, int nin, uint8_t *out, int H, int W, int range,
                           unsigned int *errors) {
    __shared__ int sh[NT];
    __shared__ int s_flag[2], s_bad, s_multi;
    const int tid = threadIdx.x;
    const int PH = H + 2, PW = W + 2;
    // narrow band: interior 4-neighbours of unknown pixels that are not unknown
    for (int k = tid; k < nin; k += NT) {
        const int i = S.ins[k];
        const int nb[4] = {i - PW, i - 1, i + PW, i + 1};
        for (int q = 0; q < 4; ++q) {
            const int p = nb[q];
            const int y = p / PW, x = p - y * PW;
            if (y >= 1 && y < PH - 1 && x >= 1 && x < PW - 1 && S.plane[p] <= 0) S.plane[p] = (Idx)-1;
        }
    }
    // clusters: min-label propagation over Chebyshev distance <= R
    const int R = range + 1 > 2 ? range + 1 : 2;
    // two convergence flags, alternating per iteration: thread 0 clears the
    // NEXT iteration's flag after this iteration's first barrier, when every
    // thread has read it (as the previous iteration's flag) and before any
    // thread can set it.  (One flag cleared at the top of the loop raced with
    // the slower waves' read of the previous iteration's value: a wave that
    // read the cleared flag left the loop alone, its barriers then paired
    // with the other waves' loop barriers, and the label arrays were indexed
    // before they had converged.)
    if (tid == 0) s_flag[0] = s_flag[1] = s_bad = s_multi = 0;
    for (int iter = 0; iter < 1 << 20; ++iter) {
        __syncthreads();
        if (tid == 0) s_flag[(iter + 1) & 1] = 0;
        int changed = 0;
        for (int k = tid; k < nin; k += NT) {
            const int i = S.ins[k];
            const int y = i / PW, x = i - y * PW;
            int m = S.lab[k];
            for (int dy = -R; dy <= R; ++dy) {
                const int yy = y + dy;
                if (yy < 1 || yy > H) continue;
                for (int dx = -R; dx <= R; ++dx) {
                    const int xx = x + dx;
                    if (xx < 1 || xx > W) continue;
                    const int c = S.plane[yy * PW + xx];
                    if (c > 0) {
                        const int l = S.lab[c - 1];
                        m = l < m ? l : m;
                    }
                }
            }
            m = S.lab[m] < m ? S.lab[m] : m;  // pointer jump
            if (m < S.lab[k]) {
                atomicMin(&S.lab[k], m);
                changed = 1;
            }
        }
        if (changed) atomicOr(&s_flag[iter & 1], 1);
        __syncthreads();
        if (!s_flag[iter & 1]) break;
    }
    // converged labels are roots (lab[lab[k]] == lab[k]); the cluster phase
    // below indexes the cluster tables by them, so a frame that left the loop
    // unconverged is counted in g_inp_errors (mdx_inpaint_errors) and left
    // un-inpainted instead of indexing with a stray label.  (Its own flag:
    // a slow wave may still be reading s_flag as it leaves the loop.)
    {
        int bad = 0;
        for (int k = tid; k < nin; k += NT) {
            const int l = S.lab[k];
            bad |= l < 0 || l > k || S.lab[l] != l;
        }
        if (bad) atomicOr(&s_bad, 1);
        __syncthreads();
        if (s_bad) {
            for (int k = tid; k < nin; k += NT) rest_pixel(S, S.ins[k], PW);
            if (tid == 0) {
                S.hdr[1] = S.hdr[2] = 0;
                atomicAdd(&g_inp_errors, 1u);
                if (errors) atomicAdd(errors, 1u);  // the caller's own count (mdx_inpaint_ns_counted)
            }
            return -1;
        }
    }
    // cluster ids for roots (lab[k] == k) in raster order, member counts, starts
    int ncl = 0;
    for (int k0 = 0; k0 < nin; k0 += NT) {
        const int k = k0 + tid;
        const int root = (k < nin && S.lab[k] == k) ? 1 : 0;
        int tot;
        const int pos = ncl + block_scan_excl<NT>(root, sh, tot);
        if (root) {
            S.fill[k] = pos;  // temporarily: root index -> cluster id
            S.cnt[pos] = 0;
        }
        ncl += tot;
    }
    __syncthreads();
    for (int k = tid; k < nin; k += NT) atomicAdd(&S.cnt[S.fill[S.lab[k]]], 1);
    __syncthreads();
    int run = 0;
    for (int c0 = 0; c0 < ncl; c0 += NT) {
        const int c = c0 + tid;
        const int v = c < ncl ? S.cnt[c] : 0;
        int tot;
        const int pos = run + block_scan_excl<NT>(v, sh, tot);
        if (c < ncl) S.start[c] = pos;
        run += tot;
    }
    if (tid == 0) S.start[ncl] = nin;
    __syncthreads();
    // members: cluster id per member, then atomic slot (sorted per cluster later)
    for (int k = tid; k < nin; k += NT) S.lab[k] = S.fill[S.lab[k]];
    __syncthreads();
    for (int c = tid; c < ncl; c += NT) S.cnt[c] = 0;
    __syncthreads();
    for (int k = tid; k < nin; k += NT) {
        const int c = S.lab[k];
        const int slot = atomicAdd(&S.cnt[c], 1);
        S.ord[S.start[c] + slot] = k;
    }
    __syncthreads();
    // one-pixel clusters now; the others listed for the march
    for (int c = tid; c < ncl; c += NT) {
        if (S.start[c + 1] - S.start[c] == 1) {
            const int j = S.ins[S.ord[S.start[c]]];
            fill_single(PlaneState<Idx>{S.plane, PW, out, W}, j / PW, j - j / PW * PW, out, H, W, range);
            rest_pixel(S, j, PW);
        } else
            S.fill[atomicAdd(&s_multi, 1)] = c;
    }
    __syncthreads();
    const int nmulti = s_multi;
    if (tid == 0) {
        S.hdr[1] = ncl;
        S.hdr[2] = nmulti;
    }
    return nmulti;
}

// bits [xa, xb] of padded row y of the bit image (xb - xa < 32), bit 0 = xa
__device__ __forceinline__ uint32_t row_span(const uint32_t *bits, int wpr, int y, int xa, int xb) {
    const uint32_t *r = bits + y * wpr;
    const int w0 = xa >> 5, w1 = xb >> 5;
    uint64_t v = r[w0];
    if (w1 != w0) v |= (uint64_t)r[w1] << 32;
    v >>= (xa & 31);
    const int n = xb - xa + 1;
    return (uint32_t)(v & (n >= 32 ? 0xffffffffull : ((1ull << n) - 1)));
}

// list index (raster order) of the unknown pixel at padded (y, x)
__device__ __forceinline__ int bit_rank(const uint32_t *bits, const uint16_t *pref, int wpr, int y, int x) {
    const int w = y * wpr + (x >> 5);
    return pref[w] + __popc(bits[w] & ((1u << (x & 31)) - 1u));
}

// another unknown pixel within Chebyshev distance R of padded (y, x)
__device__ __forceinline__ bool has_other(const uint32_t *bits, int wpr, int y, int x, int R, int H, int W) {
    const int xa = x - R > 1 ? x - R : 1, xe = x + R < W ? x + R : W;
    const int ya = y - R > 1 ? y - R : 1, ye = y + R < H ? y + R : H;
    for (int yy = ya; yy <= ye; ++yy) {
        uint32_t sp = row_span(bits, wpr, yy, xa, xe);
        if (yy == y) sp &= ~(1u << (x - xa));
        if (sp) return true;
    }
    return false;
}

// fill_single for a compile-time radius on the bit image: the (2R+3)^2 pixel
// box and the (2R+3)^2 state bits around the pixel loaded once into registers
// (every load issued up front), the taps unrolled with the serial loop's
// arithmetic (weights of taps the serial loop skips are 0: exact no-ops in
// its running sums; the distance factors fold to the same constants).
// box[r][c] = out[i - R - 2 + r][j - R - 2 + c] (unpadded, clamped: the
// clamped entries are the ones no tap reads); bit (r, c) of sb = padded
// (i - R - 1 + r, j - R - 1 + c) unknown.
template <int R>
__device__ void fill_single_box(const uint32_t *bits, int wpr, int i, int j, uint8_t *out, int H, int W) {
    const int PH = H + 2, PW = W + 2;
    if (!(i > 1 && j > 1)) return;  // the serial loop never fills the first row / column
    constexpr int WS = 2 * R + 1, BS = WS + 2;
    int box[BS][BS];
    const int r0 = i - R - 2, c0 = j - R - 2;
#pragma unroll
    for (int r = 0; r < BS; ++r) {
        const int rr = min(max(r0 + r, 0), H - 1);
#pragma unroll
        for (int c = 0; c < BS; ++c) box[r][c] = out[rr * W + min(max(c0 + c, 0), W - 1)];
    }
    uint32_t sb[BS];  // padded rows i - R - 1 .. i + R + 1, columns j - R - 1 .. j + R + 1
    {
        const int xa = j - R - 1, xb = j + R + 1;
        const int ca = xa > 0 ? xa : 0, cb = xb < PW - 1 ? xb : PW - 1;
#pragma unroll
        for (int r = 0; r < BS; ++r) {
            const int y = i - R - 1 + r;
            sb[r] = (y >= 0 && y < PH) ? row_span(bits, wpr, y, ca, cb) << (ca - xa) : 0u;
        }
    }
    float Ia = 0.0f, sw = 1.0e-20f;
#pragma unroll
    for (int a = 0; a < WS; ++a) {
#pragma unroll
        for (int b = 0; b < WS; ++b) {
            if ((a - R) * (a - R) + (b - R) * (b - R) > R * R) continue;  // outside the radius: (0, 0)
            const int k = i - R + a, l = j - R + b;
            if (!(k > 0 && l > 0 && k < PH - 1 && l < PW - 1)) continue;
            if ((sb[a + 1] >> (b + 1)) & 1u) continue;  // unknown
            const bool e0 = k == 1, e1 = k == PH - 2, f0 = l == 1, f1 = l == PW - 2;
#define BOX(rr, cc) box[rr][cc]
            const int pA = e1 ? (f0 ? BOX(a + 1, b + 2) : BOX(a + 1, b + 1)) : (f0 ? BOX(a + 2, b + 2) : BOX(a + 2, b + 1));
            const int pB = e1 ? (f0 ? BOX(a, b + 2) : BOX(a, b + 1)) : (f0 ? BOX(a + 1, b + 2) : BOX(a + 1, b + 1));
            const int pC = e0 ? (f0 ? BOX(a + 1, b + 2) : BOX(a + 1, b + 1)) : (f0 ? BOX(a, b + 2) : BOX(a, b + 1));
            const int pD = e0 ? (f1 ? BOX(a + 2, b + 1) : BOX(a + 2, b + 2)) : (f1 ? BOX(a + 1, b + 1) : BOX(a + 1, b + 2));
            const int pE = e0 ? (f0 ? BOX(a + 2, b + 2) : BOX(a + 2, b + 1)) : (f0 ? BOX(a + 1, b + 2) : BOX(a + 1, b + 1));
            const int pF = e0 ? (f0 ? BOX(a + 2, b + 1) : BOX(a + 2, b)) : (f0 ? BOX(a + 1, b + 1) : BOX(a + 1, b));
#undef BOX
            const float ry = (float)(a - R), rx = (float)(b - R);
            const float lr = rx * rx + ry * ry;
            const float dst = (float)(1. / (lr * sqrt((double)lr)));
            const bool up_ok = !((sb[a] >> (b + 1)) & 1u), dn_ok = !((sb[a + 2] >> (b + 1)) & 1u);
            const bool lf_ok = !((sb[a + 1] >> b) & 1u), rt_ok = !((sb[a + 1] >> (b + 2)) & 1u);
            float gx, gy;
            if (dn_ok) {
                if (up_ok)
                    gx = (float)(abs(pA - pB) + abs(pB - pC));
                else
                    gx = (float)(abs(pA - pB)) * 2.0f;
            } else {
                if (up_ok)
                    gx = (float)(abs(pB - pC)) * 2.0f;
                else
                    gx = 0;
            }
            if (rt_ok) {
                if (lf_ok)
                    gy = -(float)(abs(pD - pE) + abs(pE - pF));
                else
                    gy = -(float)(abs(pD - pE)) * 2.0f;
            } else {
                if (lf_ok)
                    gy = -(float)(abs(pE - pF)) * 2.0f;
                else
                    gy = 0;
            }
            const float dot = rx * gx + ry * gy;
            const float lg = gx * gx + gy * gy;
            float dir = fabsf(dot / sqrtf(lr * lg));
            if (!(dir > 0.01f)) dir = 0.000001f;
            const float w = dst * dir;
            Ia += w * (float)pE;
            sw += w;
        }
    }
    out[(i - 1) * W + (j - 1)] = ns_value(Ia, sw);
}

// Per-frame setup, one workgroup per frame, on the frame's bit image in LDS.
// Frames over the sparse capacity (or too large for the LDS image) are only
// counted and flagged for k_inp_dense.
__global__ __launch_bounds__(INP_SETUP_THREADS) void k_inp_setup(uint8_t *__restrict__ frames, int range, char *ws,
                                                                 InpLayout L, unsigned int *__restrict__ errors) {
    constexpr int NT = INP_SETUP_THREADS;
    extern __shared__ uint32_t lds[];
    __shared__ int sh[NT];
    __shared__ int s_flag[2], s_bad;
    const int tid = threadIdx.x;
    const long long f = blockIdx.x;
    if (!ws_ok(ws, L)) {  // a workspace not set up for this frame shape: counted, left as is
        if (tid == 0) {
            atomicAdd(&g_inp_errors, 1u);
            if (errors) atomicAdd(errors, 1u);
        }
        return;
    }
    const Slot<int16_t> S = slot_view<int16_t>(frame_slot(ws, L, f), L.s);
    const int H = L.H, W = L.W, PW = L.PW, wpr = L.wpr, nw = L.nw;
    const long long HW = L.hw;
    uint32_t *fbits = L.bits(ws) + f * L.bits_fstride();
    uint8_t *out = frames + f * HW;
    uint32_t *bits = lds;
    uint16_t *pref = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(lds) + L.lds_pref);
    int16_t *lab = reinterpret_cast<int16_t *>(reinterpret_cast<char *>(lds) + L.lds_lab);
    // the frame's bit image into LDS (4 words per lane per step)
    int m = 0;
    for (int w = 4 * tid; w < nw; w += 4 * NT) {
        uint32_t v[4];
        if (w + 4 <= nw) {
            const uint4 u = *reinterpret_cast<const uint4 *>(fbits + w);
            v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
        } else {
            for (int q = 0; q < 4; ++q) v[q] = w + q < nw ? fbits[w + q] : 0u;
        }
        for (int q = 0; q < 4; ++q) {
            m += __popc(v[q]);
            if (L.lds_ok && w + q < nw) bits[w + q] = v[q];
        }
    }
    const int nin = block_sum<NT>(m, sh);
    const bool dense = nin > L.cap || (!L.lds_ok && nin > 0);
    if (tid == 0) {
        S.hdr[0] = nin;
        S.hdr[1] = S.hdr[2] = 0;
        S.hdr[3] = dense;
    }
    if (nin == 0 || dense) return;  // (k_inp_dense reads and clears a dense frame's bit image)
    // the workspace's bit image back to rest (zero) where it was set
    for (int w = tid; w < nw; w += NT)
        if (bits[w]) fbits[w] = 0u;
    // rank of each word's first bit
    const int per = (nw + NT - 1) / NT, w0 = tid * per, w1 = w0 + per < nw ? w0 + per : nw;
    int c = 0;
    for (int w = w0; w < w1; ++w) c += __popc(bits[w]);
    int tot;
    int run = block_scan_excl<NT>(c, sh, tot);
    for (int w = w0; w < w1; ++w) {
        pref[w] = (uint16_t)run;
        run += __popc(bits[w]);
    }
    __syncthreads();
    // the unknown list in raster order; one-pixel clusters get label -1
    const int R = range + 1 > 2 ? range + 1 : 2;
    for (int w = w0; w < w1; ++w) {
        uint32_t b = bits[w];
        const int y = w / wpr, xb = (w - y * wpr) * 32;
        while (b) {
            const int x = xb + __ffs(b) - 1;
            b &= b - 1;
            const int k = bit_rank(bits, pref, wpr, y, x);
            S.ins[k] = y * PW + x;
            lab[k] = (int16_t)(has_other(bits, wpr, y, x, R, H, W) ? k : -1);
        }
    }
    // clusters of the others: min-label propagation over Chebyshev distance
    // <= R with pointer jumping.  Two convergence flags, alternating per
    // iteration: thread 0 clears the NEXT iteration's flag after this
    // iteration's first barrier, when every thread has read it (as the
    // previous iteration's flag) and before any thread can set it.  Each label
    // is written by its own thread only; others may read it old or new (the
    // propagation is monotone).
    if (tid == 0) s_flag[0] = s_flag[1] = s_bad = 0;
    for (int iter = 0; iter < 1 << 20; ++iter) {
        __syncthreads();
        if (tid == 0) s_flag[(iter + 1) & 1] = 0;
        int changed = 0;
        for (int w = w0; w < w1; ++w) {
            uint32_t b = bits[w];
            const int y = w / wpr, xb = (w - y * wpr) * 32;
            while (b) {
                const int x = xb + __ffs(b) - 1;
                b &= b - 1;
                const int k = bit_rank(bits, pref, wpr, y, x);
                int mn = lab[k];
                if (mn < 0) continue;
                const int xa = x - R > 1 ? x - R : 1, xe = x + R < W ? x + R : W;
                const int ya = y - R > 1 ? y - R : 1, ye = y + R < H ? y + R : H;
                for (int yy = ya; yy <= ye; ++yy) {
                    uint32_t sp = row_span(bits, wpr, yy, xa, xe);
                    while (sp) {
                        const int q = __ffs(sp) - 1;
                        sp &= sp - 1;
                        const int l = lab[bit_rank(bits, pref, wpr, yy, xa + q)];
                        mn = l < mn ? l : mn;
                    }
                }
                const int lm = lab[mn];  // pointer jump
                mn = lm < mn ? lm : mn;
                if (mn < lab[k]) {
                    lab[k] = (int16_t)mn;
                    changed = 1;
                }
            }
        }
        if (changed) atomicOr(&s_flag[iter & 1], 1);
        __syncthreads();
        if (!s_flag[iter & 1]) break;
    }
    // converged labels are roots (lab[lab[k]] == lab[k]); the cluster phase
    // below indexes the cluster tables by them, so a frame that left the loop
    // unconverged is counted in g_inp_errors (mdx_inpaint_errors) and left
    // un-inpainted (nothing has been written to its plane yet)
    {
        int bad = 0;
        for (int k = tid; k < nin; k += NT) {
            const int l = lab[k];
            if (l >= 0) bad |= l > k || lab[l] != l;
        }
        if (bad) atomicOr(&s_bad, 1);
        __syncthreads();
        if (s_bad) {
            if (tid == 0) {
                atomicAdd(&g_inp_errors, 1u);
                if (errors) atomicAdd(errors, 1u);
            }
            return;
        }
    }
    // multi-pixel clusters: ids for roots in raster order, member counts,
    // starts, member lists; their pixels' plane entries and narrow band
    int ncl = 0;
    for (int k0 = 0; k0 < nin; k0 += NT) {
        const int k = k0 + tid;
        const int root = (k < nin && lab[k] == k) ? 1 : 0;
        const int pos = ncl + block_scan_excl<NT>(root, sh, tot);
        if (root) {
            S.fill[k] = pos;  // root index -> cluster id
            S.cnt[pos] = 0;
        }
        ncl += tot;
    }
    if (ncl > 0) {  // uniform
        __syncthreads();
        for (int k = tid; k < nin; k += NT)
            if (lab[k] >= 0) atomicAdd(&S.cnt[S.fill[lab[k]]], 1);
        __syncthreads();
        run = 0;
        for (int c0 = 0; c0 < ncl; c0 += NT) {
            const int cl = c0 + tid;
            const int v = cl < ncl ? S.cnt[cl] : 0;
            const int pos = run + block_scan_excl<NT>(v, sh, tot);
            if (cl < ncl) S.start[cl] = pos;
            run += tot;
        }
        if (tid == 0) S.start[ncl] = run;
        __syncthreads();
        for (int k = tid; k < nin; k += NT)
            if (lab[k] >= 0) S.lab[k] = S.fill[lab[k]];
        __syncthreads();
        for (int cl = tid; cl < ncl; cl += NT) S.cnt[cl] = 0;
        __syncthreads();
        // member lists: list index (S.ord) and padded pixel (S.fill); the
        // march marks the plane itself for the clusters it cannot window
        for (int k = tid; k < nin; k += NT) {
            if (lab[k] < 0) continue;
            const int cl = S.lab[k];
            const int slot = atomicAdd(&S.cnt[cl], 1);
            S.ord[S.start[cl] + slot] = k;
            S.fill[S.start[cl] + slot] = S.ins[k];
        }
    }
    // one-pixel clusters, in place
    const BitState bs{bits, wpr, out, W};
    for (int k = tid; k < nin; k += NT)
        if (lab[k] < 0) {
            const int j = S.ins[k];
            if (range == 3)  // the extract path's radius
                fill_single_box<3>(bits, wpr, j / PW, j - j / PW * PW, out, H, W);
            else
                fill_single(bs, j / PW, j - j / PW * PW, out, H, W, range);
        }
    if (tid == 0) {
        S.hdr[1] = ncl;
        S.hdr[2] = ncl;  // every cluster listed here has more than one pixel
    }
}

// One cluster of m > 1 pixels on one wave, on the global plane and frame.
// Lane 0 owns the cluster's serial state (member sort, narrow band FIFO, (T,
// seq) heap); the window of every pixel being filled is evaluated one tap per
// lane and summed in the serial loop's (k, l) order (wave_tap_sum), so the
// float sums are the serial ones bit for bit.  The cluster's plane entries are
// put back to rest at the end.
template <typename Idx>
__device__ void march_cluster(const Slot<Idx> &S, int c, uint8_t *out, int H, int W, int range, float *tw,
                              float *twi) {
    const int lane = threadIdx.x & 63;
    const int PH = H + 2, PW = W + 2;
    const int s0 = S.start[c], m = S.start[c + 1] - s0;
    int *mem = S.ord + s0;
    int *band = S.scr + 7LL * s0;
    HEnt *heap = reinterpret_cast<HEnt *>(band + 4LL * m);
    Idx *code = S.plane;
    int nb = 0;
    if (lane == 0) {
        // members in raster order (unknown-list index order == raster order)
        for (int a = 1; a < m; ++a) {
            const int v = mem[a];
            int b = a - 1;
            while (b >= 0 && mem[b] > v) {
                mem[b + 1] = mem[b];
                --b;
            }
            mem[b + 1] = v;
        }
        // this cluster's narrow band, raster order, unique
        for (int a = 0; a < m; ++a) {
            const int i = S.ins[mem[a]];
            const int cand[4] = {i - PW, i - 1, i + 1, i + PW};
            for (int q = 0; q < 4; ++q) {
                const int p = cand[q];
                if (code[p] != -1) continue;
                int b = nb - 1;
                bool dup = false;
                while (b >= 0 && band[b] >= p) {
                    if (band[b] == p) {
                        dup = true;
                        break;
                    }
                    --b;
                }
                if (dup) continue;
                for (int z = nb; z > b + 1; --z) band[z] = band[z - 1];
                band[b + 1] = p;
                ++nb;
            }
        }
    }
    int head = 0, hn = 0, seq = __shfl(nb, 0);
    for (;;) {
        int idx = -1;
        if (lane == 0) {
            if (head < nb)
                idx = band[head++];
            else if (hn > 0)
                idx = heap_pop(heap, hn).idx;
        }
        idx = __shfl(idx, 0);
        if (idx < 0) break;
        const int ii = idx / PW, jj = idx - ii * PW;
        for (int q = 0; q < 4; ++q) {
            int i, j;
            if (q == 0) { i = ii - 1; j = jj; }
            else if (q == 1) { i = ii; j = jj - 1; }
            else if (q == 2) { i = ii + 1; j = jj; }
            else { i = ii; j = jj + 1; }
            if (i <= 1 || j <= 1 || i > PH - 1 || j > PW - 1) continue;
            const int v = code[i * PW + j];
            if (v <= 0) continue;
            float Ia, sw;
            wave_tap_sum(PlaneState<Idx>{code, PW, out, W}, i, j, range, PH, PW, tw, twi, Ia, sw);
            if (lane == 0) {
                const float dist = min4f(fm_solve(i - 1, j, i, j - 1, S, PW), fm_solve(i + 1, j, i, j - 1, S, PW),
                                         fm_solve(i - 1, j, i, j + 1, S, PW), fm_solve(i + 1, j, i, j + 1, S, PW));
                out[(i - 1) * W + (j - 1)] = ns_value(Ia, sw);
                S.t[v - 1] = dist;
                code[i * PW + j] = (Idx)(-v - 1);  // filled: -(k + 2)
                heap_push(heap, hn, HEnt{dist, seq++, i * PW + j});
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
    }
    for (int a = lane; a < m; a += 64) rest_pixel(S, S.ins[mem[a]], PW);
}

// A small cluster's march in LDS: the window of padded pixels within range + 1
// of the cluster's bounding box (every state and pixel value the march reads)
// staged per wave, marched with the global march's exact arithmetic and
// order, the filled values written back.  Window states: 0 KNOWN, -1 band,
// a + 1 member a (sorted list) not yet filled, -(a + 2) filled.
constexpr int WIN_MAX = 1024, WIN_MMAX = 64;
struct WinLds {
    int16_t code[WIN_MAX];
    uint8_t px[WIN_MAX];
    float tm[WIN_MMAX];
    int mem[WIN_MMAX], mloc[WIN_MMAX];
    int band[4 * WIN_MMAX];
    HEnt heap[WIN_MMAX];
    float tw[MAX_TAPS], twi[MAX_TAPS];
};

struct WinState {
    const int16_t *code;
    const uint8_t *pxv;
    int wy0, wx0, ww;
    __device__ __forceinline__ bool unknown(int k, int l) const { return code[(k - wy0) * ww + (l - wx0)] > 0; }
    __device__ __forceinline__ int px(int r, int c) const { return pxv[(r + 1 - wy0) * ww + (c + 1 - wx0)]; }
};

__device__ __forceinline__ float win_t(const WinLds &w, int li) {
    const int v = w.code[li];
    return v == 0 ? 1.0e6f : (v == -1 ? 0.0f : w.tm[v > 0 ? v - 1 : -v - 2]);
}

__device__ __forceinline__ float win_fm_solve(const WinLds &w, int l1, int l2) {
    double sol;
    const double a11 = win_t(w, l1), a22 = win_t(w, l2);
    const double m12 = a11 < a22 ? a11 : a22;
    const bool in1 = w.code[l1] > 0, in2 = w.code[l2] > 0;
    if (!in1) {
        if (!in2) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt((double)(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else
            sol = 1 + a11;
    } else if (!in2)
        sol = 1 + a22;
    else
        sol = 1 + m12;
    return (float)sol;
}

// false (nothing done) when the cluster or its window is too large.  The
// window's states come from the member pixels alone (S.fill[s0, s0 + m),
// written by k_inp_setup): members, then their interior 4-neighbours as the
// band; no other unknown pixel lies within reach of the march.
template <typename Idx>
__device__ bool march_window(const Slot<Idx> &S, int s0, int m, uint8_t *out, int H, int W, int range, WinLds &w) {
    const int lane = threadIdx.x & 63;
    const int PH = H + 2, PW = W + 2;
    if (m > WIN_MMAX) return false;
    int ymin = 1 << 30, ymax = -1, xmin = 1 << 30, xmax = -1;
    for (int a = lane; a < m; a += 64) {
        const int j = S.fill[s0 + a], y = j / PW, x = j - y * PW;
        w.mem[a] = j;
        ymin = y < ymin ? y : ymin;
        ymax = y > ymax ? y : ymax;
        xmin = x < xmin ? x : xmin;
        xmax = x > xmax ? x : xmax;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ymin = min(ymin, __shfl_xor(ymin, o));
        ymax = max(ymax, __shfl_xor(ymax, o));
        xmin = min(xmin, __shfl_xor(xmin, o));
        xmax = max(xmax, __shfl_xor(xmax, o));
    }
    const int E = range + 1;
    const int wy0 = ymin - E > 0 ? ymin - E : 0, wy1 = ymax + E < PH - 1 ? ymax + E : PH - 1;
    const int wx0 = xmin - E > 0 ? xmin - E : 0, wx1 = xmax + E < PW - 1 ? xmax + E : PW - 1;
    const int ww = wx1 - wx0 + 1, area = (wy1 - wy0 + 1) * ww;
    if (area > WIN_MAX) return false;
    for (int li = lane; li < area; li += 64) {
        const int ly = li / ww, y = wy0 + ly, x = wx0 + li - ly * ww;
        w.code[li] = 0;
        w.px[li] = (y >= 1 && y <= H && x >= 1 && x <= W) ? out[(y - 1) * W + (x - 1)] : (uint8_t)0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (lane == 0) {  // members in raster order (pixel index order == list order)
        for (int a = 1; a < m; ++a) {
            const int v = w.mem[a];
            int b = a - 1;
            while (b >= 0 && w.mem[b] > v) {
                w.mem[b + 1] = w.mem[b];
                --b;
            }
            w.mem[b + 1] = v;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    for (int a = lane; a < m; a += 64) {
        const int j = w.mem[a], y = j / PW, x = j - y * PW;
        const int li = (y - wy0) * ww + (x - wx0);
        w.mloc[a] = li;
        w.code[li] = (int16_t)(a + 1);
        w.tm[a] = 1.0e6f;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    for (int a = lane; a < m; a += 64) {  // the band: interior 4-neighbours that are not members
        const int li = w.mloc[a], ly = li / ww, y = wy0 + ly, x = wx0 + li - ly * ww;
        const int nb[4] = {li - ww, li - 1, li + 1, li + ww};
        const int ny[4] = {y - 1, y, y, y + 1}, nx[4] = {x, x - 1, x + 1, x};
        for (int q = 0; q < 4; ++q)
            if (ny[q] >= 1 && ny[q] <= H && nx[q] >= 1 && nx[q] <= W && w.code[nb[q]] <= 0) w.code[nb[q]] = -1;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    int nb = 0;
    if (lane == 0) {  // this cluster's narrow band, raster order, unique
        for (int a = 0; a < m; ++a) {
            const int i = w.mloc[a];
            const int cand[4] = {i - ww, i - 1, i + 1, i + ww};
            for (int q = 0; q < 4; ++q) {
                const int p = cand[q];
                if (w.code[p] != -1) continue;
                int b = nb - 1;
                bool dup = false;
                while (b >= 0 && w.band[b] >= p) {
                    if (w.band[b] == p) {
                        dup = true;
                        break;
                    }
                    --b;
                }
                if (dup) continue;
                for (int z = nb; z > b + 1; --z) w.band[z] = w.band[z - 1];
                w.band[b + 1] = p;
                ++nb;
            }
        }
    }
    const WinState st{w.code, w.px, wy0, wx0, ww};
    int head = 0, hn = 0, seq = __shfl(nb, 0);
    for (;;) {
        int idx = -1;
        if (lane == 0) {
            if (head < nb)
                idx = w.band[head++];
            else if (hn > 0)
                idx = heap_pop(w.heap, hn).idx;
        }
        idx = __shfl(idx, 0);
        if (idx < 0) break;
        const int iy = idx / ww, ii = wy0 + iy, jj = wx0 + idx - iy * ww;
        for (int q = 0; q < 4; ++q) {
            int i, j;
            if (q == 0) { i = ii - 1; j = jj; }
            else if (q == 1) { i = ii; j = jj - 1; }
            else if (q == 2) { i = ii + 1; j = jj; }
            else { i = ii; j = jj + 1; }
            if (i <= 1 || j <= 1 || i > PH - 1 || j > PW - 1) continue;
            const int li = (i - wy0) * ww + (j - wx0);
            const int v = w.code[li];
            if (v <= 0) continue;
            float Ia, sw;
            wave_tap_sum(st, i, j, range, PH, PW, w.tw, w.twi, Ia, sw);
            if (lane == 0) {
                const float dist = min4f(win_fm_solve(w, li - ww, li - 1), win_fm_solve(w, li + ww, li - 1),
                                         win_fm_solve(w, li - ww, li + 1), win_fm_solve(w, li + ww, li + 1));
                w.px[li] = ns_value(Ia, sw);
                w.tm[v - 1] = dist;
                w.code[li] = (int16_t)(-v - 1);  // filled: -(a + 2)
                heap_push(w.heap, hn, HEnt{dist, seq++, li});
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
    }
    for (int a = lane; a < m; a += 64) {
        const int li = w.mloc[a];
        const int ly = li / ww, y = wy0 + ly, x = wx0 + li - ly * ww;
        out[(y - 1) * W + (x - 1)] = w.px[li];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    return true;
}

// a cluster the window does not hold: its plane entries (members k + 1, T
// 1e6; their band -1), then the march on the global plane (which puts them
// back to rest)
template <typename Idx>
__device__ void march_global(const Slot<Idx> &S, int c, uint8_t *out, int H, int W, int range, float *tw,
                             float *twi) {
    const int lane = threadIdx.x & 63;
    const int PW = W + 2;
    const int s0 = S.start[c], m = S.start[c + 1] - s0;
    for (int a = lane; a < m; a += 64) {
        const int k = S.ord[s0 + a];
        S.plane[S.fill[s0 + a]] = (Idx)(k + 1);
        S.t[k] = 1.0e6f;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    for (int a = lane; a < m; a += 64) {
        const int p = S.fill[s0 + a], y = p / PW, x = p - y * PW;
        const int nb[4] = {p - PW, p - 1, p + 1, p + PW};
        const int ny[4] = {y - 1, y, y, y + 1}, nx[4] = {x, x - 1, x + 1, x};
        for (int q = 0; q < 4; ++q)
            if (ny[q] >= 1 && ny[q] <= H && nx[q] >= 1 && nx[q] <= W && S.plane[nb[q]] <= 0) S.plane[nb[q]] = (Idx)-1;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    march_cluster(S, c, out, H, W, range, tw, twi);
}

__global__ __launch_bounds__(64 * MARCH_WAVES) void k_inp_march(uint8_t *__restrict__ frames, int range, char *ws,
                                                                 InpLayout L) {
    __shared__ WinLds s_win[MARCH_WAVES];
    if (!ws_ok(ws, L)) return;
    const long long f = blockIdx.y;
    const int wid = threadIdx.x >> 6;
    const Slot<int16_t> S = slot_view<int16_t>(frame_slot(ws, L, f), L.s);
    const int nmulti = S.hdr[2];
    uint8_t *out = frames + f * (long long)L.hw;
    WinLds &w = s_win[wid];
    for (int q = blockIdx.x * MARCH_WAVES + wid; q < nmulti; q += gridDim.x * MARCH_WAVES) {
        const int s0 = S.start[q], m = S.start[q + 1] - s0;
        if (!march_window(S, s0, m, out, L.H, L.W, range, w)) march_global(S, q, out, L.H, L.W, range, w.tw, w.twi);
    }
}

// The frames over the sparse capacity, one after another on one workgroup in
// the dense slot: compaction, setup, the march on its 16 waves.  The frames'
// flags (slot header [3], set by k_inp_setup) are gathered 1024 at a time.
__global__ __launch_bounds__(INP_DENSE_THREADS) void k_inp_dense(uint8_t *__restrict__ frames, long long n, int range,
                                                                 char *ws, InpLayout L,
                                                                 unsigned int *__restrict__ errors) {
    __shared__ int sh[INP_DENSE_THREADS], s_list[INP_DENSE_THREADS];
    __shared__ float s_w[DENSE_WAVES][MAX_TAPS], s_wi[DENSE_WAVES][MAX_TAPS];
    if (!ws_ok(ws, L)) return;
    const int tid = threadIdx.x, wid = tid >> 6;
    const Slot<int> D = slot_view<int>(ws + L.o_dense, L.d);
    const long long HW = L.hw;
    for (long long f0 = 0; f0 < n; f0 += INP_DENSE_THREADS) {
        const int flag = f0 + tid < n ? reinterpret_cast<const int *>(frame_slot(ws, L, f0 + tid))[3] : 0;
        int ndense;
        const int at = block_scan_excl<INP_DENSE_THREADS>(flag, sh, ndense);
        if (flag) s_list[at] = tid;
        __syncthreads();
        for (int q = 0; q < ndense; ++q) {
            const long long f = f0 + s_list[q];
            // the unknown list in raster order from the frame's bit image
            uint32_t *fb = L.bits(ws) + f * L.bits_fstride();
            int nin = 0;
            for (int w0 = 0; w0 < L.nw; w0 += INP_DENSE_THREADS) {
                const int w = w0 + tid;
                const uint32_t v = w < L.nw ? fb[w] : 0u;
                int tot;
                int pos = nin + block_scan_excl<INP_DENSE_THREADS>(__popc(v), sh, tot);
                const int y = w / L.wpr, xb = (w - y * L.wpr) * 32;
                if (v) fb[w] = 0u;  // back to rest
                for (uint32_t b = v; b; b &= b - 1) {
                    const int j = y * L.PW + xb + __ffs(b) - 1;
                    D.ins[pos] = j;
                    D.plane[j] = pos + 1;
                    D.lab[pos] = pos;
                    D.t[pos] = 1.0e6f;
                    ++pos;
                }
                nin += tot;
            }
            __syncthreads();
            uint8_t *out = frames + f * HW;
            const int nmulti = setup_body<int, INP_DENSE_THREADS>(D, nin, out, L.H, L.W, range, errors);
            for (int c = wid; c < nmulti; c += DENSE_WAVES)
                march_cluster(D, D.fill[c], out, L.H, L.W, range, s_w[wid], s_wi[wid]);
            __syncthreads();
        }
        __syncthreads();
    }
}

}  // namespace mdx

using namespace mdx;

extern "C" int mdx_inpaint_errors(int reset) {
    unsigned int v = 0;
    MDX_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_inp_errors), sizeof(v)));
    if (reset) {
        const unsigned int z = 0;
        MDX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_inp_errors), &z, sizeof(z)));
    }
    return (int)v;
}

extern "C" int64_t mdx_inpaint_workspace_bytes(int64_t n, int H, int W) {
    if (n <= 0 || H <= 0 || W <= 0 || (int64_t)(H + 2) * (W + 2) >= (1ll << 30)) return 0;
    const InpLayout L = inp_layout(H, W);
    return L.o_slots + n * L.s.bytes;
}

extern "C" int mdx_inpaint_sparse_capacity(int H, int W) {
    if (H <= 0 || W <= 0 || (int64_t)(H + 2) * (W + 2) >= (1ll << 30)) return 0;
    return inp_layout(H, W).cap;
}

extern "C" int mdx_inpaint_workspace_init(void *workspace, int64_t bytes, int H, int W, mdx_stream_t stream) {
    MDX_REQUIRE(workspace != nullptr, "mdx_inpaint_workspace_init: null workspace");
    MDX_REQUIRE(H > 0 && W > 0 && (int64_t)(H + 2) * (W + 2) < (1ll << 30), "mdx_inpaint_workspace_init: bad shape");
    MDX_REQUIRE(bytes >= mdx_inpaint_workspace_bytes(1, H, W),
                "mdx_inpaint_workspace_init: %lld bytes is less than one frame's workspace", (long long)bytes);
    hipStream_t s = as_stream(stream);
    MDX_HIP(hipMemsetAsync(workspace, 0, (size_t)bytes, s));
    hipLaunchKernelGGL(k_inp_header, dim3(1), dim3(64), 0, s, (int *)workspace, H, W);
    MDX_CHECK_LAUNCH("mdx_inpaint_workspace_init");
    return MDX_OK;
}

// setup / march / dense on the bit images already in the workspace's slots
static int run_inpaint(uint8_t *frames, int64_t n, const InpLayout &L, int radius, char *ws, unsigned int *errors,
                       hipStream_t s) {
    if (L.lds_bytes > 64 * 1024) {
        static std::atomic<int> attr_bytes{0};  // raised once per size
        if (L.lds_bytes > attr_bytes.load()) {
            MDX_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_inp_setup),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, L.lds_bytes));
            attr_bytes.store(L.lds_bytes);
        }
    }
    hipLaunchKernelGGL(k_inp_setup, dim3((unsigned)n), dim3(INP_SETUP_THREADS), L.lds_bytes, s, frames, radius, ws, L,
                       errors);
    hipLaunchKernelGGL(k_inp_march, dim3(INP_MARCH_BLOCKS, (unsigned)n), dim3(64 * MARCH_WAVES), 0, s, frames, radius,
                       ws, L);
    hipLaunchKernelGGL(k_inp_dense, dim3(1), dim3(INP_DENSE_THREADS), 0, s, frames, (long long)n, radius, ws, L,
                       errors);
    MDX_CHECK_LAUNCH("mdx_inpaint_ns");
    return MDX_OK;
}

extern "C" int mdx_inpaint_ns_counted(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                                      void *workspace, unsigned int *errors, mdx_stream_t stream) {
    MDX_REQUIRE(frames && invalid, "mdx_inpaint_ns: null frames/invalid");
    MDX_REQUIRE(radius >= 0 && radius <= 7, "mdx_inpaint_ns: radius must be in [0, 7] (got %d)", radius);
    MDX_REQUIRE(H > 0 && W > 0, "mdx_inpaint_ns: bad shape");
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(workspace != nullptr, "mdx_inpaint_ns: null workspace");
    MDX_REQUIRE((int64_t)(H + 2) * (W + 2) < (1ll << 30) && H + 2 <= 65535, "mdx_inpaint_ns: frame too large");
    MDX_REQUIRE(n <= 65535, "mdx_inpaint_ns: at most 65535 frames per call");
    const InpLayout L = inp_layout(H, W);
    hipStream_t s = as_stream(stream);
    char *ws = (char *)workspace;
    hipLaunchKernelGGL(k_inp_bits, dim3((unsigned)ceil_div(L.hw, 256), (unsigned)n), dim3(256), 0, s, invalid, ws, L);
    return run_inpaint(frames, n, L, radius, ws, errors, s);
}

extern "C" int mdx_inpaint_ns(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                              void *workspace, mdx_stream_t stream) {
    return mdx_inpaint_ns_counted(frames, invalid, n, H, W, radius, workspace, nullptr, stream);
}

extern "C" int mdx_prep_inpaint(const int16_t *raw, int64_t n, int H, int W, const double *bg, const uint8_t *roi,
                                int y0, int y1, int x0, int x1, int flags, double vmin, double vmax, uint8_t *out,
                                uint8_t *invalid, int radius, void *workspace, unsigned int *errors,
                                mdx_stream_t stream) {
    MDX_REQUIRE(raw && out, "mdx_prep_inpaint: null raw/out");
    MDX_REQUIRE(n >= 0 && H > 0 && W > 0, "mdx_prep_inpaint: bad shape n=%lld H=%d W=%d", (long long)n, H, W);
    MDX_REQUIRE(0 <= y0 && y0 < y1 && y1 <= H && 0 <= x0 && x0 < x1 && x1 <= W,
                "mdx_prep_inpaint: bad crop [%d,%d)x[%d,%d) for %dx%d", y0, y1, x0, x1, H, W);
    MDX_REQUIRE(radius >= 0 && radius <= 7, "mdx_prep_inpaint: radius must be in [0, 7] (got %d)", radius);
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(workspace != nullptr, "mdx_prep_inpaint: null workspace");
    const int oh = y1 - y0, ow = x1 - x0;
    MDX_REQUIRE((int64_t)(oh + 2) * (ow + 2) < (1ll << 30) && oh + 2 <= 65535, "mdx_prep_inpaint: frame too large");
    MDX_REQUIRE(n <= 65535, "mdx_prep_inpaint: at most 65535 frames per call");  // k_inp_setup's grid
    const InpLayout L = inp_layout(oh, ow);
    hipStream_t s = as_stream(stream);
    char *ws = (char *)workspace;
    const int rc = launch_prep(raw, n, H, W, bg, roi, y0, y1, x0, x1, flags, vmin, vmax, out, invalid, L.bits(ws),
                               L.bits_fstride(), L.wpr, s);
    if (rc != MDX_OK) return rc;
    return run_inpaint(out, n, L, radius, ws, errors, s);
}
