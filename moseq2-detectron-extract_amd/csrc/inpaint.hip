// fill_invalid_pixels -> cv2.inpaint(frame, invalid, 3, cv2.INPAINT_NS)
// (M/proc/proc.py:189-210; OpenCV imgproc/inpaint.cpp icvNSInpaintFMM as
// restated in oracle/frameops.c orc_inpaint_ns_one).
//
// Parallel decomposition that is EXACT w.r.t. the serial fast-marching order:
// computing an unknown pixel reads state only within Chebyshev distance
// `range + 1` of it (window taps +-range, gradients +-1, FMM neighbours +-1),
// and writes only the pixel itself.  Unknown pixels are therefore grouped into
// clusters (connected under Chebyshev distance <= range + 1); two clusters
// never read each other's changing state.  OpenCV's priority list pops by
// (T, insertion order); restricted to one cluster that order is the order a
// cluster-local list produces (its initial narrow band is pushed in raster
// order with T = 0, every later push has T >= 0.5), so each cluster can be
// marched independently -- one lane per cluster -- and the result is
// bit-identical to the serial algorithm.
//
//   k_inp_fill    code = KNOWN, T = 1e6 over every padded frame (wide grid)
//   k_inp_count / k_inp_compact  (4096-pixel chunks x frames): raster-ordered
//                 unknown-pixel list (chunk counts, chunk offsets, block scan)
//   k_inp_setup   (one workgroup per frame): narrow band, cluster labels
//                 (min-label propagation + pointer jumping), member lists.
//   k_inp_march   (one wave per cluster): local FIFO(band) + heap(T, seq) FMM
//                 with the NS weights (window taps one per lane, summed in
//                 the serial order), pixel values written in place.
#include <cmath>

#include "common.h"

#pragma clang fp contract(off)

namespace mdx {

// code image: >= 0 unknown (index into the unknown list); -1 KNOWN; -2 BAND
constexpr int C_KNOWN = -1, C_BAND = -2;
constexpr int INP_SETUP_THREADS = 256, INP_MARCH_BLOCKS = 64;

struct InpLayout {
    long long np;  // padded pixels
    // offsets (in int32 units) of the per-frame arrays
    long long o_code, o_t, o_ins, o_lab, o_cnt, o_start, o_fill, o_ord, o_scr, o_hdr, o_cc, total;
    int nch;       // compaction chunks of INP_CHUNK unpadded pixels
};

constexpr int INP_CHUNK = 4096;  // 256 lanes x 16 pixels

static inline InpLayout inp_layout(int H, int W) {
    InpLayout L;
    L.np = (long long)(H + 2) * (W + 2);
    long long o = 0;
    L.o_hdr = o; o += 16;
    L.nch = (int)(((long long)H * W + INP_CHUNK - 1) / INP_CHUNK);
    L.o_cc = o; o += (L.nch + 3) / 4 * 4;
    L.o_code = o; o += L.np;
    L.o_t = o; o += L.np;
    L.o_ins = o; o += L.np;
    L.o_lab = o; o += L.np;
    L.o_cnt = o; o += L.np;
    L.o_start = o; o += L.np + 1;
    L.o_fill = o; o += L.np;
    L.o_ord = o; o += L.np;
    L.o_scr = o; o += 7 * L.np;
    L.total = (o + 3) / 4 * 4;
    return L;
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

__device__ __forceinline__ float fm_solve(int i1, int j1, int i2, int j2, const int *code, const float *t, int PW) {
    double sol;
    const double a11 = t[i1 * PW + j1], a22 = t[i2 * PW + j2];
    const double m12 = a11 < a22 ? a11 : a22;
    const bool in1 = code[i1 * PW + j1] >= 0, in2 = code[i2 * PW + j2] >= 0;
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

__device__ __forceinline__ int block_scan_excl(int v, int *sh, int &total) {
    // exclusive prefix sum over a 256-thread block (sh: >= 256 ints)
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int o = 1; o < INP_SETUP_THREADS; o <<= 1) {
        const int a = tid >= o ? sh[tid - o] : 0;
        __syncthreads();
        sh[tid] += a;
        __syncthreads();
    }
    const int incl = sh[tid];
    total = sh[INP_SETUP_THREADS - 1];
    __syncthreads();
    return incl - v;
}

// code = KNOWN, t = 1e6 over every frame's padded image; grid (pixel
// blocks, frame), 32-bit indices (a 64-bit division per element made this
// kernel cost more than the march itself)
__global__ __launch_bounds__(256) void k_inp_fill(int *__restrict__ ws, InpLayout L) {
    int *base = ws + (long long)blockIdx.y * L.total;
    int *code = base + L.o_code;
    float *t = reinterpret_cast<float *>(base + L.o_t);
    const int np = (int)L.np;
    for (int k = blockIdx.x * 256 + threadIdx.x; k < np; k += gridDim.x * 256) {
        code[k] = C_KNOWN;
        t[k] = 1.0e6f;
    }
}

// the 16 mask bytes of lane `tid` in chunk c (unpadded raster order)
__device__ __forceinline__ void chunk_bytes(const uint8_t *msk, long long HW, int c, int tid, uint8_t *v) {
    const long long p0 = (long long)c * INP_CHUNK + tid * 16;
    if (p0 + 16 <= HW && ((reinterpret_cast<uintptr_t>(msk + p0) & 15) == 0)) {
        const uint4 u = *reinterpret_cast<const uint4 *>(msk + p0);
        const uint8_t *e = reinterpret_cast<const uint8_t *>(&u);
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = e[k];
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = (p0 + k < HW) ? msk[p0 + k] : 0;
    }
}

__device__ __forceinline__ int block_sum(int v, int *sh) {
    int total;
    block_scan_excl(v, sh, total);
    return total;
}

// unknown pixels per chunk
__global__ __launch_bounds__(INP_SETUP_THREADS) void k_inp_count(const uint8_t *__restrict__ invalid, int H, int W,
                                                                 int *__restrict__ ws, InpLayout L) {
    __shared__ int sh[INP_SETUP_THREADS];
    const long long f = blockIdx.y;
    const int c = blockIdx.x;
    const long long HW = (long long)H * W;
    uint8_t v[16];
    chunk_bytes(invalid + f * HW, HW, c, threadIdx.x, v);
    int m = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) m += v[k] != 0;
    const int tot = block_sum(m, sh);
    if (threadIdx.x == 0) ws[f * L.total + L.o_cc + c] = tot;
}

// ordered compaction of the unknown pixels: chunk offset = sum of the previous
// chunks' counts, lane offset = block scan; ins[k] = padded index (raster order)
__global__ __launch_bounds__(INP_SETUP_THREADS) void k_inp_compact(const uint8_t *__restrict__ invalid, int H, int W,
                                                                   int *__restrict__ ws, InpLayout L) {
    __shared__ int sh[INP_SETUP_THREADS];
    const long long f = blockIdx.y;
    const int c = blockIdx.x, tid = threadIdx.x;
    int *base = ws + f * L.total;
    const int *cc = base + L.o_cc;
    int prev = 0;
    for (int q = tid; q < c; q += INP_SETUP_THREADS) prev += cc[q];
    const int off = block_sum(prev, sh);
    if (cc[c] == 0) return;  // uniform per block
    const long long HW = (long long)H * W;
    uint8_t v[16];
    chunk_bytes(invalid + f * HW, HW, c, tid, v);
    int m = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) m += v[k] != 0;
    int tot;
    int pos = off + block_scan_excl(m, sh, tot);
    if (!m) return;
    int *code = base + L.o_code, *ins = base + L.o_ins, *lab = base + L.o_lab;
    const int PW = W + 2;
    const long long p0 = (long long)c * INP_CHUNK + tid * 16;
    for (int k = 0; k < 16; ++k) {
        if (!v[k]) continue;
        const long long p = p0 + k;
        const int y = (int)(p / W), x = (int)(p - (long long)y * W);
        const int j = (y + 1) * PW + x + 1;
        ins[pos] = j;
        code[j] = pos;
        lab[pos] = pos;
        ++pos;
    }
}

// frames whose label propagation ended unconverged (see k_inp_setup)
__device__ unsigned int g_inp_errors = 0;

__global__ __launch_bounds__(INP_SETUP_THREADS) void k_inp_setup(const uint8_t *__restrict__ invalid, int H, int W,
                                                                 int range, int *__restrict__ ws, InpLayout L,
                                                                 unsigned int *__restrict__ errors) {
    __shared__ int sh[INP_SETUP_THREADS];
    __shared__ int s_flag[2], s_bad;
    const int tid = threadIdx.x;
    const long long f = blockIdx.x;
    int *base = ws + f * L.total;
    int *hdr = base + L.o_hdr;
    int *code = base + L.o_code;
    float *t = reinterpret_cast<float *>(base + L.o_t);
    int *ins = base + L.o_ins, *lab = base + L.o_lab, *cnt = base + L.o_cnt, *start = base + L.o_start;
    int *fill = base + L.o_fill, *ord = base + L.o_ord;
    const int PH = H + 2, PW = W + 2;
    int part = 0;
    for (int q = tid; q < L.nch; q += INP_SETUP_THREADS) part += base[L.o_cc + q];
    const int nin = block_sum(part, sh);
    if (nin == 0) {
        if (tid == 0) hdr[0] = hdr[1] = 0;
        return;
    }
    // narrow band: interior 4-neighbours of unknown pixels that are not unknown
    for (int k = tid; k < nin; k += INP_SETUP_THREADS) {
        const int i = ins[k];
        const int nb[4] = {i - PW, i - 1, i + PW, i + 1};
        for (int q = 0; q < 4; ++q) {
            const int p = nb[q];
            const int y = p / PW, x = p - y * PW;
            if (y >= 1 && y < PH - 1 && x >= 1 && x < PW - 1 && code[p] < 0) {
                code[p] = C_BAND;
                t[p] = 0.0f;
            }
        }
    }
    __syncthreads();
    // clusters: min-label propagation over Chebyshev distance <= range + 1
    const int R = range + 1;
    // two convergence flags, alternating per iteration: thread 0 clears the
    // NEXT iteration's flag after this iteration's first barrier, when every
    // thread has read it (as the previous iteration's flag) and before any
    // thread can set it.  (One flag cleared at the top of the loop raced with
    // the slower waves' read of the previous iteration's value: a wave that
    // read the cleared flag left the loop alone, its barriers then paired
    // with the other waves' loop barriers, and the label arrays were indexed
    // before they had converged.)
    if (tid == 0) s_flag[0] = s_flag[1] = s_bad = 0;
    for (int iter = 0; iter < 1 << 20; ++iter) {
        __syncthreads();
        if (tid == 0) s_flag[(iter + 1) & 1] = 0;
        int changed = 0;
        for (int k = tid; k < nin; k += INP_SETUP_THREADS) {
            const int i = ins[k];
            const int y = i / PW, x = i - y * PW;
            int m = lab[k];
            for (int dy = -R; dy <= R; ++dy) {
                const int yy = y + dy;
                if (yy < 1 || yy > H) continue;
                for (int dx = -R; dx <= R; ++dx) {
                    const int xx = x + dx;
                    if (xx < 1 || xx > W) continue;
                    const int c = code[yy * PW + xx];
                    if (c >= 0) {
                        const int l = lab[c];
                        m = l < m ? l : m;
                    }
                }
            }
            m = lab[m] < m ? lab[m] : m;  // pointer jump
            if (m < lab[k]) {
                atomicMin(&lab[k], m);
                changed = 1;
            }
        }
        if (changed) atomicOr(&s_flag[iter & 1], 1);
        __syncthreads();
        if (!s_flag[iter & 1]) break;
    }
    // converged labels are roots (lab[lab[k]] == lab[k]); the cluster phase
    // below indexes fill[] / cnt[] by them, so a frame that left the loop
    // unconverged is counted in g_inp_errors (mdx_inpaint_errors) and left
    // un-inpainted instead of indexing with a stray label.  (Its own flag:
    // a slow wave may still be reading s_flag as it leaves the loop.)
    {
        int bad = 0;
        for (int k = tid; k < nin; k += INP_SETUP_THREADS) {
            const int l = lab[k];
            bad |= l < 0 || l > k || lab[l] != l;
        }
        if (bad) atomicOr(&s_bad, 1);
        __syncthreads();
        if (s_bad) {
            if (tid == 0) {
                hdr[0] = hdr[1] = 0;
                atomicAdd(&g_inp_errors, 1u);
                if (errors) atomicAdd(errors, 1u);  // the caller's own count (mdx_inpaint_ns_counted)
            }
            return;
        }
    }
    // cluster ids for roots (lab[k] == k) in raster order, member counts, starts
    int ncl = 0;
    for (int k0 = 0; k0 < nin; k0 += INP_SETUP_THREADS) {
        const int k = k0 + tid;
        const int root = (k < nin && lab[k] == k) ? 1 : 0;
        int tot;
        const int pos = ncl + block_scan_excl(root, sh, tot);
        if (root) {
            fill[k] = pos;  // temporarily: root index -> cluster id
            cnt[pos] = 0;
        }
        ncl += tot;
    }
    __syncthreads();
    for (int k = tid; k < nin; k += INP_SETUP_THREADS) atomicAdd(&cnt[fill[lab[k]]], 1);
    __syncthreads();
    int run = 0;
    for (int c0 = 0; c0 < ncl; c0 += INP_SETUP_THREADS) {
        const int c = c0 + tid;
        const int v = c < ncl ? cnt[c] : 0;
        int tot;
        const int pos = run + block_scan_excl(v, sh, tot);
        if (c < ncl) start[c] = pos;
        run += tot;
    }
    if (tid == 0) start[ncl] = nin;
    __syncthreads();
    // members: cluster id per member, then atomic slot (sorted per cluster later)
    for (int k = tid; k < nin; k += INP_SETUP_THREADS) lab[k] = fill[lab[k]];
    __syncthreads();
    for (int c = tid; c < ncl; c += INP_SETUP_THREADS) cnt[c] = 0;
    __syncthreads();
    for (int k = tid; k < nin; k += INP_SETUP_THREADS) {
        const int c = lab[k];
        const int slot = atomicAdd(&cnt[c], 1);
        ord[start[c] + slot] = k;
    }
    if (tid == 0) {
        hdr[0] = nin;
        hdr[1] = ncl;
    }
}

// One NS window tap (k, l) around the pixel (i, j) being filled: returns the
// weight w and the product w * I exactly as the serial loop forms them (0, 0
// for a tap the loop skips, an exact no-op in its running sums).
__device__ __forceinline__ void ns_tap(int k, int l, int i, int j, int range, int PH, int PW, int W,
                                       const int *__restrict__ code, const uint8_t *out, float &w_out, float &wi_out) {
    w_out = 0.f;
    wi_out = 0.f;
    const int km = k - 1 + (k == 1), kp = k - 1 - (k == PH - 2);
    const int lm = l - 1 + (l == 1), lp = l - 1 - (l == PW - 2);
    if (!(k > 0 && l > 0 && k < PH - 1 && l < PW - 1)) return;
    if (code[k * PW + l] >= 0) return;
    if ((l - j) * (l - j) + (k - i) * (k - i) > range * range) return;
    const float ry = (float)(k - i), rx = (float)(l - j);
    const float lr = rx * rx + ry * ry;
    const float dst = (float)(1. / (lr * sqrt((double)lr)));
    const bool up_ok = code[(k - 1) * PW + l] < 0, dn_ok = code[(k + 1) * PW + l] < 0;
    const bool lf_ok = code[k * PW + l - 1] < 0, rt_ok = code[k * PW + l + 1] < 0;
    float gx, gy;
    if (dn_ok) {
        if (up_ok)
            gx = (float)(abs(out[(kp + 1) * W + lm] - out[kp * W + lm]) + abs(out[kp * W + lm] - out[(km - 1) * W + lm]));
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
            gy = -(float)(abs(out[km * W + lp + 1] - out[km * W + lm]) + abs(out[km * W + lm] - out[km * W + lm - 1]));
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
    const float w = dst * dir;
    w_out = w;
    wi_out = w * (float)out[km * W + lm];
}

constexpr int MARCH_WAVES = 4, MAX_TAPS = 15 * 15;

// One wave per cluster.  Lane 0 owns the cluster's serial state (member sort,
// narrow band FIFO, (T, seq) heap); the window of every pixel being filled is
// evaluated one tap per lane and summed by lane 0 in the serial loop's (k, l)
// order, so the float sums are the serial ones bit for bit.
__global__ __launch_bounds__(64 * MARCH_WAVES) void k_inp_march(uint8_t *__restrict__ frames, int H, int W, int range,
                                                                 int *__restrict__ ws, InpLayout L) {
    __shared__ float s_w[MARCH_WAVES][MAX_TAPS], s_wi[MARCH_WAVES][MAX_TAPS];
    const long long f = blockIdx.y;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int *base = ws + f * L.total;
    const int ncl = base[L.o_hdr + 1];
    int *code = base + L.o_code;
    float *t = reinterpret_cast<float *>(base + L.o_t);
    const int *ins = base + L.o_ins;
    const int *start = base + L.o_start;
    int *ord = base + L.o_ord;
    int *scr = base + L.o_scr;
    uint8_t *out = frames + f * (long long)H * W;
    const int PH = H + 2, PW = W + 2;
    const int wside = 2 * range + 1, ntaps = wside * wside;
    float *tw = s_w[wid], *twi = s_wi[wid];
    for (int c = blockIdx.x * MARCH_WAVES + wid; c < ncl; c += gridDim.x * MARCH_WAVES) {
        const int s0 = start[c], m = start[c + 1] - s0;
        int *mem = ord + s0;
        int *band = scr + 7LL * s0;
        HEnt *heap = reinterpret_cast<HEnt *>(band + 4LL * m);
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
                const int i = ins[mem[a]];
                const int cand[4] = {i - PW, i - 1, i + 1, i + PW};
                for (int q = 0; q < 4; ++q) {
                    const int p = cand[q];
                    if (code[p] != C_BAND) continue;
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
                if (idx >= 0) code[idx] = C_KNOWN;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
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
                if (code[i * PW + j] < 0) continue;
                for (int tp = lane; tp < ntaps; tp += 64) {
                    const int k = i - range + tp / wside, l = j - range + tp % wside;
                    ns_tap(k, l, i, j, range, PH, PW, W, code, out, tw[tp], twi[tp]);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                if (lane == 0) {
                    const float dist =
                        min4f(fm_solve(i - 1, j, i, j - 1, code, t, PW), fm_solve(i + 1, j, i, j - 1, code, t, PW),
                              fm_solve(i - 1, j, i, j + 1, code, t, PW), fm_solve(i + 1, j, i, j + 1, code, t, PW));
                    float Ia = 0.0f, sw = 1.0e-20f;
                    for (int tp = 0; tp < ntaps; ++tp) {
                        Ia += twi[tp];
                        sw += tw[tp];
                    }
                    const double v = (double)Ia / sw;
                    const int r = __double2int_rn(v);
                    out[(i - 1) * W + (j - 1)] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
                    t[i * PW + j] = dist;
                    code[i * PW + j] = C_BAND;
                    heap_push(heap, hn, HEnt{dist, seq++, i * PW + j});
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
        }
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
    if (n <= 0 || H <= 0 || W <= 0) return 0;
    return n * inp_layout(H, W).total * 4;
}

extern "C" int mdx_inpaint_ns_counted(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                                      void *workspace, unsigned int *errors, mdx_stream_t stream) {
    MDX_REQUIRE(frames && invalid, "mdx_inpaint_ns: null frames/invalid");
    MDX_REQUIRE(radius >= 0 && radius <= 7, "mdx_inpaint_ns: radius must be in [0, 7] (got %d)", radius);
    MDX_REQUIRE(H > 0 && W > 0, "mdx_inpaint_ns: bad shape");
    if (n == 0) return MDX_OK;
    MDX_REQUIRE(workspace != nullptr, "mdx_inpaint_ns: null workspace");
    MDX_REQUIRE((int64_t)(H + 2) * (W + 2) < (1ll << 30), "mdx_inpaint_ns: frame too large");
    MDX_REQUIRE(n <= 65535, "mdx_inpaint_ns: at most 65535 frames per call");
    const InpLayout L = inp_layout(H, W);
    hipStream_t s = as_stream(stream);
    MDX_REQUIRE(L.np < (1ll << 31), "mdx_inpaint_ns: frame too large");
    hipLaunchKernelGGL(k_inp_fill, dim3((unsigned)ceil_div(L.np, 1024), (unsigned)n), dim3(256), 0, s,
                       (int *)workspace, L);
    hipLaunchKernelGGL(k_inp_count, dim3(L.nch, (unsigned)n), dim3(INP_SETUP_THREADS), 0, s, invalid, H, W,
                       (int *)workspace, L);
    hipLaunchKernelGGL(k_inp_compact, dim3(L.nch, (unsigned)n), dim3(INP_SETUP_THREADS), 0, s, invalid, H, W,
                       (int *)workspace, L);
    hipLaunchKernelGGL(k_inp_setup, dim3((unsigned)n), dim3(INP_SETUP_THREADS), 0, s, invalid, H, W, radius,
                       (int *)workspace, L, errors);
    hipLaunchKernelGGL(k_inp_march, dim3(INP_MARCH_BLOCKS, (unsigned)n), dim3(64 * MARCH_WAVES), 0, s, frames, H, W,
                       radius, (int *)workspace, L);
    MDX_CHECK_LAUNCH("mdx_inpaint_ns");
    return MDX_OK;
}

extern "C" int mdx_inpaint_ns(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                              void *workspace, mdx_stream_t stream) {
    return mdx_inpaint_ns_counted(frames, invalid, n, H, W, radius, workspace, nullptr, stream);
}
