// Minimal reproduction of the fp16 GroupNorm statistics that changed from
// run to run under concurrency when model_ops.hip was compiled with the
// packed-FP32 VALU forms ("Concurrency").  The GroupNorm
// kernels are the library's own (model_ops.hip is included, not copied);
// the host loop launches k_gn_partial + k_gn_final on stream A over the same
// fp16 input again and again while stream B runs a background load, and
// compares every result with the first one bit for bit.  A pure function
// of its input must never change; any change means a race, a read of
// uninitialised memory or an execution hazard.
//
// Build (two binaries, the flag the only difference):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I. -munsafe-fp-atomics \
//     tools/native/gn_repro.hip -o gn_repro_pk
//   ... -Xclang -target-feature -Xclang -packed-fp32-ops ... -o gn_repro_nopk
// Run: gn_repro_<v> REPS BG [H W] (BG bits: 1 VALU loop, 2 HBM copy, 4 the
// library's fp16 3x3 conv (LDS-DMA k_convg), 8 its fp32 3x3 conv (k_conv_sb),
// both from libmdx.so through dlopen, 16 a packed-FP32 VALU loop (two-lane
// vector FMAs / adds with lane swaps), 128 / 256 / 512 f16 / bf16 / f32
// MFMA loops, 32 the GN statistics kernels on a
// second 8 x 112 x 128 map; the FPN level maps of a 448x512 input: 112x128,
// 56x64, 28x32, 14x16)
#include "moseq2-detectron-extract_amd/csrc/model_ops.hip"
namespace mdx {
void set_error(const char *, ...) {}
}

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

// background VALU load: long dependent FMA chains on registers
__global__ __launch_bounds__(256) void k_bg_valu(float *out, int iters) {
    float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-4f, c = 1.0001f;
    for (int i = 0; i < iters; ++i) {
        a = fmaf(a, c, b);
        b = fmaf(b, c, a);
    }
    if (a == 12345.f) out[threadIdx.x] = a + b;  // keep the loop
}

// background packed-FP32 load: two-lane vectors (v_pk_fma_f32 / v_pk_add_f32
// with op_sel lane swaps in the packed build, scalar FMAs in the other)
typedef float f2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_bg_pk(float *out, int iters) {
    f2v a = {threadIdx.x * 1e-3f, 0.5f}, b = {blockIdx.x * 1e-4f, 0.25f}, c = {1.0001f, 0.9999f};
    for (int i = 0; i < iters; ++i) {
        a = a * c + b;
        b = b * c + a.yx;
        a = a + b.xx;
    }
    if (a.x == 12345.f) out[threadIdx.x] = a.y + b.x + b.y;  // keep the loop
}

// background matrix-core loads: chains of 16x16x32 f16 / bf16 or 16x16x4 f32
// MFMAs on register operands (4 independent accumulators per wave)
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
template <int KIND>
__global__ __launch_bounds__(256) void k_bg_mfma(float *out, int iters) {
    f4v acc[4] = {};
    const float s = threadIdx.x * 1e-3f;
    h8v ha, hb;
    b8v ba, bb;
    for (int e = 0; e < 8; ++e) {
        ha[e] = (_Float16)(s + e);
        hb[e] = (_Float16)(1.f - s);
        ba[e] = (__bf16)(s + e);
        bb[e] = (__bf16)(1.f - s);
    }
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (KIND == 0) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[q], 0, 0, 0);
            else if constexpr (KIND == 1) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, acc[q], 0, 0, 0);
            else acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(s, s + 1.f, acc[q], 0, 0, 0);
        }
    float t = 0.f;
    for (int q = 0; q < 4; ++q) t += acc[q][0] + acc[q][3];
    if (t == 12345.f) out[threadIdx.x] = t;  // keep the loop
}

// background HBM load: streaming copy
__global__ __launch_bounds__(256) void k_bg_copy(const float4 *src, float4 *dst, long long n) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        dst[i] = src[i];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int bg = argc > 2 ? atoi(argv[2]) : 3;
    const int H = argc > 3 ? atoi(argv[3]) : 112, W = argc > 4 ? atoi(argv[4]) : 128;
    const int N = 4, C = 256, G = 32, HW = H * W;
    const int nch = (HW + mdx::GN_CHUNK_PIX - 1) / mdx::GN_CHUNK_PIX;
    const size_t nx = (size_t)N * HW * C;
    std::vector<_Float16> hx(nx);
    unsigned s = 12345u;
    for (size_t i = 0; i < nx; ++i) {
        s = s * 1664525u + 1013904223u;
        hx[i] = (_Float16)(((s >> 8) & 0xffff) / 65536.0f * 8.0f - 3.0f);
    }
    _Float16 *x, *up, *y;
    float *part, *stats, *bgout, *gamma, *beta;
    float4 *bsrc, *bdst;
    const long long nbg = 64ll << 20;  // 1 GiB each way
    CK(hipMalloc(&x, nx * 2));
    // the FPN top-down form of the apply kernel: y = (GN(x) + up2(up)) / 2
    const size_t nup = nx / 4;
    std::vector<_Float16> hu(nup);
    for (size_t i = 0; i < nup; ++i) {
        s = s * 1664525u + 1013904223u;
        hu[i] = (_Float16)(((s >> 8) & 0xffff) / 65536.0f * 6.0f - 2.0f);
    }
    std::vector<float> hg(C), hb(C);
    for (int c = 0; c < C; ++c) {
        hg[c] = 0.8f + 0.001f * c;
        hb[c] = -0.1f + 0.0005f * c;
    }
    CK(hipMalloc(&up, nup * 2));
    CK(hipMalloc(&y, nx * 2));
    CK(hipMalloc(&gamma, C * 4));
    CK(hipMalloc(&beta, C * 4));
    CK(hipMemcpy(up, hu.data(), nup * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(gamma, hg.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(beta, hb.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&part, (size_t)N * G * nch * 3 * 4));
    CK(hipMalloc(&stats, (size_t)N * G * 2 * 4));
    CK(hipMalloc(&bgout, 4096));
    CK(hipMalloc(&bsrc, nbg * 16));
    CK(hipMalloc(&bdst, nbg * 16));
    CK(hipMemset(bsrc, 0, nbg * 16));
    CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
    // background convs: the library's own kernels (fp16 and fp32 3x3, 8 x 112 x 128 x 256)
    typedef int (*conv_fn)(const void *, int, int, int, int, const void *, const float *, int, int, int, int, int,
                           const void *, int, int, int, int, void *, void *);
    conv_fn conv = nullptr;
    void *cx = nullptr, *cw = nullptr, *co = nullptr;
    if (bg & 12) {
        void *lib = dlopen("moseq2-detectron-extract_amd/libmdx.so", RTLD_NOW | RTLD_LOCAL);
        if (!lib) {
            fprintf(stderr, "dlopen: %s\n", dlerror());
            return 2;
        }
        conv = (conv_fn)dlsym(lib, "mdx_conv2d");
        // BG_CONV_REG=1: the register-staged fp16 kernels (k_conv_sb / k_conv_sbg)
        // instead of the LDS-DMA tiles (large tiles and the 256x256 split-K off)
        if (getenv("BG_CONV_REG")) {
            typedef int (*set1_fn)(int);
            typedef int (*set2_fn)(int, int);
            ((set1_fn)dlsym(lib, "mdx_conv_set_large_tiles"))(0);
            ((set2_fn)dlsym(lib, "mdx_conv_set_split256"))(0, 18);
        }
        const size_t nin = 8ull * 112 * 128 * 256;
        CK(hipMalloc(&cx, nin * 4));
        CK(hipMalloc(&co, nin * 4));
        CK(hipMalloc(&cw, 256ull * 2304 * 4));
        CK(hipMemset(cx, 0x3c, nin * 4));
        CK(hipMemset(cw, 0x1c, 256ull * 2304 * 4));
    }
    // background GN: the same kernels over a second, larger map
    // (GN_BG="H W N": another map size, e.g. "14 16 4" = the level-5 map of a 4-image batch)
    int BH = 112, BW = 128, BN_ = 8;
    if (const char *e = getenv("GN_BG")) sscanf(e, "%d %d %d", &BH, &BW, &BN_);
    const int bnch = (BH * BW + mdx::GN_CHUNK_PIX - 1) / mdx::GN_CHUNK_PIX;
    _Float16 *bx = nullptr;
    float *bpart = nullptr, *bstats = nullptr;
    if (bg & 32) {
        const size_t nb = (size_t)BN_ * BH * BW * C;
        std::vector<_Float16> hb2(nb);
        for (size_t i = 0; i < nb; ++i) {
            s = s * 1664525u + 1013904223u;
            hb2[i] = (_Float16)(((s >> 8) & 0xffff) / 65536.0f * 4.0f - 1.0f);
        }
        CK(hipMalloc(&bx, nb * 2));
        CK(hipMemcpy(bx, hb2.data(), nb * 2, hipMemcpyHostToDevice));
        CK(hipMalloc(&bpart, (size_t)BN_ * G * bnch * 3 * 4));
        CK(hipMalloc(&bstats, (size_t)BN_ * G * 2 * 4));
    }
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    const size_t npart = (size_t)N * G * nch * 3, nstat = (size_t)N * G * 2;
    std::vector<float> p0(npart), s0(nstat), p1(npart), s1(nstat);
    std::vector<uint16_t> y0(nx), y1(nx);
    int bad_part = 0, bad_stat = 0, bad_y = 0;
    for (int r = 0; r <= reps; ++r) {
        CK(hipMemsetAsync(part, 0xff, npart * 4, sa));  // stale partials would show as NaN
        if (r > 0 && (bg & 1))
            hipLaunchKernelGGL(k_bg_valu, dim3(2048), dim3(256), 0, sb, bgout, 20000 + 997 * (r % 7));
        if (r > 0 && (bg & 2)) hipLaunchKernelGGL(k_bg_copy, dim3(4096), dim3(256), 0, sb, bsrc, bdst, nbg);
        // 128 / 256 / 512: f16 / bf16 / f32 MFMA loops
        if (r > 0 && (bg & 128))
            hipLaunchKernelGGL(k_bg_mfma<0>, dim3(2048), dim3(256), 0, sb, bgout, 2000 + 97 * (r % 7));
        if (r > 0 && (bg & 256))
            hipLaunchKernelGGL(k_bg_mfma<1>, dim3(2048), dim3(256), 0, sb, bgout, 2000 + 97 * (r % 7));
        if (r > 0 && (bg & 512))
            hipLaunchKernelGGL(k_bg_mfma<2>, dim3(2048), dim3(256), 0, sb, bgout, 2000 + 97 * (r % 7));
        if (r > 0 && (bg & 16))
            hipLaunchKernelGGL(k_bg_pk, dim3(2048), dim3(256), 0, sb, bgout, 20000 + 997 * (r % 7));
        const int gn_bg_launches = getenv("GN_BG_LAUNCHES") ? atoi(getenv("GN_BG_LAUNCHES")) : 4;
        for (int k = 0; r > 0 && (bg & 32) && k < gn_bg_launches + r % 5; ++k) {
            hipLaunchKernelGGL(mdx::k_gn_partial<_Float16>, dim3(bnch, BN_), dim3(256), 0, sb, bx, BH * BW, C, G, bpart);
            hipLaunchKernelGGL(mdx::k_gn_final, dim3((BN_ * G + 3) / 4), dim3(256), 0, sb, bpart, BN_ * G, bnch, 1e-5f,
                               bstats);
        }
        for (int k = 0; r > 0 && (bg & 12) && k < 1 + r % 3; ++k) {
            const int f16 = (bg & 4) ? 1 : 0;
            if (conv(cx, 8, 112, 128, 256, cw, nullptr, 256, 3, 3, 1, 1, nullptr, 0, 0, f16, f16, co, sb) != 0) {
                fprintf(stderr, "background conv failed\n");
                return 2;
            }
        }
        hipLaunchKernelGGL(mdx::k_gn_partial<_Float16>, dim3(nch, N), dim3(256), 0, sa, x, HW, C, G, part);
        hipLaunchKernelGGL(mdx::k_gn_final, dim3((N * G + 3) / 4), dim3(256), 0, sa, part, N * G, nch, 1e-5f, stats);
        hipLaunchKernelGGL(mdx::k_gn_apply<_Float16>, dim3(2048), dim3(256), 0, sa, x, N, H, W, C, G, stats, gamma, beta,
                           up, 2, y);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<float> &pp = r == 0 ? p0 : p1, &ss = r == 0 ? s0 : s1;
        CK(hipMemcpy(pp.data(), part, npart * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ss.data(), stats, nstat * 4, hipMemcpyDeviceToHost));
        std::vector<uint16_t> &yy = r == 0 ? y0 : y1;
        CK(hipMemcpy(yy.data(), y, nx * 2, hipMemcpyDeviceToHost));
        if (r == 0) continue;
        if (memcmp(y0.data(), y1.data(), nx * 2)) {
            ++bad_y;
            if (bad_y <= 3) {
                size_t nd = 0, first = (size_t)-1;
                for (size_t i = 0; i < nx; ++i)
                    if (y0[i] != y1[i]) {
                        if (first == (size_t)-1) first = i;
                        ++nd;
                    }
                const size_t c = first % C, pix = first / C;
                printf("rep %d: %zu outputs differ; first: image %zu pixel %zu channel %zu\n", r, nd, pix / HW,
                       pix % HW, c);
            }
        }
        if (memcmp(p0.data(), p1.data(), npart * 4)) {
            ++bad_part;
            if (bad_part <= 3) {
                int nd = 0, first = -1;
                for (size_t i = 0; i < npart; ++i)
                    if (memcmp(&p0[i], &p1[i], 4)) {
                        if (first < 0) first = (int)i;
                        ++nd;
                    }
                // partial index -> (image, group, chunk, field)
                const int f = first % 3, ch = (first / 3) % nch, g = (first / 3 / nch) % G, n = first / 3 / nch / G;
                printf("rep %d: %d partial floats differ; first: image %d group %d chunk %d field %d: %.9g vs %.9g\n",
                       r, nd, n, g, ch, f, p0[first], p1[first]);
            }
        }
        if (memcmp(s0.data(), s1.data(), nstat * 4)) ++bad_stat;
    }
    printf("{\"reps\": %d, \"background\": %d, \"partials_differ\": %d, \"stats_differ\": %d, \"apply_differ\": %d}\n",
           reps, bg, bad_part, bad_stat, bad_y);
    return 0;
}
