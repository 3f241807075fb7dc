// Which packed-FP32 instruction forms change their results while another
// kernel's waves run 16-bit matrix instructions on the same CUs.
//
// tools/native/gn_repro.hip showed the library's GroupNorm statistics kernel,
// built with packed-FP32 forms, giving different results run to run beside a
// bare loop of v_mfma_f32_16x16x32_bf16 / _f16 (register operands only, no
// memory traffic) and never beside v_mfma_f32_16x16x4f32, nor when built
// without the packed forms.  Here each victim kernel runs one packed-FP32
// instruction form (inline asm, so the form is exactly the one named) in a
// dependent chain over per-lane inputs, and every rep's output is compared
// bit for bit with the first rep's (run alone).  The victims' arithmetic is a
// pure function of the inputs: any difference is an execution fault.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/native/pk_hazard.hip -o tools/native/pk_hazard
// Run:   pk_hazard REPS BG [FIRST_FORM]   (BG: 0 none, 1 bf16 MFMA loop, 2 f16, 3 f32)
#include <hip/hip_runtime.h>

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

typedef float f2 __attribute__((ext_vector_type(2)));

// the forms: 0 v_pk_add_f32 (plain), 1 v_pk_add_f32 op_sel:[0,1] op_sel_hi:[1,0]
// (the GN partial's cross-half accumulate), 2 v_pk_add_f32 op_sel_hi:[1,0]
// neg_lo:[0,1] neg_hi:[0,1] (its broadcast subtract), 3 v_pk_mul_f32 (plain),
// 4 v_pk_fma_f32 (plain), 5 scalar v_add_f32 pair (control); round 5, the
// other forms the shipped library holds (tools/isa_lint.py lists them):
// 6 v_pk_add_f32 neg_lo:[0,1] neg_hi:[0,1] (subtract), 7 v_pk_add_f32 with an
// inline constant op_sel_hi:[1,0], 8 v_pk_fma_f32 constant op_sel_hi:[1,0,1],
// 9 v_pk_fma_f32 SGPR pair op_sel_hi:[1,0,1], 10 v_pk_mul_f32 SGPR pair,
// 11 v_pk_mul_f32 constant op_sel_hi:[1,0], 12 v_pk_mul_f32 SGPR pair
// op_sel_hi:[1,0], 13 v_pk_min_u16 / v_pk_max_u16 (plain, and an SGPR with
// op_sel_hi:[1,0]); 14 v_pk_minimum3_f16 (three VGPRs, no modifiers) over
// halves 0x6400 + v (v < 256: the normal f16 values 1024 + v), the form a
// 3-input minimum in the clean_frames morphology would use
constexpr int NFORMS = 15;

template <int F>
__global__ __launch_bounds__(256) void k_victim(const f2 *__restrict__ in, f2 *__restrict__ out, int iters,
                                                unsigned long long sc) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    f2 a = in[i], b = in[i + gridDim.x * 256];
    const f2 c = f2{0.9990234375f, 1.0009765625f};
    for (int k = 0; k < iters; ++k) {
        if constexpr (F == 0) {
            asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
        } else if constexpr (F == 1) {
            asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "+v"(a) : "v"(b));
        } else if constexpr (F == 2) {
            f2 d;
            asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
            a = d;
        } else if constexpr (F == 3) {
            asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(c));
        } else if constexpr (F == 4) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(c), "v"(b));
        } else if constexpr (F == 6) {
            asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(a) : "v"(b));
        } else if constexpr (F == 7) {
            asm volatile("v_pk_add_f32 %0, %0, 0.5 op_sel_hi:[1,0]" : "+v"(a));
            float x = a.x, y = a.y;
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(b.x));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(y) : "v"(b.y));
            a = f2{x, y};
        } else if constexpr (F == 8) {
            asm volatile("v_pk_fma_f32 %0, %0, 0.5, %1 op_sel_hi:[1,0,1]" : "+v"(a) : "v"(b));
        } else if constexpr (F == 9) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[1,0,1]" : "+v"(a) : "s"(sc), "v"(b));
        } else if constexpr (F == 10 || F == 11 || F == 12) {
            if constexpr (F == 10) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "s"(sc));
            if constexpr (F == 11) asm volatile("v_pk_mul_f32 %0, %0, 2.0 op_sel_hi:[1,0]" : "+v"(a));
            if constexpr (F == 12) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(a) : "s"(sc));
            float x = a.x, y = a.y;  // keep the magnitude and feed b in, scalar forms only
            asm volatile("v_mul_f32 %0, 0.5, %0" : "+v"(x));
            asm volatile("v_mul_f32 %0, 0.5, %0" : "+v"(y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(b.y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(y) : "v"(b.x));
            a = f2{x, y};
        } else if constexpr (F == 13) {
            unsigned x = __builtin_bit_cast(unsigned, a.x), y = __builtin_bit_cast(unsigned, a.y);
            const unsigned bx = __builtin_bit_cast(unsigned, b.x), by = __builtin_bit_cast(unsigned, b.y);
            const unsigned su = (unsigned)sc;
            asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x) : "v"(by));
            asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(y) : "v"(bx));
            asm volatile("v_pk_min_u16 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(y) : "s"(su));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(by));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(y) : "v"(bx));
            a = f2{__builtin_bit_cast(float, x), __builtin_bit_cast(float, y)};
        } else if constexpr (F == 14) {
            unsigned x = __builtin_bit_cast(unsigned, a.x), y = __builtin_bit_cast(unsigned, a.y);
            const unsigned bx = __builtin_bit_cast(unsigned, b.x), by = __builtin_bit_cast(unsigned, b.y);
            const unsigned p = (x & 0x00FF00FFu) | 0x64006400u, q = (by & 0x00FF00FFu) | 0x64006400u,
                           r = ((bx >> 5) & 0x00FF00FFu) | 0x64006400u;
            unsigned d;
            asm volatile("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(p), "v"(q), "v"(r));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(d));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(y) : "v"(d));
            a = f2{__builtin_bit_cast(float, x), __builtin_bit_cast(float, y)};
        } else {
            float x = a.x, y = a.y;
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(b.y));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(y) : "v"(b.x));
            a = f2{x, y};
        }
        // b drifts so the chain is not periodic; scalar multiplies (inline asm,
        // so no packed form appears outside the one under test)
        float bx = b.x, by = b.y;
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(bx) : "v"(c.x));
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(by) : "v"(c.y));
        b = f2{bx, by};
    }
    out[i] = a;
}

typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
template <int KIND>
__global__ __launch_bounds__(256) void k_bg_mfma(float *out, int iters) {
    f4v acc[4] = {};
    const float s = threadIdx.x * 1e-3f;
    b8v ba, bb;
    h8v ha, hb;
    for (int e = 0; e < 8; ++e) {
        ba[e] = (__bf16)(s + e);
        bb[e] = (__bf16)(1.f - s);
        ha[e] = (_Float16)(s + e);
        hb[e] = (_Float16)(1.f - s);
    }
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (KIND == 1) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, acc[q], 0, 0, 0);
            else if constexpr (KIND == 2) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[q], 0, 0, 0);
            else acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(s, s + 1.f, acc[q], 0, 0, 0);
        }
    float t = 0.f;
    for (int q = 0; q < 4; ++q) t += acc[q][0] + acc[q][3];
    if (t == 12345.f) out[threadIdx.x] = t;  // keep the loop
}

template <int F>
static void launch(const f2 *in, f2 *out, int blocks, int iters, hipStream_t s) {
    // SGPR operand: (0.9990234375f, 1.0009765625f) as one 64-bit pair
    const float c2[2] = {0.9990234375f, 1.0009765625f};
    unsigned long long sc;
    memcpy(&sc, c2, 8);
    hipLaunchKernelGGL(k_victim<F>, dim3(blocks), dim3(256), 0, s, in, out, iters, sc);
}
static void launch_form(int f, const f2 *in, f2 *out, int blocks, int iters, hipStream_t s) {
    switch (f) {
        case 0: launch<0>(in, out, blocks, iters, s); break;
        case 1: launch<1>(in, out, blocks, iters, s); break;
        case 2: launch<2>(in, out, blocks, iters, s); break;
        case 3: launch<3>(in, out, blocks, iters, s); break;
        case 4: launch<4>(in, out, blocks, iters, s); break;
        case 5: launch<5>(in, out, blocks, iters, s); break;
        case 6: launch<6>(in, out, blocks, iters, s); break;
        case 7: launch<7>(in, out, blocks, iters, s); break;
        case 8: launch<8>(in, out, blocks, iters, s); break;
        case 9: launch<9>(in, out, blocks, iters, s); break;
        case 10: launch<10>(in, out, blocks, iters, s); break;
        case 11: launch<11>(in, out, blocks, iters, s); break;
        case 12: launch<12>(in, out, blocks, iters, s); break;
        case 13: launch<13>(in, out, blocks, iters, s); break;
        default: launch<14>(in, out, blocks, iters, s); break;
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int bg = argc > 2 ? atoi(argv[2]) : 1;
    const int f0 = argc > 3 ? atoi(argv[3]) : 0;  // first form to run
    const int blocks = 512, iters = 256, n = blocks * 256;
    std::vector<f2> hin(2 * n);
    unsigned s = 777u;
    for (auto &v : hin) {
        s = s * 1664525u + 1013904223u;
        const float a = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
        s = s * 1664525u + 1013904223u;
        const float b = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
        v = f2{a, b};
    }
    f2 *in, *out;
    float *bgout;
    CK(hipMalloc(&in, 2 * n * sizeof(f2)));
    CK(hipMalloc(&out, n * sizeof(f2)));
    CK(hipMalloc(&bgout, 4096));
    CK(hipMemcpy(in, hin.data(), 2 * n * sizeof(f2), hipMemcpyHostToDevice));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    std::vector<f2> ref(n), got(n);
    printf("{\"reps\": %d, \"background\": %d", reps, bg);
    for (int f = f0; f < NFORMS; ++f) {
        int bad = 0, lanes_hi = 0, lanes_lo = 0;
        for (int r = 0; r <= reps; ++r) {
            if (r > 0 && bg == 1) hipLaunchKernelGGL(k_bg_mfma<1>, dim3(2048), dim3(256), 0, sb, bgout, 400 + 37 * (r % 5));
            if (r > 0 && bg == 2) hipLaunchKernelGGL(k_bg_mfma<2>, dim3(2048), dim3(256), 0, sb, bgout, 400 + 37 * (r % 5));
            if (r > 0 && bg == 3) hipLaunchKernelGGL(k_bg_mfma<3>, dim3(2048), dim3(256), 0, sb, bgout, 400 + 37 * (r % 5));
            launch_form(f, in, out, blocks, iters, sa);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(r == 0 ? ref.data() : got.data(), out, n * sizeof(f2), hipMemcpyDeviceToHost));
            if (r == 0) continue;
            if (memcmp(ref.data(), got.data(), n * sizeof(f2))) {
                ++bad;
                const unsigned *ru = reinterpret_cast<const unsigned *>(ref.data());
                const unsigned *gu = reinterpret_cast<const unsigned *>(got.data());
                for (int i = 0; i < n; ++i) {
                    lanes_lo += ru[2 * i] != gu[2 * i];
                    lanes_hi += ru[2 * i + 1] != gu[2 * i + 1];
                }
            }
        }
        printf(", \"form%d\": {\"reps_differing\": %d, \"lo_values_differing\": %d, \"hi_values_differing\": %d}", f, bad,
               lanes_lo, lanes_hi);
    }
    printf("}\n");
    return 0;
}
