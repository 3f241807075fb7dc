// Shared helpers of the mdx HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/mdx.h"

namespace mdx {

void set_error(const char *fmt, ...);
inline hipStream_t as_stream(mdx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-error check after every kernel launch (asynchronous errors surface
// at the next synchronising call made by the caller).
#define MDX_CHECK_LAUNCH(name)                                                       \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) {                                                      \
            ::mdx::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));  \
            return MDX_EHIP;                                                         \
        }                                                                            \
    } while (0)

#define MDX_REQUIRE(cond, ...)                  \
    do {                                        \
        if (!(cond)) {                          \
            ::mdx::set_error(__VA_ARGS__);      \
            return MDX_EINVAL;                  \
        }                                       \
    } while (0)

#define MDX_HIP(call)                                                                 \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            ::mdx::set_error("%s: %s", #call, hipGetErrorString(e_));                 \
            return MDX_EHIP;                                                          \
        }                                                                             \
    } while (0)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Profiling hook of the model handle (mdx_model_profile): while set on the
// calling thread, mdx_conv3x3_winograd records ev[0] / ev[1] around its input
// transform, ev[2] / ev[3] around the batched GEMM and ev[4] / ev[5] around
// the output transform, and stores the GEMM's MDX_CONV_KERNEL_* id.
struct WinoProbe {
    hipEvent_t ev[6];
    int gemm_kernel;
};
void wino_probe(WinoProbe *p);
WinoProbe *wino_probe_current();
// the kernel id / K slices mdx_conv2d_last_plan reports for this thread
void set_last_plan(int kernel, int ksplit);
// the fp32 Winograd input transform with two channels per thread (wino_fused.hip,
// built without packed FP32): grid (tiles, channel pairs / bd), bd threads
void launch_wino_in2(int m, dim3 grid, unsigned bd, hipStream_t s, const float *x, int N, int H, int W, int C,
                     int TH, int TW, float *V);
bool winograd_planes_enabled();  // the model runs Winograd GEMMs on k_gemm_x6 (MDX_WINO_X6 set)
// weights of the next split-plane conv launch on this thread as bf16 planes
// (mdx_split_x6 layout), or null; the model handle sets it around a layer
void x3_weight_planes(const void *planes);

}  // namespace mdx
