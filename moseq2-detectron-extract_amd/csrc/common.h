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
bool winograd_planes_enabled();  // the model runs Winograd GEMMs on k_gemm_x6 (MDX_WINO_X6 set)
// weights of the next split-plane conv launch on this thread as bf16 planes
// (mdx_split_x6 layout), or null; the model handle sets it around a layer
void x3_weight_planes(const void *planes);

// prep_raw_frames' kernel (frameops.hip); bits (or null): the invalid pixels
// ORed into the inpaint workspace's bit images (zero at rest; padded rows of
// wpr words, frame stride bits_fstride words)
int launch_prep(const int16_t *raw, int64_t n, int H, int W, const double *bg, const uint8_t *roi, int y0, int y1,
                int x0, int x1, int flags, double vmin, double vmax, uint8_t *out, uint8_t *invalid, uint32_t *bits,
                int64_t bits_fstride, int wpr, hipStream_t s);

// the kernel-selection policy in force on this thread (include/mdx.h,
// mdx_policy): the running model handle's inside its entry points
// (PolicyScope), else the thread's own (mdx_policy_set)
const mdx_policy &pol();
struct PolicyScope {
    const mdx_policy *prev;
    explicit PolicyScope(const mdx_policy *p);
    ~PolicyScope();
    PolicyScope(const PolicyScope &) = delete;
    PolicyScope &operator=(const PolicyScope &) = delete;
};

}  // namespace mdx
