// Register-only MFMA throughput probe: every wave runs NITER x 32 independent
// v_mfma_f32_16x16x32_f16 on operands loaded once from memory (random or
// zero), 8 waves per CU.  Prints TFLOP/s.  Build: hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_peak(const half8 *src, float *out, int niter) {
    const int lane = threadIdx.x & 63;
    half8 a[4], b[4];
    for (int i = 0; i < 4; ++i) {
        a[i] = src[(blockIdx.x * 8 + i) * 64 + lane];
        b[i] = src[(blockIdx.x * 8 + 4 + i) * 64 + lane];
    }
    float4v acc[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0, 0, 0, 0};
    for (int it = 0; it < niter; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[i], a[j], acc[i][j], 0, 0, 0);
    }
    float s = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 4, threads = 512, niter = 4000;
    const size_t n = (size_t)blocks * 8 * 64;
    std::vector<_Float16> h(n * 8);
    for (int mode = 0; mode < 2; ++mode) {
        for (size_t i = 0; i < h.size(); ++i)
            h[i] = mode == 0 ? (_Float16)0.f : (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
        half8 *d;
        float *o;
        hipMalloc(&d, n * 16);
        hipMalloc(&o, (size_t)blocks * threads * 4);
        hipMemcpy(d, h.data(), n * 16, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(threads), 0, 0, d, o, 10);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(threads), 0, 0, d, o, niter);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = (double)blocks * (threads / 64) * niter * 32 * 16384.0;
        printf("%s operands: %.1f TFLOP/s (%.3f ms)\n", mode == 0 ? "zero" : "random", flops / ms / 1e9, ms);
        hipFree(d);
        hipFree(o);
    }
    return 0;
}
