// HBM access-shape probe (round 5): is the 1x1 layers' ~3.8 TB/s a property of the MFMA lane layout's access shape?
// The streaming 1x1 kernels load / store straight in the 32x32 MFMA layout: lane (r, h) of a wave touches pixel r's
// row at 16-byte pieces 32 bytes apart, so one wave-instruction covers 32 pixel rows x 32 bytes. Same bytes moved by
//   coalesced: every wave-instruction covers 1 KB contiguous (4 lanes per 64-byte piece... 64 lanes x 16 B in a row)
//   mfma     : the streaming kernels' pattern (X [P][64] read, R [P][128] read, Y [P][128] written; P = 262144)
//   rows64   : 64 bytes per pixel row per instruction (4 lanes per row, 16 rows)
// Standalone:  hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/access_probe.hip -o scripts/access_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int P = 262144;

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// coalesced: thread i handles Y float4 i (P*32 of them): R float4 i, X float4 i/2
__global__ __launch_bounds__(256) void k_coalesced(const float4* X, const float4* R, float4* Y) {
    const long long n = (long long)P * 32;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        Y[i] = add4(R[i], X[i >> 1]);
    }
}

// mfma layout: wave tile = 32 pixels; lane (r, h): X pieces 16s + 8h + 4u (floats) for s<4, u<2;
// R / Y pieces 32t + 8q + 4h for t<4, q<4
__global__ __launch_bounds__(256) void k_mfma(const float* X, const float* R, float* Y) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 31, lh = lane >> 5;
    const int ntile = P / 32;
    for (int tile = blockIdx.x * 4 + wave; tile < ntile; tile += gridDim.x * 4) {
        const long long p = tile * 32LL + lr;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int u = 0; u < 2; ++u) acc = add4(acc, *reinterpret_cast<const float4*>(X + p * 64 + 16 * s + 8 * lh + 4 * u));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long o = p * 128 + 32 * t + 8 * q + 4 * lh;
                *reinterpret_cast<float4*>(Y + o) = add4(*reinterpret_cast<const float4*>(R + o), acc);
            }
    }
}

// rows64: 4 lanes per pixel row (64 B contiguous), 16 rows per wave-instruction
__global__ __launch_bounds__(256) void k_rows64(const float* X, const float* R, float* Y) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane >> 2, lc = lane & 3;
    const int ntile = P / 16;
    for (int tile = blockIdx.x * 4 + wave; tile < ntile; tile += gridDim.x * 4) {
        const long long p = tile * 16LL + lr;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = add4(acc, *reinterpret_cast<const float4*>(X + p * 64 + 16 * s + 4 * lc));
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const long long o = p * 128 + 16 * s + 4 * lc;
            *reinterpret_cast<float4*>(Y + o) = add4(*reinterpret_cast<const float4*>(R + o), acc);
        }
    }
}

int main() {
    float *X, *R, *Y;
    CK(hipMalloc(&X, (size_t)P * 64 * 4));
    CK(hipMalloc(&R, (size_t)P * 128 * 4));
    CK(hipMalloc(&Y, (size_t)P * 128 * 4));
    CK(hipMemset(X, 0, (size_t)P * 64 * 4));
    CK(hipMemset(R, 0, (size_t)P * 128 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)P * (64 + 128 + 128) * 4;
    for (int grid : {512, 1024, 2048, 8192}) {
        for (int k = 0; k < 3; ++k) {
            auto run = [&]() {
                if (k == 0) hipLaunchKernelGGL(k_coalesced, dim3(grid), dim3(256), 0, 0, (const float4*)X, (const float4*)R, (float4*)Y);
                if (k == 1) hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, X, R, Y);
                if (k == 2) hipLaunchKernelGGL(k_rows64, dim3(grid), dim3(256), 0, 0, X, R, Y);
            };
            for (int i = 0; i < 5; ++i) run();
            CK(hipEventRecord(e0));
            for (int i = 0; i < 50; ++i) run();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / 50;
            printf("grid %5d %-10s %7.1f us  %6.0f GB/s\n", grid, k == 0 ? "coalesced" : k == 1 ? "mfma" : "rows64", us,
                   bytes / us / 1e3);
        }
    }
    return 0;
}
