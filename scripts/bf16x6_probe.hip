// Probe: is an fp32-accurate GEMM on the bf16 MFMA (each fp32 operand split into three bf16 pieces, the six cross
// products with i + j <= 2, fp32 accumulation) faster than the native fp32 MFMA (v_mfma_f32_32x32x2_f32) at the
// shapes of the fp32 train step's convs? Standalone (not part of the library): times both GEMM cores with the same
// 128 x 128 block tiling and reports the error of each against an fp64 host reference on sampled outputs.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/bf16x6_probe.hip -o scripts/bf16x6_probe && scripts/bf16x6_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = 128, BN = 128, BK = 32;  // block tile; 4 waves as 2 x 2, each 64 x 64 (2 x 2 MFMA tiles)

// ---- native fp32 MFMA (the library's conv main loop, simplified): K chunks of 32 floats staged in LDS
__global__ __launch_bounds__(256) void gemm_f32(const float* A, const float* B, float* C, int M, int N, int K) {
    __shared__ float As[BM][BK + 4], Bs[BN][BK + 4];  // A row-major [m][k], B as [n][k]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    floatx16 acc[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int k0 = 0; k0 < K; k0 += BK) {
        for (int e = tid; e < BM * BK / 4; e += 256) {
            const int r = e / (BK / 4), c = 4 * (e % (BK / 4));
            *reinterpret_cast<float4*>(&As[r][c]) = *reinterpret_cast<const float4*>(&A[(long long)(m0 + r) * K + k0 + c]);
            *reinterpret_cast<float4*>(&Bs[r][c]) = *reinterpret_cast<const float4*>(&B[(long long)(n0 + r) * K + k0 + c]);
        }
        __syncthreads();
        for (int kk = 0; kk < BK; kk += 2) {
            float a[2], b[2];
            for (int i = 0; i < 2; ++i) a[i] = As[wm * 64 + 32 * i + lr][kk + lh];
            for (int j = 0; j < 2; ++j) b[j] = Bs[wn * 64 + 32 * j + lr][kk + lh];
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int n = n0 + wn * 64 + 32 * j + lr;
                C[(long long)m * N + n] = acc[i][j][r];
            }
}

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r1 = x - (float)h;
    m = (__bf16)r1;
    l = (__bf16)(r1 - (float)m);
}

// ---- bf16x6: the same tiling; the staged chunk is split into hi / mid / lo bf16 planes in LDS
constexpr int PB = BK + 8;  // bf16 row pitch (80 B)
__global__ __launch_bounds__(256) void gemm_bf16x6(const float* A, const float* B, float* C, int M, int N, int K) {
    __shared__ __bf16 Ap[3][BM][PB], Bp[3][BN][PB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    floatx16 acc[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int k0 = 0; k0 < K; k0 += BK) {
        for (int e = tid; e < BM * BK / 4; e += 256) {
            const int r = e / (BK / 4), c = 4 * (e % (BK / 4));
            const float4 a = *reinterpret_cast<const float4*>(&A[(long long)(m0 + r) * K + k0 + c]);
            const float4 b = *reinterpret_cast<const float4*>(&B[(long long)(n0 + r) * K + k0 + c]);
            const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
            for (int u = 0; u < 4; ++u) {
                split3(av[u], Ap[0][r][c + u], Ap[1][r][c + u], Ap[2][r][c + u]);
                split3(bv[u], Bp[0][r][c + u], Bp[1][r][c + u], Bp[2][r][c + u]);
            }
        }
        __syncthreads();
        for (int kk = 0; kk < BK; kk += 16) {
            bf16x8 a[3][2], b[3][2];
            for (int p = 0; p < 3; ++p) {
                for (int i = 0; i < 2; ++i) a[p][i] = *reinterpret_cast<const bf16x8*>(&Ap[p][wm * 64 + 32 * i + lr][kk + 8 * lh]);
                for (int j = 0; j < 2; ++j) b[p][j] = *reinterpret_cast<const bf16x8*>(&Bp[p][wn * 64 + 32 * j + lr][kk + 8 * lh]);
            }
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) {
                    // small terms first (fp32 accumulation of six exact bf16 x bf16 products)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int n = n0 + wn * 64 + 32 * j + lr;
                C[(long long)m * N + n] = acc[i][j][r];
            }
}

int main(int argc, char** argv) {
    const int M = 262144, N = 128, K = 576;  // the 128^2 3x3 64->64 conv of the bs16 step as a GEMM (M px, K = 9*64)
    std::vector<float> hA((size_t)M * K), hB((size_t)N * K);
    std::mt19937 g(1);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& v : hA) v = u(g);
    for (auto& v : hB) v = u(g) * 0.05f;
    float *dA, *dB, *dC;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB, hB.size() * 4));
    CK(hipMalloc(&dC, (size_t)M * N * 4));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(M / BM, N / BN);
    std::vector<float> hC((size_t)M * N);
    for (int which = 0; which < 2; ++which) {
        auto run = [&]() {
            if (which == 0) hipLaunchKernelGGL(gemm_f32, grid, dim3(256), 0, 0, dA, dB, dC, M, N, K);
            else hipLaunchKernelGGL(gemm_bf16x6, grid, dim3(256), 0, 0, dA, dB, dC, M, N, K);
        };
        for (int i = 0; i < 5; ++i) run();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) run();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        CK(hipMemcpy(hC.data(), dC, hC.size() * 4, hipMemcpyDeviceToHost));
        double maxrel = 0.0, sumsq = 0.0, sumref = 0.0;
        for (int s = 0; s < 4096; ++s) {
            const int m = (int)((s * 2654435761u) % (unsigned)M), n = (s * 40503) % N;
            double ref = 0.0, mag = 0.0;
            for (int k = 0; k < K; ++k) {
                ref += (double)hA[(size_t)m * K + k] * (double)hB[(size_t)n * K + k];
                mag += std::fabs((double)hA[(size_t)m * K + k] * (double)hB[(size_t)n * K + k]);
            }
            const double err = std::fabs((double)hC[(size_t)m * N + n] - ref);
            maxrel = std::max(maxrel, err / mag);
            sumsq += err * err;
            sumref += ref * ref;
        }
        const double tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12;
        printf("%s: %.1f us  %.1f TFLOP/s (fp32-equivalent)  err vs fp64: max %.2e of sum|a*b|, normwise %.2e\n",
               which == 0 ? "fp32 MFMA  " : "bf16x6 MFMA", ms * 1e3, tf, maxrel, std::sqrt(sumsq / sumref));
    }
    return 0;
}
