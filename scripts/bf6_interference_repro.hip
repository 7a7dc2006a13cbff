// Minimal reproducer of the bf16x6 cross-kernel interference (DESIGN §4 "Cross-kernel interference").
//
// One C-ABI call of the library (hyres_conv_forward: 3x3 64->64 conv, 2 x 256 x 256, bf16x6 weight-resident kernel)
// on stream A, small victim kernels of this file on stream B, each checked bit for bit against its own result
// computed alone. hyres_conv_tuning key 9 selects the conv's register allocation: 0 = 224 VGPRs per wave (2 waves
// per SIMD leave a 64-VGPR hole another kernel's wave can take), 1 = the shipped 256 (no hole).
//
// Victims (each thread handles one float4 = 4 channels of one pixel, so lanes 16q..16q+15 of a wave are 16
// consecutive float4s of one pixel's 64 channels):
//   bilin   x1/2 bilinear resize, compiler-formed packed fp32 (v_pk_mul_f32 / v_pk_fma_f32), = the library's
//   scalar  the same, every multiply / fma forced to the unpacked v_mul_f32 / v_fma_f32 by inline asm
//   copy    float4 load -> float4 store of the same registers (no VALU on the data)
//   copy4   four float4 loads (the bilinear's four taps) -> stored unmodified to four outputs
//   lib bilinear  the library's own hyres_bilinear_fwd (bilinear_fwd_kernel<4,false>), the kernel the model runs
//
// For each victim: wrong float4 components, how many 16-lane groups ("events") they fall in, which lane group of
// the wave (0..3), which float4 component, and (bilinear) whether the error equals one 0.25-weighted tap lost.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude scripts/bf6_interference_repro.hip \
//       -Lhyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip -lhyres_hip \
//       -Wl,-rpath,'$ORIGIN/../hyres-residual-enhanced-hybrid-image-compression_amd/hyres_hip' \
//       -o scripts/bf6_interference_repro
//   scripts/bf6_interference_repro [reps] [delay_us between the conv's launch and the victims'] [wres|native|igemm|ru|wg1x1|wghalo|native-b6v]
//
// native-b6v (round 6, the r5v pairing of profiles/r5v_refine_determinism_fail.log): the native fp32-MFMA weight-resident
// 3x3 as the hog and, as an extra victim, a bf16x6 conv of the library (3x3 64->64 on the bf16x6 implicit GEMM,
// conv_fwd_b6_kernel: hyres_conv_tuning key 7 = 1 and key 14 = 0 while the victim is enqueued, key 7 = 0 and key 14 = 1
// while the hog is) — the mixed-GEMM configuration in which the native kernel's hole was hit.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "hyres_hip.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)
#define CH(x)                                                                         \
    do {                                                                              \
        int r_ = (x);                                                                 \
        if (r_ != 0) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hyres_last_error_string()); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ float mul_s(float a, float b) {
    float r;
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fma_s(float a, float b, float c) {
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// x [2][256][256][64] -> y [2][128][128][64] (KIND 0, 1); KIND 2: y = x's first quarter copied; KIND 3: the four
// taps of each output copied into y[0..3] planes. One block row per output row, 256 threads, thread = float4.
template <int KIND>
__global__ __launch_bounds__(256) void victim(const float* __restrict__ x, float* __restrict__ y) {
    const int row = blockIdx.y, b = row / 128, oh = row % 128;
    const int i = blockIdx.x * 256 + threadIdx.x;  // < 2048 = 128 pixels x 16 float4
    const int ow = i >> 4, c = (i & 15) * 4;
    const long long o = ((long long)row * 128 + ow) * 64 + c;
    if constexpr (KIND == 2) {
        *reinterpret_cast<float4*>(y + o) = *reinterpret_cast<const float4*>(x + o);
        return;
    }
    const long long r0 = ((long long)(b * 256 + 2 * oh) * 256 + 2 * ow) * 64 + c, r1 = r0 + 256 * 64;
    const float4 a = *reinterpret_cast<const float4*>(x + r0), q = *reinterpret_cast<const float4*>(x + r0 + 64);
    const float4 r = *reinterpret_cast<const float4*>(x + r1), d = *reinterpret_cast<const float4*>(x + r1 + 64);
    if constexpr (KIND == 3) {
        const long long n = 2LL * 128 * 128 * 64;
        *reinterpret_cast<float4*>(y + o) = a;
        *reinterpret_cast<float4*>(y + n + o) = q;
        *reinterpret_cast<float4*>(y + 2 * n + o) = r;
        *reinterpret_cast<float4*>(y + 3 * n + o) = d;
        return;
    }
    // the library kernel's arithmetic for scale 2: every weight 0.5 (lh0 = lh1 = lw0 = lw1)
    const float lh0 = 0.5f + (float)(row >> 30), lh1 = 0.5f, lw0 = 0.5f + (float)(i >> 30), lw1 = 0.5f;
    float4 v;
    if constexpr (KIND == 0) {
        v.x = lh0 * (lw0 * a.x + lw1 * q.x) + lh1 * (lw0 * r.x + lw1 * d.x);
        v.y = lh0 * (lw0 * a.y + lw1 * q.y) + lh1 * (lw0 * r.y + lw1 * d.y);
        v.z = lh0 * (lw0 * a.z + lw1 * q.z) + lh1 * (lw0 * r.z + lw1 * d.z);
        v.w = lh0 * (lw0 * a.w + lw1 * q.w) + lh1 * (lw0 * r.w + lw1 * d.w);
    } else {
        v.x = fma_s(lh1, fma_s(lw0, r.x, mul_s(lw1, d.x)), mul_s(lh0, fma_s(lw0, a.x, mul_s(lw1, q.x))));
        v.y = fma_s(lh1, fma_s(lw0, r.y, mul_s(lw1, d.y)), mul_s(lh0, fma_s(lw0, a.y, mul_s(lw1, q.y))));
        v.z = fma_s(lh1, fma_s(lw0, r.z, mul_s(lw1, d.z)), mul_s(lh0, fma_s(lw0, a.z, mul_s(lw1, q.z))));
        v.w = fma_s(lh1, fma_s(lw0, r.w, mul_s(lw1, d.w)), mul_s(lh0, fma_s(lw0, a.w, mul_s(lw1, q.w))));
    }
    *reinterpret_cast<float4*>(y + o) = v;
}

static double wall() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const char* KNAME[] = {"bilin(pk_f32)", "scalar(v_fma)", "copy", "copy4", "lib bilinear", "lib bf16x6 conv"};
constexpr long long NOUT = 2LL * 128 * 128 * 64;

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const double delay_us = argc > 2 ? atof(argv[2]) : 30.0;
    // the kernel beside the victims: wres (the bf16x6 weight-resident 3x3, both allocations), native (the fp32-MFMA
    // weight-resident 3x3: 184 VGPRs, a 144-VGPR hole), igemm (a dilation-2 3x3 on the bf16x6 implicit GEMM
    // conv_fwd_b6_kernel), ru (the AMP fused ResidualUnit ru_fused_f16_kernel: 232 VGPRs, a 48-VGPR hole)
    // (round 5) wg1x1 / wghalo: the bf16x6 weight gradients — wgrad1x1_bf6_kernel<2, 1, 2, 2> (256 threads, one block
    // per CU by LDS, 168 VGPRs: a 344-VGPR hole per SIMD) and wgrad_halo_bf6_kernel<1, 3, 1, 1> (2 blocks, 208 VGPRs:
    // 96) — both convert with v_cvt_pk_bf16_f32 and run bf16 MFMAs, as the two guarded kernels do
    const char* hogname = argc > 3 ? argv[3] : "wres";
    const bool ru = strcmp(hogname, "ru") == 0;
    const bool wg1 = strcmp(hogname, "wg1x1") == 0, wgh = strcmp(hogname, "wghalo") == 0, wg = wg1 || wgh;
    const bool b6v = strcmp(hogname, "native-b6v") == 0;
    const bool native = b6v || strcmp(hogname, "native") == 0;
    const int B = 2, H = 256, W = 256, C = 64;
    const long long nx = (long long)B * H * W * C;
    std::vector<float> hx(nx), hf(nx), hw(C * C * 9), hb(C);
    std::mt19937 rng(74);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& v : hx) v = u(rng);
    for (auto& v : hf) v = u(rng);
    for (auto& v : hw) v = u(rng) / 24.f;
    for (auto& v : hb) v = u(rng) * 0.1f;
    float *dx, *dfeat, *dw, *dw2, *db, *dy, *dslope, *dout, *dref;
    CK(hipMalloc(&dx, nx * 4));
    CK(hipMalloc(&dfeat, nx * 4));
    CK(hipMalloc(&dw, hw.size() * 4));
    CK(hipMalloc(&dw2, hw.size() * 4));
    CK(hipMalloc(&db, C * 4));
    CK(hipMalloc(&dy, nx * 4));
    CK(hipMalloc(&dslope, 4));
    const int NV = 3;  // victim launches per conv launch
    CK(hipMalloc(&dout, NOUT * 4 * 4 * NV));
    CK(hipMalloc(&dref, NOUT * 4 * 4));
    CK(hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dfeat, hf.data(), nx * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), C * 4, hipMemcpyHostToDevice));
    const float slope = 0.25f;
    CK(hipMemcpy(dslope, &slope, 4, hipMemcpyHostToDevice));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    const int dil = strcmp(hogname, "igemm") == 0 ? 2 : 1;
    hyres_conv_geom g;
    CH(hyres_geom_conv2d(&g, B, H, W, C, C, C, C, 3, 3, 1, dil, dil));
    CH(hyres_conv_weight_prep(&g, dw, dw2, HYRES_WPREP_CONV, C, C, 3, 3, dil, nullptr, sa));
    // ru: x / y fp16 [2][256][256][128], weights fp32 (w1 [64][128], w2 [64][64][3][3], w3 [128][64])
    void *rx = nullptr, *ry = nullptr;
    float *rw1 = nullptr, *rw3 = nullptr, *rb3 = nullptr;
    if (ru) {
        std::vector<_Float16> hr(nx * 2);
        for (auto& v : hr) v = (_Float16)u(rng);
        std::vector<float> h13(128 * 64);
        for (auto& v : h13) v = u(rng) / 11.f;
        CK(hipMalloc(&rx, nx * 4));
        CK(hipMalloc(&ry, nx * 4));
        CK(hipMalloc(&rw1, h13.size() * 4));
        CK(hipMalloc(&rw3, h13.size() * 4));
        CK(hipMalloc(&rb3, 128 * 4));
        CK(hipMemcpy(rb3, h13.data(), 128 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rx, hr.data(), nx * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rw1, h13.data(), h13.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rw3, h13.data(), h13.size() * 4, hipMemcpyHostToDevice));
        CH(hyres_ru_fused_f16_ok(B, H, W, 128) ? 0 : 1);
    }
    // weight-gradient hogs: P = dY [2*256*256][Co], Q = X [2*256*256][Ci]
    hyres_wgrad_desc wd;
    float *wp = nullptr, *wq = nullptr, *wdst = nullptr;
    void* wws = nullptr;
    long long wwsb = 0, wdn = 0;
    if (wg) {
        const int Ci = wg1 ? 128 : 64, Co = 64, K = wg1 ? 1 : 3;
        CH(hyres_wgrad_desc_conv2d(&wd, B, H, W, Ci, Ci, Co, Co, K, K, 1, K / 2, 1));
        wd.sm = Ci * K * K;
        wwsb = hyres_wgrad_workspace_bytes(&wd);
        wdn = (long long)Co * Ci * K * K;
        std::vector<float> hp((long long)B * H * W * Ci);
        for (auto& v : hp) v = u(rng);
        CK(hipMalloc(&wp, (long long)B * H * W * Co * 4));
        CK(hipMalloc(&wq, (long long)B * H * W * Ci * 4));
        CK(hipMalloc(&wdst, wdn * 4));
        CK(hipMalloc(&wws, wwsb + 256));
        CK(hipMemcpy(wp, hp.data(), (long long)B * H * W * Co * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(wq, hp.data(), (long long)B * H * W * Ci * 4, hipMemcpyHostToDevice));
    }
    hyres_epilogue e;
    memset(&e, 0, sizeof e);
    e.kind = HYRES_EPI_BIAS;
    e.act = HYRES_ACT_PRELU;
    e.bias = db;
    e.slope = dslope;
    CH(hyres_conv_tuning(HYRES_TUNE_F32_GEMM, native ? 0 : 1, nullptr));
    char kname[128];
    // the bf16x6 victim conv: x [2][256][256][64] -> [2][256][256][64] (4 * NOUT floats), its own weight layout
    float* dw2v = nullptr;
    if (b6v) {
        CK(hipMalloc(&dw2v, hw.size() * 4));
        CH(hyres_conv_weight_prep(&g, dw, dw2v, HYRES_WPREP_CONV, C, C, 3, 3, 1, nullptr, sa));
        CK(hipStreamSynchronize(sa));
    }
    auto conv = [&]() {
        if (b6v) {  // the hog: the native weight-resident kernel
            CH(hyres_conv_tuning(HYRES_TUNE_F32_GEMM, 0, nullptr));
            CH(hyres_conv_tuning(HYRES_TUNE_WRES32, 1, nullptr));
        }
        if (wg)
            CH(hyres_conv_wgrad(&wd, wp, wq, wdst, nullptr, wws, wwsb, sa));
        else if (ru)
            CH(hyres_ru_fused_f16(rx, ry, B, H, W, 128, rw1, db, dw, db, rw3, rb3, 1, nullptr, nullptr, sa));
        else
            CH(hyres_conv_forward(&g, dfeat, dw2, 9 * C, dy, &e, nullptr, 0, sa));
    };
    auto launch = [&](int kind, float* out, hipStream_t s) {
        const dim3 grid(8, 2 * 128);
        if (kind == 0) hipLaunchKernelGGL(victim<0>, grid, dim3(256), 0, s, dx, out);
        if (kind == 1) hipLaunchKernelGGL(victim<1>, grid, dim3(256), 0, s, dx, out);
        if (kind == 2) hipLaunchKernelGGL(victim<2>, grid, dim3(256), 0, s, dx, out);
        if (kind == 3) hipLaunchKernelGGL(victim<3>, grid, dim3(256), 0, s, dx, out);
        if (kind == 4) CH(hyres_bilinear_fwd(dx, 64, out, 64, 2, 256, 256, 128, 128, 64, 2.0f, 2.0f, 0, s));
        if (kind == 5) {  // bf16x6 implicit GEMM while the hog's keys are restored by the next conv()
            CH(hyres_conv_tuning(HYRES_TUNE_F32_GEMM, 1, nullptr));
            CH(hyres_conv_tuning(HYRES_TUNE_WRES32, 0, nullptr));
            CH(hyres_conv_forward(&g, dx, dw2v, 9 * C, out, &e, nullptr, 0, s));
        }
    };
    const long long vsz[6] = {NOUT, NOUT, NOUT, 4 * NOUT, NOUT, 4 * NOUT};
    std::vector<float> ref(4 * NOUT), got(4 * NOUT * NV), y0(nx), y1(nx);
    const bool wres = strcmp(hogname, "wres") == 0;
    for (int guard = wres ? 0 : 1; guard < 2; ++guard) {
        CH(hyres_conv_tuning(HYRES_TUNE_WRES_BF6_GUARD, guard, nullptr));
        conv();
        CK(hipStreamSynchronize(sa));
        if (wg) CK(hipMemcpy(y0.data(), wdst, wdn * 4, hipMemcpyDeviceToHost));
        else CK(hipMemcpy(y0.data(), ru ? ry : dy, nx * 4, hipMemcpyDeviceToHost));
        if (wres)
            printf("== conv 3x3 64->64 2x256x256 bf16x6 weight-resident, %s\n",
                   guard ? "guarded (256 VGPRs: no room beside it)" : "UNGUARDED (224 VGPRs: a 64-VGPR hole per SIMD)");
        else
            printf("== %s\n", wg1 ? "1x1 weight gradient 128->64 2x256x256 (wgrad1x1_bf6_kernel)"
                               : wgh ? "3x3 weight gradient 64->64 2x256x256 (wgrad_halo_bf6_kernel)"
                               : ru ? "fused ResidualUnit f16 (ru_fused_f16_kernel, 2x256x256x128)"
                                  : (dil == 2 ? "dilation-2 3x3 64->64 2x256x256 on the bf16x6 implicit GEMM"
                                              : b6v ? "3x3 64->64 2x256x256 fp32-MFMA weight-resident (native), bf16x6 conv victim"
                                              : "3x3 64->64 2x256x256 fp32-MFMA weight-resident (native)"));
        for (int kind = b6v ? 5 : 4; kind >= (b6v ? 4 : 0); --kind) {
            launch(kind, dref, sa);
            CK(hipStreamSynchronize(sa));
            CK(hipMemcpy(ref.data(), dref, vsz[kind] * 4, hipMemcpyDeviceToHost));
            size_t wrong = 0, events = 0, conv_bad = 0, hit = 0;
            size_t grp[4] = {0, 0, 0, 0}, comp[4] = {0, 0, 0, 0}, lost[4] = {0, 0, 0, 0}, other = 0, perev16 = 0;
            for (int rep = 0; rep < reps; ++rep) {
                CK(hipDeviceSynchronize());
                conv();
                // let the conv's blocks take the CUs first (as the library's branch streams do: the side stream's
                // kernels are enqueued tens of microseconds after the main stream's conv); the victims then run in
                // the holes its waves leave
                const double t0 = wall();
                while (wall() - t0 < delay_us * 1e-6) {
                }
                for (int v = 0; v < NV; ++v) launch(kind, dout + v * 4 * NOUT, sb);
                CK(hipDeviceSynchronize());
                if (wg) CK(hipMemcpy(y1.data(), wdst, wdn * 4, hipMemcpyDeviceToHost));
                else CK(hipMemcpy(y1.data(), ru ? ry : dy, nx * 4, hipMemcpyDeviceToHost));
                conv_bad += memcmp(y0.data(), y1.data(), nx * 4) != 0;
                for (int v = 0; v < NV; ++v)
                    CK(hipMemcpy(got.data() + v * 4 * NOUT, dout + v * 4 * NOUT, vsz[kind] * 4, hipMemcpyDeviceToHost));
                const size_t before = wrong;
                for (int v = 0; v < NV; ++v) {
                    long long last_ev = -1;
                    int evcount = 0;
                    for (long long k = 0; k < vsz[kind]; ++k) {
                        const float a = got[v * 4 * NOUT + k], r = ref[k];
                        if (memcmp(&a, &r, 4) == 0) continue;
                        ++wrong;
                        const long long kk = k % NOUT;              // element within one output plane
                        const long long thread = kk / 4;            // float4 index = thread of its row
                        const long long ev = (long long)v * 8 * NOUT + (k / NOUT) * NOUT + thread / 16;
                        if (ev != last_ev) {
                            if (evcount == 16) ++perev16;
                            ++events;
                            last_ev = ev;
                            evcount = 0;
                        }
                        ++evcount;
                        grp[(thread % 64) / 16]++;
                        comp[kk % 4]++;
                        if (kind < 2 || kind == 4) {
                            const int c = kk % 64, ow = (kk / 64) % 128, oh = (kk / 64 / 128) % 128,
                                      b = kk / 64 / 128 / 128;
                            bool m = false;
                            for (int t = 0; t < 4 && !m; ++t) {
                                const float tv = hx[((long long)(b * 256 + 2 * oh + (t >> 1)) * 256 + 2 * ow + (t & 1)) * 64 + c];
                                if (std::fabs((r - a) - 0.25f * tv) < 1e-6f) {
                                    lost[t]++;
                                    m = true;
                                }
                            }
                            other += !m;
                        }
                    }
                    if (evcount == 16) ++perev16;
                }
                hit += wrong > before;
            }
            printf("  %-14s reps hit %2zu/%d  wrong %7zu  in %5zu 16-lane groups (%zu with exactly 16)  lane group "
                   "0/1/2/3: %zu/%zu/%zu/%zu  component x/y/z/w: %zu/%zu/%zu/%zu",
                   KNAME[kind], hit, reps, wrong, events, perev16, grp[0], grp[1], grp[2], grp[3], comp[0], comp[1],
                   comp[2], comp[3]);
            if ((kind < 2 || kind == 4) && wrong)
                printf("  tap lost a/q/r/d: %zu/%zu/%zu/%zu other %zu", lost[0], lost[1], lost[2], lost[3], other);
            printf("  [conv output changed in %zu reps]\n", conv_bad);
            fflush(stdout);
        }
    }
    snprintf(kname, sizeof kname, "done");
    printf("%s\n", kname);
    return 0;
}
