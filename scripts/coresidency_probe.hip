// Co-residency probe (DESIGN §4 "Cross-kernel interference", VERDICT r4 "next" 1b). Standalone, not part of the library.
//
// Round 4 found that a side-stream bilinear resize computed wrong values (up to 0.25 off) while the library's
// conv3x3_wres_bf6_kernel ran beside it, and only when the conv's VGPR allocation (224 per wave, 2 waves per SIMD)
// left room for a bilinear wave on the same SIMD. This program isolates the ingredients:
//
//   hog<MODE, NREG>  one 512-thread block per CU (148.5 KB static LDS), 2 waves per SIMD, VGPR allocation forced to
//                    NREG per wave (an empty asm that clobbers v[NREG-1]; 0 = the compiler's own, ~64), running for a
//                    few ms a loop shaped like the conv's inner loop — per tap 6 ds_read_b128 then MODE's work:
//                      0 bf16x6: v_cvt_pk_bf16_f32 splits + 6 v_mfma_f32_32x32x16_bf16   (the conv's mix)
//                      1 bf16 MFMA only (no converts)
//                      2 f16 MFMA only (v_mfma_f32_32x32x16_f16, ru_fused_f16_kernel's instruction)
//                      3 fp32 MFMA only (v_mfma_f32_32x32x2f32, the native kernel's instruction)
//                      4 VALU only: the bf16 splits, no MFMA
//   victims          on a second stream while the hog runs, each against its own result computed alone:
//                      bilinear  the library's bilinear_fwd_kernel<4,false> body (x1/2, NHWC, float4): the compiler
//                                forms it with packed fp32 VALU (v_pk_mul_f32 / v_pk_fma_f32 with op_sel)
//                      scalar    the same arithmetic, every multiply / fma forced to the unpacked v_mul_f32 / v_fma_f32
//                      intmix    the same four loads combined with integer VALU only (xor / add / rotate)
//   controls         each victim alone at one wave per SIMD (150 KB dynamic LDS: one 256-thread block per CU), and
//                    hog then victim on ONE stream (no overlap).
//
// For every wrong bilinear output it also reports which of the four 0.25-weighted taps the error equals (a tap dropped
// or doubled = a load returned a wrong value / a register lost; anything else = arithmetic on a clobbered operand).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/coresidency_probe.hip -o scripts/coresidency_probe
//   scripts/coresidency_probe [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// ------------------------------------------------------------------------------------------------ victims
__device__ __forceinline__ void src_index(float scale, int o, int in, int& i0, int& i1, float& l0, float& l1) {
    float src = scale * ((float)o + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    i0 = (int)src;
    if (i0 > in - 1) i0 = in - 1;
    i1 = i0 + ((i0 < in - 1) ? 1 : 0);
    l1 = src - (float)i0;
    l0 = 1.0f - l1;
}

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

// KIND 0 bilinear (compiler's packed fp32), 1 scalar (unpacked asm), 2 intmix (integer only)
template <int KIND>
__global__ __launch_bounds__(256) void victim(const float* x, float* y, int Hi, int Wi, int Ho, int Wo, int C, float s) {
    extern __shared__ float dyn[];  // only to cap occupancy in the control runs
    if (threadIdx.x == 1023) dyn[0] = 0.f;
    const int CG = C / 4;
    const int row = blockIdx.y;
    const int b = row / Ho, oh = row - b * Ho;
    int h0, h1;
    float lh0, lh1;
    src_index(s, oh, Hi, h0, h1, lh0, lh1);
    const long long x0 = ((long long)b * Hi + h0) * Wi * C, x1 = ((long long)b * Hi + h1) * Wi * C;
    const long long yr = (long long)row * Wo * C;
    const int n = Wo * CG;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int ow = i / CG;
        const int c = (i - ow * CG) * 4;
        int w0, w1;
        float lw0, lw1;
        src_index(s, ow, Wi, w0, w1, lw0, lw1);
        const float4 a = *reinterpret_cast<const float4*>(x + x0 + w0 * C + c);
        const float4 q = *reinterpret_cast<const float4*>(x + x0 + w1 * C + c);
        const float4 r = *reinterpret_cast<const float4*>(x + x1 + w0 * C + c);
        const float4 d = *reinterpret_cast<const float4*>(x + x1 + w1 * C + c);
        float4 v;
        if constexpr (KIND == 0) {
            v.x = lh0 * (lw0 * a.x + lw1 * q.x) + lh1 * (lw0 * r.x + lw1 * d.x);
            v.y = lh0 * (lw0 * a.y + lw1 * q.y) + lh1 * (lw0 * r.y + lw1 * d.y);
            v.z = lh0 * (lw0 * a.z + lw1 * q.z) + lh1 * (lw0 * r.z + lw1 * d.z);
            v.w = lh0 * (lw0 * a.w + lw1 * q.w) + lh1 * (lw0 * r.w + lw1 * d.w);
        } else if constexpr (KIND == 1) {
            v.x = fma_s(lh1, fma_s(lw0, r.x, mul_s(lw1, d.x)), mul_s(lh0, fma_s(lw0, a.x, mul_s(lw1, q.x))));
            v.y = fma_s(lh1, fma_s(lw0, r.y, mul_s(lw1, d.y)), mul_s(lh0, fma_s(lw0, a.y, mul_s(lw1, q.y))));
            v.z = fma_s(lh1, fma_s(lw0, r.z, mul_s(lw1, d.z)), mul_s(lh0, fma_s(lw0, a.z, mul_s(lw1, q.z))));
            v.w = fma_s(lh1, fma_s(lw0, r.w, mul_s(lw1, d.w)), mul_s(lh0, fma_s(lw0, a.w, mul_s(lw1, q.w))));
        } else {
            auto mix = [](float p, float t, float u, float w) {
                unsigned h = __float_as_uint(p) ^ ((__float_as_uint(t) << 7) | (__float_as_uint(t) >> 25));
                h += __float_as_uint(u) ^ 0x9E3779B9u;
                h ^= (__float_as_uint(w) >> 3) + 0x7F4A7C15u;
                return __uint_as_float(h & 0x3FFFFFFFu);  // finite, exact bit pattern
            };
            v.x = mix(a.x, q.x, r.x, d.x);
            v.y = mix(a.y, q.y, r.y, d.y);
            v.z = mix(a.z, q.z, r.z, d.z);
            v.w = mix(a.w, q.w, r.w, d.w);
        }
        *reinterpret_cast<float4*>(y + yr + (long long)ow * C + c) = v;
    }
}

// ------------------------------------------------------------------------------------------------ hog
constexpr int HOG_LDS = 74240;  // bf16 elements = 148,480 B (the conv's 148.7 KB: one block per CU)
typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// MODE = 4 * CVT + MF.  CVT: 0 none, 1 v_cvt_pk_bf16_f32 splits, 2 v_cvt_pk_f16_f32 splits (ru_fused_f16_kernel's
// convert).  MF: 0 none, 1 v_mfma_f32_32x32x16_bf16, 2 v_mfma_f32_32x32x16_f16, 3 v_mfma_f32_32x32x2f32.
template <int CVT>
__device__ __forceinline__ float2v split2(float2v x) {  // x -> hi + mid + lo pieces; returns a dependent sum
    if constexpr (CVT == 1) {
        const bf16x2 h = __builtin_convertvector(x, bf16x2);
        const float2v r = x - __builtin_convertvector(h, float2v);
        const bf16x2 m = __builtin_convertvector(r, bf16x2);
        const bf16x2 l = __builtin_convertvector(r - __builtin_convertvector(m, float2v), bf16x2);
        return __builtin_convertvector(m, float2v) + __builtin_convertvector(l, float2v);
    } else if constexpr (CVT == 2) {
        const f16x2 h = __builtin_convertvector(x, f16x2);
        const float2v r = x - __builtin_convertvector(h, float2v);
        const f16x2 m = __builtin_convertvector(r, f16x2);
        const f16x2 l = __builtin_convertvector(r - __builtin_convertvector(m, float2v), f16x2);
        return __builtin_convertvector(m, float2v) + __builtin_convertvector(l, float2v);
    } else {
        return x * 0.5f + 0.25f;
    }
}

template <int MODE, int NREG>
__global__ __launch_bounds__(512, 1) void hog(const float* in, float* out, int iters) {
    constexpr int CVT = MODE >> 2, MF = MODE & 3;
    __shared__ __attribute__((aligned(16))) unsigned short lds[HOG_LDS];
    if constexpr (NREG == 216) asm volatile("" ::: "v215");
    if constexpr (NREG == 224) asm volatile("" ::: "v223");
    if constexpr (NREG == 232) asm volatile("" ::: "v231");
    if constexpr (NREG == 256) asm volatile("" ::: "v255");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    for (int i = tid; i < HOG_LDS / 2; i += 512) {  // operand images: bf16 / f16 bit patterns of small numbers
        const float v = in[(blockIdx.x * 997 + i) & 262143];
        const unsigned u = __float_as_uint(v * 0.125f);
        lds[2 * i] = (unsigned short)(u >> 16);
        lds[2 * i + 1] = (unsigned short)(0x3000 | (u & 0x03FF));
    }
    __syncthreads();
    floatx16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float2v hv = {in[(blockIdx.x * 512 + tid) & 262143], in[(blockIdx.x * 512 + tid + 7) & 262143]};
    float2v hw = hv * 0.5f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int base = (((it * 9 + t) * 67 + wave * 1031 + lr * 16) & 32767) * 2 + lh * 8;
            const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(&lds[base & ~7]);
            const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(&lds[(base + 16384) & ~7]);
            const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(&lds[(base + 32768) & ~7]);
            const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(&lds[(base + 40960) & ~7]);
            const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(&lds[(base + 49152) & ~7]);
            const bf16x8 x2 = *reinterpret_cast<const bf16x8*>(&lds[(base + 57344) & ~7]);
            if constexpr (MF == 1) {
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, x0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x2, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x0, acc, 0, 0, 0);
            } else if constexpr (MF == 2) {
                const f16x8 a0 = __builtin_bit_cast(f16x8, w0), a1 = __builtin_bit_cast(f16x8, w1);
                const f16x8 b0 = __builtin_bit_cast(f16x8, x0), b1 = __builtin_bit_cast(f16x8, x1);
                const f16x8 a2 = __builtin_bit_cast(f16x8, w2), b2 = __builtin_bit_cast(f16x8, x2);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b2, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
            } else if constexpr (MF == 3) {
                const floatx4v p = __builtin_bit_cast(floatx4v, w0), q = __builtin_bit_cast(floatx4v, x0);
                const floatx4v p1 = __builtin_bit_cast(floatx4v, w1), q1 = __builtin_bit_cast(floatx4v, x1);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(p[u], q[u], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(p1[u], q1[u], acc, 0, 0, 0);
                }
            } else {  // no MFMA: keep the LDS reads live
                const floatx4v p = __builtin_bit_cast(floatx4v, w0) + __builtin_bit_cast(floatx4v, x2);
                const floatx4v q = __builtin_bit_cast(floatx4v, x0) + __builtin_bit_cast(floatx4v, w2);
                acc[t] += p[0] * q[1] + __builtin_bit_cast(floatx4v, w1)[2] + __builtin_bit_cast(floatx4v, x1)[3];
            }
            // the conv's per-step split work, interleaved with the MFMAs (three pieces of two operands per tap)
            hv = split2<CVT>(hv + (float)t);
            hw = split2<CVT>(hw + hv);
            hv = split2<CVT>(hv - hw);
        }
        __syncthreads();
        if ((it & 1) == 0) {
            const int o = ((it * 131 + tid * 8) & (HOG_LDS / 2 - 1)) & ~7;
            for (int k = 0; k < 8; ++k) lds[HOG_LDS / 2 + o + k] = (unsigned short)(__float_as_uint(acc[k]) >> 20);
        }
        __syncthreads();
    }
    float keep = 0.f;
    for (int r = 0; r < 16; ++r) keep += acc[r];
    out[blockIdx.x * 512 + tid] = keep + hv[0] + hv[1] + hw[0] + hw[1];
}

// ------------------------------------------------------------------------------------------------ host
struct Geo {
    int B = 2, Hi = 256, Wi = 256, C = 64, Ho = 128, Wo = 128;
    size_t in_elems() const { return (size_t)B * Hi * Wi * C; }
    size_t out_elems() const { return (size_t)B * Ho * Wo * C; }
};

static void launch_victim(int kind, const float* x, float* y, const Geo& g, hipStream_t s, size_t dyn) {
    const int CG = g.C / 4;
    const dim3 grid((unsigned)((g.Wo * CG + 255) / 256), (unsigned)(g.B * g.Ho));
    if (kind == 0) hipLaunchKernelGGL(victim<0>, grid, dim3(256), dyn, s, x, y, g.Hi, g.Wi, g.Ho, g.Wo, g.C, 2.0f);
    if (kind == 1) hipLaunchKernelGGL(victim<1>, grid, dim3(256), dyn, s, x, y, g.Hi, g.Wi, g.Ho, g.Wo, g.C, 2.0f);
    if (kind == 2) hipLaunchKernelGGL(victim<2>, grid, dim3(256), dyn, s, x, y, g.Hi, g.Wi, g.Ho, g.Wo, g.C, 2.0f);
}

typedef void (*HogFn)(const float*, float*, int);
struct HogCfg {
    int mode, nreg;
    HogFn fn;
};
#define HOGS(M) {M, 216, hog<M, 216>}, {M, 224, hog<M, 224>}, {M, 232, hog<M, 232>}, {M, 256, hog<M, 256>}

static const char* CVT_NAME[] = {"no cvt", "cvt_pk_bf16", "cvt_pk_f16"};
static const char* MF_NAME[] = {"no mfma", "bf16 mfma", "f16 mfma", "fp32 mfma"};
static const char* KIND_NAME[] = {"bilinear(pk_f32)", "scalar(v_fma)", "intmix(int)"};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    Geo g;
    std::vector<float> hx(g.in_elems());
    std::mt19937 rng(74);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& v : hx) v = u(rng);
    float *dx, *dref[3], *dout, *hin, *hout;
    const int NV = 6;  // victim launches per hog launch
    CK(hipMalloc(&dx, hx.size() * 4));
    for (int k = 0; k < 3; ++k) CK(hipMalloc(&dref[k], g.out_elems() * 4));
    CK(hipMalloc(&dout, g.out_elems() * 4 * NV));
    CK(hipMalloc(&hin, 262144 * 4));
    CK(hipMalloc(&hout, 256 * 512 * 4));
    CK(hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(hin, hx.data(), 262144 * 4, hipMemcpyHostToDevice));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    std::vector<std::vector<float>> ref(3, std::vector<float>(g.out_elems()));
    for (int k = 0; k < 3; ++k) {
        launch_victim(k, dx, dref[k], g, sa, 0);
        CK(hipStreamSynchronize(sa));
        CK(hipMemcpy(ref[k].data(), dref[k], g.out_elems() * 4, hipMemcpyDeviceToHost));
    }
    {
        int bad = 0;
        for (size_t i = 0; i < g.out_elems(); i += 97) {
            const int c = i % g.C, ow = (i / g.C) % g.Wo, oh = (i / g.C / g.Wo) % g.Ho, b = i / g.C / g.Wo / g.Ho;
            double sm = 0;
            for (int dy = 0; dy < 2; ++dy)
                for (int dxx = 0; dxx < 2; ++dxx)
                    sm += 0.25 * hx[(((size_t)b * g.Hi + 2 * oh + dy) * g.Wi + 2 * ow + dxx) * g.C + c];
            bad += std::fabs(sm - ref[0][i]) > 1e-6;
        }
        printf("reference bilinear vs host formula: %d bad of %zu sampled\n", bad, g.out_elems() / 97);
    }
    std::vector<float> got(g.out_elems() * NV);
    auto taps = [&](size_t i, float t[4]) {
        const int c = i % g.C, ow = (i / g.C) % g.Wo, oh = (i / g.C / g.Wo) % g.Ho, b = i / g.C / g.Wo / g.Ho;
        for (int k = 0; k < 4; ++k) t[k] = hx[(((size_t)b * g.Hi + 2 * oh + (k >> 1)) * g.Wi + 2 * ow + (k & 1)) * g.C + c];
    };
    // Error statistics. A thread handles one output pixel's 4 channels (a float4): lane = i % 64 of the row's
    // 2048 threads, so a 16-lane group (one pass of the 16-wide SIMD over a wave64 instruction) = one pixel's 16
    // channel groups. An "event" = one (victim launch, row, wave, 16-lane group) with a wrong value.
    struct Stat {
        size_t wrong = 0, events = 0, full_groups = 0, reps_hit = 0;
        size_t comp[4] = {0, 0, 0, 0}, tap[6] = {0, 0, 0, 0, 0, 0};
        double worst = 0;
    };
    auto check = [&](int kind, Stat& st, bool show) {
        CK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
        const size_t before = st.wrong;
        std::vector<int> grp;  // wrong lanes per (launch, row, wave, group)
        long long cur = -1;
        int cnt = 0;
        auto flush = [&]() {
            if (cur >= 0) {
                st.events++;
                if (cnt == 16 * 4 || cnt >= 16) st.full_groups += cnt >= 16;
            }
        };
        int shown = 0;
        for (int v = 0; v < NV; ++v)
            for (size_t i = 0; i < g.out_elems(); ++i) {
                const float a = got[v * g.out_elems() + i], r = ref[kind][i];
                if (memcmp(&a, &r, 4) == 0) continue;
                ++st.wrong;
                st.worst = std::max(st.worst, std::fabs((double)a - r));
                const int c = i % g.C;
                const long long pix = (long long)(i / g.C);  // (b, oh, ow) flattened
                const long long key = (long long)v * (1LL << 40) + pix;  // one pixel = one 16-lane group
                if (key != cur) {
                    flush();
                    cur = key;
                    cnt = 0;
                }
                ++cnt;
                st.comp[c & 3]++;
                if (kind == 0) {
                    float t[4];
                    taps(i, t);
                    int m = 5;
                    for (int k = 0; k < 4; ++k)
                        if (std::fabs(std::fabs(a - r) - 0.25f * std::fabs(t[k])) < 1e-6f) m = k;
                    st.tap[m]++;
                    if (show && shown < 4) {
                        const int ow = (i / g.C) % g.Wo, oh = (i / g.C / g.Wo) % g.Ho;
                        printf("        launch %d oh %d ow %d (wave lane group %d) c %d: got %.6f want %.6f, err/0.25 = "
                               "%.4f, taps %.4f %.4f %.4f %.4f\n", v, oh, ow, ow & 3, c, a, r, (a - r) / 0.25f, t[0],
                               t[1], t[2], t[3]);
                        ++shown;
                    }
                }
            }
        flush();
        if (st.wrong > before) st.reps_hit++;
    };
    HogCfg cfgs[] = {HOGS(5), HOGS(1), HOGS(4), HOGS(10), HOGS(2), HOGS(8), HOGS(7), HOGS(6), HOGS(9), HOGS(0)};
    // size the hog to ~4 ms
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int iters = 400;
    {
        hipLaunchKernelGGL(cfgs[0].fn, dim3(256), dim3(512), 0, sa, hin, hout, iters);
        CK(hipEventRecord(e0, sa));
        hipLaunchKernelGGL(cfgs[0].fn, dim3(256), dim3(512), 0, sa, hin, hout, iters);
        CK(hipEventRecord(e1, sa));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        iters = std::max(50, (int)(iters * 4.0f / std::max(ms, 0.01f)));
        printf("hog mode 5 %d iters -> %.3f ms; using %d iters, %d reps x %d victim launches per config\n", 400, ms,
               iters, reps, NV);
    }
    for (const HogCfg& h : cfgs) {
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, (const void*)h.fn));
        printf("== hog %-12s + %-10s nreg %3d (numRegs %d)\n", CVT_NAME[h.mode >> 2], MF_NAME[h.mode & 3], h.nreg,
               fa.numRegs);
        for (int kind = 0; kind < 3; ++kind) {
            Stat st;
            for (int r = 0; r < reps; ++r) {
                CK(hipMemset(dout, 0, g.out_elems() * 4 * NV));
                CK(hipDeviceSynchronize());
                hipLaunchKernelGGL(h.fn, dim3(256), dim3(512), 0, sa, hin, hout, iters);
                for (int v = 0; v < NV; ++v) launch_victim(kind, dx, dout + v * g.out_elems(), g, sb, 0);
                CK(hipDeviceSynchronize());
                check(kind, st, st.wrong == 0);
            }
            printf("    %-18s reps hit %2zu/%d  wrong %7zu  events %4zu (full 16-lane %4zu)  comp x/y/z/w %zu/%zu/%zu/%zu", KIND_NAME[kind],
                   st.reps_hit, reps, st.wrong, st.events, st.full_groups, st.comp[0], st.comp[1], st.comp[2], st.comp[3]);
            if (kind == 0 && st.wrong)
                printf("  taps a/q/r/d %zu/%zu/%zu/%zu other %zu", st.tap[0], st.tap[1], st.tap[2], st.tap[3], st.tap[5]);
            printf("  max %.2e\n", st.worst);
        }
        fflush(stdout);
    }
    return 0;
}
