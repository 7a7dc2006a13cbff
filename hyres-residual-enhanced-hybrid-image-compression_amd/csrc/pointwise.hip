// Elementwise, reduction and optimiser kernels of the HyRES hot path (gfx950).
// All are HBM-bound streams: grid-stride loops, 256-thread blocks, float4 where the layout allows.
#include "common.h"

#include <mutex>

namespace hyres {

static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
int ok() { return HYRES_OK; }

static inline int grid_for(long long n, int per_thread = 1) {
    long long b = (n / per_thread + 255) / 256;
    if (b < 1) b = 1;
    if (b > 8192) b = 8192;
    return (int)b;
}

#define GRID_STRIDE(i, n) \
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

// ---------------------------------------------------------------- layout
__global__ void nchw_to_nhwc_kernel(const float* x, float* y, int B, int C, int H, int W, int ldy) {
    const long long n = (long long)B * H * W * C;
    GRID_STRIDE(i, n) {
        int c = (int)(i % C);
        long long p = i / C;  // (b,h,w)
        int hw = (int)(p % ((long long)H * W));
        int b = (int)(p / ((long long)H * W));
        y[p * ldy + c] = x[((long long)b * C + c) * H * W + hw];
    }
}
__global__ void nhwc_to_nchw_kernel(const float* x, int ldx, float* y, int B, int C, int H, int W) {
    const long long n = (long long)B * C * H * W;
    GRID_STRIDE(i, n) {
        int hw = (int)(i % ((long long)H * W));
        long long bc = i / ((long long)H * W);
        int c = (int)(bc % C);
        int b = (int)(bc / C);
        y[i] = x[((long long)b * H * W + hw) * ldx + c];
    }
}

// ---------------------------------------------------------------- elementwise
__global__ void axpby_kernel(const float* a, const float* b, float alpha, float* y, long long n) {
    GRID_STRIDE(i, n) y[i] = a[i] + alpha * b[i];
}
__global__ void add_clamp01_kernel(const float* x0, const float* r, float* y, long long n) {
    GRID_STRIDE(i, n) y[i] = fminf(fmaxf(x0[i] + r[i], 0.f), 1.f);
}
__global__ void add_clamp01_bwd_kernel(const float* pre, const float* g, float* gx, int acc, long long n) {
    // torch.clamp backward: gradient passes where min <= x <= max
    GRID_STRIDE(i, n) {
        float v = pre[i];
        float gv = (v >= 0.f && v <= 1.f) ? g[i] : 0.f;
        gx[i] = acc ? gx[i] + gv : gv;
    }
}
__global__ void relu_bwd_kernel(const float* y, const float* g, float* gx, long long n) {
    GRID_STRIDE(i, n) gx[i] = y[i] > 0.f ? g[i] : 0.f;
}
// H (here and below): the saved activation operand is fp16 in HBM (AMP training); G: the gradients (in and out)
// are fp16 too (AMP's fp16 activation gradients inside the f16_region), arithmetic fp32
template <bool H = false, bool G = false>
__global__ void relu_bwd_2d_kernel(const float* y, int ldy, const float* g, int ldg, float* gx, int ldgx,
                                   long long P, int C) {
    const long long n = P * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        stv<G>(gx, p * ldgx + c, ldv<H>(y, p * ldy + c) > 0.f ? ldv<G>(g, p * ldg + c) : 0.f);
    }
}
template <bool H = false, bool G = false>
__global__ void prelu_bwd_kernel(const float* x, int ldx, const float* g, int ldg, float* gx, int ldgx,
                                 long long P, int C, const float* slope, float* part) {
    const float a = slope[0];
    const long long n = P * C;
    float s = 0.f;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        float xv = ldv<H>(x, p * ldx + c);
        float gv = ldv<G>(g, p * ldg + c);
        stv<G>(gx, p * ldgx + c, xv > 0.f ? gv : a * gv);
        if (!(xv > 0.f)) s += xv * gv;
    }
    // block reduce
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void sum_partials_kernel(const float* part, int nb, float* out, int accumulate) {
    __shared__ float red[256];
    // 8 independent loads in flight per thread (a serial walk over nb/256 partials was latency-bound: ~19 us)
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int i = threadIdx.x;
    for (; i + 7 * 256 < nb; i += 8 * 256)
#pragma unroll
        for (int k = 0; k < 8; ++k) s8[k] += part[i + k * 256];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (i + k * 256 < nb) s8[k] += part[i + k * 256];
    const float s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = accumulate ? out[0] + red[0] : red[0];
}
__global__ void attn_gate_fwd_kernel(const float* a, const float* b, const float* x, float* out, long long n) {
    GRID_STRIDE(i, n) {
        float s = 1.0f / (1.0f + expf(-b[i]));
        out[i] = a[i] * s + x[i];
    }
}
// fp32, 4 elements per thread (round 6: the scalar kernels above ran the 32^2 AttentionBlock gates at ~0.9 TB/s); same
// arithmetic per element (bit-identical). MASK (backward): the gradient of a — the last ResidualUnit's ReLU output —
// with that ReLU's backward folded in, (a > 0) ? g * s : 0 (ops.attn_gate marks a's gradient masked)
__global__ __launch_bounds__(256) void attn_gate_fwd4_kernel(const float* a, const float* b, const float* x, float* out,
                                                             long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 av = ld4(a + 4 * i), bv = ld4(b + 4 * i), xv = ld4(x + 4 * i);
        const float s[4] = {1.0f / (1.0f + expf(-bv.x)), 1.0f / (1.0f + expf(-bv.y)), 1.0f / (1.0f + expf(-bv.z)),
                            1.0f / (1.0f + expf(-bv.w))};
        *reinterpret_cast<float4*>(out + 4 * i) =
            make_float4(av.x * s[0] + xv.x, av.y * s[1] + xv.y, av.z * s[2] + xv.z, av.w * s[3] + xv.w);
    }
}
// H: a, b fp16 (AMP's saved activations); G: g, ga, gb fp16 (AMP's fp16 gradients) — as attn_gate_bwd_kernel<H, G>
template <bool H, bool G, bool MASK>
__global__ __launch_bounds__(256) void attn_gate_bwd4_kernel(const float* a, const float* b, const float* g, float* ga,
                                                             float* gb, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 av4 = ldv4<H>(a, 4 * i), bv4 = ldv4<H>(b, 4 * i), gv4 = ldv4<G>(g, 4 * i);
        const float av[4] = {av4.x, av4.y, av4.z, av4.w}, bv[4] = {bv4.x, bv4.y, bv4.z, bv4.w};
        const float gv[4] = {gv4.x, gv4.y, gv4.z, gv4.w};
        float oa[4], ob[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float s = 1.0f / (1.0f + expf(-bv[c]));
            oa[c] = gv[c] * s;
            if constexpr (MASK) oa[c] = av[c] > 0.f ? oa[c] : 0.f;
            ob[c] = gv[c] * av[c] * s * (1.0f - s);
        }
        stv4<G>(ga, 4 * i, make_float4(oa[0], oa[1], oa[2], oa[3]));
        stv4<G>(gb, 4 * i, make_float4(ob[0], ob[1], ob[2], ob[3]));
    }
}
// fp16 activations (autocast inference): a, b, x, out fp16, 4 elements per thread, fp32 arithmetic
__global__ void attn_gate_fwd4h_kernel(const float* a, const float* b, const float* x, float* out, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 av = ldv4<true>(a, 4 * i), bv = ldv4<true>(b, 4 * i), xv = ldv4<true>(x, 4 * i);
        const float4 s = make_float4(1.0f / (1.0f + expf(-bv.x)), 1.0f / (1.0f + expf(-bv.y)),
                                     1.0f / (1.0f + expf(-bv.z)), 1.0f / (1.0f + expf(-bv.w)));
        stv4<true>(out, 4 * i, make_float4(av.x * s.x + xv.x, av.y * s.y + xv.y, av.z * s.z + xv.z, av.w * s.w + xv.w));
    }
}
template <bool H = false, bool G = false>
__global__ void attn_gate_bwd_kernel(const float* a, const float* b, const float* g, float* ga, float* gb,
                                     long long n) {
    GRID_STRIDE(i, n) {
        float s = 1.0f / (1.0f + expf(-ldv<H>(b, i)));
        float gv = ldv<G>(g, i);
        stv<G>(ga, i, gv * s);
        stv<G>(gb, i, gv * ldv<H>(a, i) * s * (1.0f - s));
    }
}
template <bool G = false>
__global__ void accumulate_kernel(const float* x, float* y, long long n) {
    GRID_STRIDE(i, n) stv<G>(y, i, ldv<G>(y, i) + ldv<G>(x, i));
}
// XH / YH: x / y stored fp16 (fp32 arithmetic)
template <bool XH = false, bool YH = false>
__global__ void add2d_kernel(const float* x, int ldx, float* y, int ldy, long long P, int C, int acc) {
    const long long n = P * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        float v = ldv<XH>(x, p * ldx + c);
        if (acc) v += ldv<YH>(y, p * ldy + c);
        stv<YH>(y, p * ldy + c, v);
    }
}
// float4 variants of the [P][C]-strided elementwise passes (C, every ld % 4 == 0, 16B-aligned, P*C < 2^31):
// 32-bit index math, 16 B per lane (8 B for fp16 operands)
template <bool XH = false, bool YH = false>
__global__ __launch_bounds__(256) void add2d4_kernel(const float* x, int ldx, float* y, int ldy, int P, int C4,
                                                     int acc) {
    const int n = P * C4;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int p = i / C4, c = 4 * (i - (i / C4) * C4);
        float4 v = ldv4<XH>(x, (long long)p * ldx + c);
        if (acc) {
            const float4 o = ldv4<YH>(y, (long long)p * ldy + c);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        stv4<YH>(y, (long long)p * ldy + c, v);
    }
}
template <bool H = false, bool G = false>
__global__ __launch_bounds__(256) void relu_bwd_2d4_kernel(const float* y, int ldy, const float* g, int ldg,
                                                           float* gx, int ldgx, int P, int C4) {
    const int n = P * C4;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int p = i / C4, c = 4 * (i - (i / C4) * C4);
        const float4 yv = ldv4<H>(y, (long long)p * ldy + c);
        const float4 gv = ldv4<G>(g, (long long)p * ldg + c);
        stv4<G>(gx, (long long)p * ldgx + c,
                make_float4(yv.x > 0.f ? gv.x : 0.f, yv.y > 0.f ? gv.y : 0.f, yv.z > 0.f ? gv.z : 0.f,
                            yv.w > 0.f ? gv.w : 0.f));
    }
}
template <bool H = false, bool G = false>
__global__ __launch_bounds__(256) void prelu_bwd4_kernel(const float* x, int ldx, const float* g, int ldg, float* gx,
                                                         int ldgx, int P, int C4, const float* slope, float* part) {
    const float a = slope[0];
    const int n = P * C4;
    float s = 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int p = i / C4, c = 4 * (i - (i / C4) * C4);
        const float4 xv = ldv4<H>(x, (long long)p * ldx + c);
        const float4 gv = ldv4<G>(g, (long long)p * ldg + c);
        stv4<G>(gx, (long long)p * ldgx + c,
                make_float4(xv.x > 0.f ? gv.x : a * gv.x, xv.y > 0.f ? gv.y : a * gv.y, xv.z > 0.f ? gv.z : a * gv.z,
                            xv.w > 0.f ? gv.w : a * gv.w));
        if (!(xv.x > 0.f)) s += xv.x * gv.x;
        if (!(xv.y > 0.f)) s += xv.y * gv.y;
        if (!(xv.z > 0.f)) s += xv.z * gv.z;
        if (!(xv.w > 0.f)) s += xv.w * gv.w;
    }
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

static inline bool vec4_2d(long long P, int C, const void* a, int lda, const void* b, int ldb, const void* c, int ldc) {
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
    return C % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && al(a) && al(b) && al(c) &&
           P * (long long)C < (1LL << 31);
}

__global__ void mul_kernel(const float* a, const float* b, float* y, long long n) {
    GRID_STRIDE(i, n) y[i] = a[i] * b[i];
}

// ---------------------------------------------------------------- GDN pieces
constexpr float kPedestal = 1.4551915228366852e-11f;  // 2^-36
__device__ __forceinline__ float beta_bound() { return 0.0010000000000072760f; }  // sqrt(1e-6 + 2^-36) as fp32
__device__ __forceinline__ float gamma_bound() { return 3.814697265625e-06f; }     // 2^-18

__global__ void gdn_reparam_fwd_kernel(const float* beta, const float* gamma, float* bp, float* gp, int C) {
    const long long n = (long long)C * C;
    GRID_STRIDE(i, n) {
        float v = fmaxf(gamma[i], gamma_bound());
        gp[i] = v * v - kPedestal;
        if (i < C) {
            float u = fmaxf(beta[i], beta_bound());
            bp[i] = u * u - kPedestal;
        }
    }
}
__device__ __forceinline__ float lb_sq_bwd(float x, float bound, float g) {
    // out = max(x, b)^2 - ped ; LowerBound passes where x >= b or grad < 0
    float lb = fmaxf(x, bound);
    float gl = g * 2.0f * lb;
    return (x >= bound || gl < 0.f) ? gl : 0.f;
}
__global__ void gdn_reparam_bwd_kernel(const float* beta, const float* gamma, const float* dbp, const float* dgp,
                                       float* db, float* dg, int C, int acc) {
    const long long n = (long long)C * C;
    GRID_STRIDE(i, n) {
        float v = lb_sq_bwd(gamma[i], gamma_bound(), dgp[i]);
        dg[i] = acc ? dg[i] + v : v;
        if (i < C) {
            float u = lb_sq_bwd(beta[i], beta_bound(), dbp[i]);
            db[i] = acc ? db[i] + u : u;
        }
    }
}
template <bool H = false, bool G = false>
__global__ void gdn_dnorm_kernel(const float* g, const float* y, const float* nrm, float* dn, long long n,
                                 float coef) {
    GRID_STRIDE(i, n) stv<G>(dn, i, coef * ldv<G>(g, i) * ldv<H>(y, i) / ldv<H>(nrm, i));
}

// ---------------------------------------------------------------- RNG
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void uniform_noise_kernel(float* out, long long n, unsigned long long seed, unsigned long long off) {
    GRID_STRIDE(i, n) {
        unsigned long long h = splitmix64(seed ^ splitmix64(off + (unsigned long long)i));
        float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
        out[i] = u - 0.5f;
    }
}

// Graph-replayable draw: the seed lives in device memory and is advanced after the draw by
// seed_advance_kernel (stream-ordered), so every replay of a captured HIP graph draws fresh noise.
__global__ void uniform_noise_dev_kernel(float* out, long long n, const unsigned long long* seed_dev,
                                         unsigned long long salt) {
    const unsigned long long seed = splitmix64(*seed_dev ^ salt);
    GRID_STRIDE(i, n) {
        unsigned long long h = splitmix64(seed ^ splitmix64((unsigned long long)i));
        float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
        out[i] = u - 0.5f;
    }
}
__global__ void seed_advance_kernel(unsigned long long* seed_dev) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *seed_dev = splitmix64(*seed_dev + 0x9E3779B97F4A7C15ull);
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float block_sum(float v, float* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int k = blockDim.x / 2; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    float r = red[0];
    __syncthreads();
    return r;
}
__global__ void sum_log_kernel(const float* x, long long n, float* part) {
    __shared__ float red[256];
    float s = 0.f;
    GRID_STRIDE(i, n) s += logf(x[i]);
    float r = block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}
__global__ void sum_sqdiff_kernel(const float* a, const float* b, long long n, float* part) {
    __shared__ float red[256];
    float s = 0.f;
    GRID_STRIDE(i, n) {
        float d = a[i] - b[i];
        s += d * d;
    }
    float r = block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}
// Sum of squares for clip_grad_norm_ and GradScaler's found_inf, accumulated AND returned in fp64: a large
// but finite gradient never overflows the sum (torch's found_inf is an element-wise !isfinite test, and its
// clip norm is taken on the unscaled gradient), so the result is +inf only when an element is +-inf and NaN
// only when an element is NaN.
__global__ void sumsq_kernel(const float* x, long long n, double* part) {
    __shared__ double red[256];
    double s = 0.0;
    GRID_STRIDE(i, n) {
        const double v = (double)x[i];
        s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void sumsq_final_kernel(const double* part, int nb, double* out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0];
}
__global__ void scale_recip_kernel(const float* x, const float* coef, float scale, float* g, long long n) {
    const float c = coef[0] * scale;
    GRID_STRIDE(i, n) g[i] = c / x[i];
}
__global__ void scale_diff_kernel(const float* a, const float* b, const float* coef, float scale, float* g,
                                  long long n) {
    const float c = coef[0] * scale;
    GRID_STRIDE(i, n) g[i] = c * (a[i] - b[i]);
}
__global__ void scale_kernel(const float* x, const float* coef, float scale, float* y, long long n, int acc) {
    const float c = coef ? coef[0] * scale : scale;
    GRID_STRIDE(i, n) {
        float v = c * x[i];
        y[i] = acc ? y[i] + v : v;
    }
}

// ---------------------------------------------------------------- RateDistortionLoss scalars
// sums = [sum log lik_y, sum log lik_z, sum (x_hat - x)^2]; out = [loss, bpp, residual_bpp, y_bpp, z_bpp, mse]
struct RdOut {
    float* o[6];
};
__global__ void rd_finalize_kernel(const float* sums, const float* jpeg_bpp, float lmbda, float npx, float nel,
                                   RdOut out) {
    if (threadIdx.x != 0) return;
    const float den = -0.69314718055994531f * npx;  // -ln2 * num_pixels
    const float yb = sums[0] / den, zb = sums[1] / den;
    const float res = yb + zb;
    const float bpp = res + (jpeg_bpp ? jpeg_bpp[0] : 0.f);
    const float mse = sums[2] / nel * 65025.0f;
    out.o[0][0] = lmbda * mse + bpp;
    out.o[1][0] = bpp;
    out.o[2][0] = res;
    out.o[3][0] = yb;
    out.o[4][0] = zb;
    out.o[5][0] = mse;
}
// coef = [c_y, c_z, c_mse] with d/dlik_y = c_y / lik_y, d/dlik_z = c_z / lik_z, d/dx_hat = c_mse*(x_hat - x)
__global__ void rd_bwd_coef_kernel(const float* g0, const float* g1, const float* g2, const float* g3,
                                   const float* g4, const float* g5, float lmbda, float npx, float nel, float* coef) {
    if (threadIdx.x != 0) return;
    const float den = -0.69314718055994531f * npx;
    const float gl = g0[0], gb = g1[0], gr = g2[0], gy = g3[0], gz = g4[0], gm = g5[0];
    const float common = gl + gb + gr;
    coef[0] = (common + gy) / den;
    coef[1] = (common + gz) / den;
    coef[2] = (lmbda * gl + gm) * 65025.0f * 2.0f / nel;
}

// ---------------------------------------------------------------- Adam (torch.optim.Adam, foreach math)
// torch computes 1-beta, the bias corrections, step_size and sqrt(bc2) in Python double precision and
// hands them to the fp32 foreach kernels as scalars; the same is done here per thread (the step count
// lives on the device so that a skipped step — GradScaler found_inf — needs no host round trip).
struct AdamHyper {
    double lr, beta1, beta2, eps, max_norm;
    float omb1, omb2, epsf;  // (float)(1 - beta) computed in double, (float)eps
};

// skip: 0 never; 1 when sumsq is not finite (GradScaler found_inf); 2 when sumsq is NaN
__device__ __forceinline__ bool adam_skip(const double* sumsq, int skip) {
    if (!skip || !sumsq) return false;
    const double v = sumsq[0];
    return skip == 1 ? !isfinite(v) : isnan(v);
}

__global__ void adam_kernel(float* p, const float* g, float* m, float* v, long long n, AdamHyper h,
                            const float* step_dev, const double* sumsq, const float* gscale, int skip) {
    if (adam_skip(sumsq, skip)) return;
    const double t = (double)step_dev[0] + 1.0;
    const double bc1 = 1.0 - pow(h.beta1, t);
    const double bc2 = 1.0 - pow(h.beta2, t);
    const float step_size = (float)(h.lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float gs = gscale ? gscale[0] : 1.0f;  // GradScaler unscale_: grad * inv_scale
    float clip = 1.0f;
    if (sumsq && h.max_norm > 0.0) {
        // clip_grad_norm_ on the unscaled gradient: total = ||g * gs|| = sqrt(sumsq) * gs
        const float total = (float)(sqrt(sumsq[0]) * (double)gs);
        const float coef = (float)h.max_norm / (total + 1e-6f);
        clip = fminf(coef, 1.0f);
    }
    GRID_STRIDE(i, n) {
        float gv = g[i];
        if (gscale) gv = gv * gs;
        gv = gv * clip;
        float mv = m[i];
        mv = mv + h.omb1 * (gv - mv);                             // exp_avg.lerp_(grad, 1-beta1)
        const float vv = v[i] * (float)h.beta2 + h.omb2 * (gv * gv);  // mul_(beta2).addcmul_(g, g, 1-beta2)
        m[i] = mv;
        v[i] = vv;
        const float denom = sqrtf(vv) / bc2_sqrt + h.epsf;
        p[i] = p[i] - step_size * (mv / denom);
    }
}

__global__ void adam_finish_kernel(float* step_dev, const double* sumsq, int skip) {
    if (threadIdx.x == 0 && !adam_skip(sumsq, skip)) step_dev[0] = step_dev[0] + 1.0f;
}

// torch.amp.GradScaler.update (aten _amp_update_scale_): found_inf = !isfinite(sumsq of the scaled grads), which
// is exactly "some element is inf/NaN" because hyres_sumsq accumulates in fp64 (no overflow of finite sums)
__global__ void grad_scaler_update_kernel(const double* sumsq, float* scale, float* inv_scale, int* tracker,
                                          float growth, float backoff, int interval) {
    if (threadIdx.x != 0) return;
    const bool found_inf = !isfinite(sumsq[0]);
    float s = scale[0];
    if (found_inf) {
        s = s * backoff;
        tracker[0] = 0;
    } else {
        const int succ = tracker[0] + 1;
        if (succ == interval) {
            const float ns = s * growth;
            if (isfinite(ns)) s = ns;
            tracker[0] = 0;
        } else {
            tracker[0] = succ;
        }
    }
    scale[0] = s;
    inv_scale[0] = (float)(1.0 / (double)s);  // scale.double().reciprocal().float()
}

}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_version(void) { return 10000; }
const char* hyres_last_error_string(void) { return g_err.c_str(); }

int hyres_nchw_to_nhwc(const float* x, float* y, int B, int C, int H, int W, int ldy, hyres_stream_t s) {
    HY_REQUIRE(x && y && ldy >= C, HYRES_E_ARG, "nchw_to_nhwc: bad args");
    long long n = (long long)B * C * H * W;
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x, y, B, C, H, W, ldy);
    return HY_LAUNCH_CHECK("nchw_to_nhwc");
}
int hyres_nhwc_to_nchw(const float* x, int ldx, float* y, int B, int C, int H, int W, hyres_stream_t s) {
    HY_REQUIRE(x && y && ldx >= C, HYRES_E_ARG, "nhwc_to_nchw: bad args");
    long long n = (long long)B * C * H * W;
    hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x, ldx, y, B, C, H, W);
    return HY_LAUNCH_CHECK("nhwc_to_nchw");
}
int hyres_axpby(const float* a, const float* b, float alpha, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(a && b && y, HYRES_E_ARG, "axpby: NULL");
    hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), a, b, alpha, y, n);
    return HY_LAUNCH_CHECK("axpby");
}
int hyres_add_clamp01(const float* x0, const float* r, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(x0 && r && y, HYRES_E_ARG, "add_clamp01: NULL");
    hipLaunchKernelGGL(add_clamp01_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x0, r, y, n);
    return HY_LAUNCH_CHECK("add_clamp01");
}
int hyres_add_clamp01_bwd(const float* pre, const float* g, float* gx, int accumulate, long long n,
                          hyres_stream_t s) {
    HY_REQUIRE(pre && g && gx, HYRES_E_ARG, "add_clamp01_bwd: NULL");
    hipLaunchKernelGGL(add_clamp01_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), pre, g, gx,
                       accumulate, n);
    return HY_LAUNCH_CHECK("add_clamp01_bwd");
}
int hyres_relu_bwd(const float* y, const float* g, float* gx, long long n, hyres_stream_t s) {
    HY_REQUIRE(y && g && gx, HYRES_E_ARG, "relu_bwd: NULL");
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), y, g, gx, n);
    return HY_LAUNCH_CHECK("relu_bwd");
}
extern "C++" {
template <bool H, bool G>
static int relu_bwd_2d_impl(const float* y, int ldy, const float* g, int ldg, float* gx, int ldgx, long long P, int C,
                            hyres_stream_t s) {
    HY_REQUIRE(y && g && gx, HYRES_E_ARG, "relu_bwd_2d: NULL");
    if (vec4_2d(P, C, y, ldy, g, ldg, gx, ldgx)) {
        hipLaunchKernelGGL((relu_bwd_2d4_kernel<H, G>), dim3(grid_for(P * C / 4)), dim3(256), 0, as_stream(s), y, ldy,
                           g, ldg, gx, ldgx, (int)P, C / 4);
        return HY_LAUNCH_CHECK("relu_bwd_2d4");
    }
    hipLaunchKernelGGL((relu_bwd_2d_kernel<H, G>), dim3(grid_for(P * C)), dim3(256), 0, as_stream(s), y, ldy, g, ldg,
                       gx, ldgx, P, C);
    return HY_LAUNCH_CHECK("relu_bwd_2d");
}
}  // extern "C++"
int hyres_relu_bwd_2d(const float* y, int ldy, const float* g, int ldg, float* gx, int ldgx, long long P, int C,
                      hyres_stream_t s) {
    return relu_bwd_2d_impl<false, false>(y, ldy, g, ldg, gx, ldgx, P, C, s);
}
int hyres_relu_bwd_2d_f16(const void* y, int ldy, const void* g, int ldg, void* gx, int ldgx, long long P, int C,
                          int g16, hyres_stream_t s) {
    if (g16) return relu_bwd_2d_impl<true, true>((const float*)y, ldy, (const float*)g, ldg, (float*)gx, ldgx, P, C, s);
    return relu_bwd_2d_impl<true, false>((const float*)y, ldy, (const float*)g, ldg, (float*)gx, ldgx, P, C, s);
}
long long hyres_reduce_workspace_bytes(long long n) { return (long long)grid_for(n, 4) * 8 + 256; }  // fp64 partials

extern "C++" {
template <bool H, bool G>
static int prelu_bwd_impl(const float* x, int ldx, const float* g, int ldg, float* gx, int ldgx, long long P, int C,
                          const float* slope, float* dslope, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && g && gx && slope && dslope, HYRES_E_ARG, "prelu_bwd: NULL");
    int nb = grid_for(P * C, 4);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * 4, HYRES_E_WORKSPACE, "prelu_bwd: workspace");
    if (vec4_2d(P, C, x, ldx, g, ldg, gx, ldgx))
        hipLaunchKernelGGL((prelu_bwd4_kernel<H, G>), dim3(nb), dim3(256), 0, as_stream(s), x, ldx, g, ldg, gx, ldgx,
                           (int)P, C / 4, slope, (float*)ws);
    else
        hipLaunchKernelGGL((prelu_bwd_kernel<H, G>), dim3(nb), dim3(256), 0, as_stream(s), x, ldx, g, ldg, gx, ldgx, P,
                           C, slope, (float*)ws);
    int rc = HY_LAUNCH_CHECK("prelu_bwd");
    if (rc) return rc;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, as_stream(s), (const float*)ws, nb, dslope, 1);
    return HY_LAUNCH_CHECK("prelu_bwd_final");
}
}  // extern "C++"
int hyres_prelu_bwd(const float* x, int ldx, const float* g, int ldg, float* gx, int ldgx, long long P, int C,
                    const float* slope, float* dslope, void* ws, long long ws_bytes, hyres_stream_t s) {
    return prelu_bwd_impl<false, false>(x, ldx, g, ldg, gx, ldgx, P, C, slope, dslope, ws, ws_bytes, s);
}
int hyres_prelu_bwd_f16(const void* x, int ldx, const void* g, int ldg, void* gx, int ldgx, long long P, int C,
                        const float* slope, float* dslope, void* ws, long long ws_bytes, int g16, hyres_stream_t s) {
    if (g16)
        return prelu_bwd_impl<true, true>((const float*)x, ldx, (const float*)g, ldg, (float*)gx, ldgx, P, C, slope,
                                          dslope, ws, ws_bytes, s);
    return prelu_bwd_impl<true, false>((const float*)x, ldx, (const float*)g, ldg, (float*)gx, ldgx, P, C, slope, dslope,
                                       ws, ws_bytes, s);
}
static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
int hyres_attn_gate_fwd(const float* a, const float* b, const float* x, float* out, long long n, hyres_stream_t s) {
    HY_REQUIRE(a && b && x && out, HYRES_E_ARG, "attn_gate_fwd: NULL");
    if (n % 4 == 0 && al16(a) && al16(b) && al16(x) && al16(out)) {
        hipLaunchKernelGGL(attn_gate_fwd4_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(s), a, b, x, out, n / 4);
        return HY_LAUNCH_CHECK("attn_gate_fwd4");
    }
    hipLaunchKernelGGL(attn_gate_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), a, b, x, out, n);
    return HY_LAUNCH_CHECK("attn_gate_fwd");
}
int hyres_attn_gate_fwd_f16(const void* a, const void* b, const void* x, void* out, long long n, hyres_stream_t s) {
    HY_REQUIRE(a && b && x && out && n % 4 == 0, HYRES_E_ARG, "attn_gate_fwd_f16: NULL or n %% 4 != 0");
    hipLaunchKernelGGL(attn_gate_fwd4h_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(s), (const float*)a,
                       (const float*)b, (const float*)x, (float*)out, n / 4);
    return HY_LAUNCH_CHECK("attn_gate_fwd_f16");
}
int hyres_attn_gate_bwd_relu(const float* a, const float* b, const float* g, float* ga, float* gb, long long n,
                             hyres_stream_t s) {
    HY_REQUIRE(a && b && g && ga && gb && n % 4 == 0 && al16(a) && al16(b) && al16(g) && al16(ga) && al16(gb), HYRES_E_ARG,
               "attn_gate_bwd_relu: NULL, n %% 4 != 0 or an operand not 16B-aligned");
    hipLaunchKernelGGL((attn_gate_bwd4_kernel<false, false, true>), dim3(grid_for(n / 4)), dim3(256), 0, as_stream(s), a,
                       b, g, ga, gb, n / 4);
    return HY_LAUNCH_CHECK("attn_gate_bwd4");
}
int hyres_attn_gate_bwd(const float* a, const float* b, const float* g, float* ga, float* gb, long long n,
                        hyres_stream_t s) {
    HY_REQUIRE(a && b && g && ga && gb, HYRES_E_ARG, "attn_gate_bwd: NULL");
    if (n % 4 == 0 && al16(a) && al16(b) && al16(g) && al16(ga) && al16(gb)) {
        hipLaunchKernelGGL((attn_gate_bwd4_kernel<false, false, false>), dim3(grid_for(n / 4)), dim3(256), 0, as_stream(s),
                           a, b, g, ga, gb, n / 4);
        return HY_LAUNCH_CHECK("attn_gate_bwd4");
    }
    hipLaunchKernelGGL((attn_gate_bwd_kernel<false, false>), dim3(grid_for(n)), dim3(256), 0, as_stream(s), a, b, g,
                       ga, gb, n);
    return HY_LAUNCH_CHECK("attn_gate_bwd");
}
static bool al8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }
// the vector path of the fp16-activation gate backward: n % 4 == 0, fp16 operands 8B-aligned, fp32 ones 16B-aligned
static bool gate_f16_vec(const void* a, const void* b, const void* g, const void* ga, const void* gb, long long n,
                         int g16) {
    auto gal = [&](const void* p) { return g16 ? al8(p) : al16(p); };
    return n % 4 == 0 && al8(a) && al8(b) && gal(g) && gal(ga) && gal(gb);
}
extern "C++" {
template <bool MASK>
static void launch_gate_bwd4h(const void* a, const void* b, const void* g, void* ga, void* gb, long long n, int g16,
                              hipStream_t st) {
    if (g16)
        hipLaunchKernelGGL((attn_gate_bwd4_kernel<true, true, MASK>), dim3(grid_for(n / 4)), dim3(256), 0, st,
                           (const float*)a, (const float*)b, (const float*)g, (float*)ga, (float*)gb, n / 4);
    else
        hipLaunchKernelGGL((attn_gate_bwd4_kernel<true, false, MASK>), dim3(grid_for(n / 4)), dim3(256), 0, st,
                           (const float*)a, (const float*)b, (const float*)g, (float*)ga, (float*)gb, n / 4);
}
}  // extern "C++"
int hyres_attn_gate_bwd_relu_f16(const void* a, const void* b, const void* g, void* ga, void* gb, long long n, int g16,
                                 hyres_stream_t s) {
    HY_REQUIRE(a && b && g && ga && gb && gate_f16_vec(a, b, g, ga, gb, n, g16), HYRES_E_ARG,
               "attn_gate_bwd_relu_f16: NULL, n %% 4 != 0 or a misaligned operand");
    launch_gate_bwd4h<true>(a, b, g, ga, gb, n, g16, as_stream(s));
    return HY_LAUNCH_CHECK("attn_gate_bwd4h");
}
int hyres_attn_gate_bwd_f16(const void* a, const void* b, const void* g, void* ga, void* gb, long long n, int g16,
                            hyres_stream_t s) {
    HY_REQUIRE(a && b && g && ga && gb, HYRES_E_ARG, "attn_gate_bwd_f16: NULL");
    if (gate_f16_vec(a, b, g, ga, gb, n, g16)) {
        launch_gate_bwd4h<false>(a, b, g, ga, gb, n, g16, as_stream(s));
        return HY_LAUNCH_CHECK("attn_gate_bwd4h");
    }
    if (g16)
        hipLaunchKernelGGL((attn_gate_bwd_kernel<true, true>), dim3(grid_for(n)), dim3(256), 0, as_stream(s),
                           (const float*)a, (const float*)b, (const float*)g, (float*)ga, (float*)gb, n);
    else
        hipLaunchKernelGGL((attn_gate_bwd_kernel<true, false>), dim3(grid_for(n)), dim3(256), 0, as_stream(s),
                           (const float*)a, (const float*)b, (const float*)g, (float*)ga, (float*)gb, n);
    return HY_LAUNCH_CHECK("attn_gate_bwd_f16");
}
int hyres_accumulate(const float* x, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(x && y, HYRES_E_ARG, "accumulate: NULL");
    hipLaunchKernelGGL(accumulate_kernel<false>, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x, y, n);
    return HY_LAUNCH_CHECK("accumulate");
}
int hyres_accumulate_f16(const void* x, void* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(x && y, HYRES_E_ARG, "accumulate_f16: NULL");
    hipLaunchKernelGGL(accumulate_kernel<true>, dim3(grid_for(n)), dim3(256), 0, as_stream(s), (const float*)x,
                       (float*)y, n);
    return HY_LAUNCH_CHECK("accumulate_f16");
}
extern "C++" {
template <bool XH, bool YH>
static int add2d_impl(const float* x, int ldx, float* y, int ldy, long long P, int C, int accumulate, hyres_stream_t s) {
    if (vec4_2d(P, C, x, ldx, y, ldy, y, ldy)) {
        hipLaunchKernelGGL((add2d4_kernel<XH, YH>), dim3(grid_for(P * C / 4)), dim3(256), 0, as_stream(s), x, ldx, y,
                           ldy, (int)P, C / 4, accumulate);
        return HY_LAUNCH_CHECK("add2d4");
    }
    hipLaunchKernelGGL((add2d_kernel<XH, YH>), dim3(grid_for(P * C)), dim3(256), 0, as_stream(s), x, ldx, y, ldy, P, C,
                       accumulate);
    return HY_LAUNCH_CHECK("add2d");
}
}  // extern "C++"
int hyres_add2d(const float* x, int ldx, float* y, int ldy, long long P, int C, int accumulate,
                hyres_stream_t s) {
    HY_REQUIRE(x && y, HYRES_E_ARG, "add2d: NULL");
    return add2d_impl<false, false>(x, ldx, y, ldy, P, C, accumulate, s);
}
int hyres_add2d_f16(const void* x, int ldx, void* y, int ldy, long long P, int C, int accumulate, int io,
                    hyres_stream_t s) {
    HY_REQUIRE(x && y && io >= 0 && io <= 3, HYRES_E_ARG, "add2d_f16: NULL or io %d", io);
    const float* xf = (const float*)x;
    float* yf = (float*)y;
    switch (io) {
        case 1: return add2d_impl<true, false>(xf, ldx, yf, ldy, P, C, accumulate, s);
        case 2: return add2d_impl<false, true>(xf, ldx, yf, ldy, P, C, accumulate, s);
        case 3: return add2d_impl<true, true>(xf, ldx, yf, ldy, P, C, accumulate, s);
        default: return add2d_impl<false, false>(xf, ldx, yf, ldy, P, C, accumulate, s);
    }
}
int hyres_mul(const float* a, const float* b, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(a && b && y, HYRES_E_ARG, "mul: NULL");
    hipLaunchKernelGGL(mul_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), a, b, y, n);
    return HY_LAUNCH_CHECK("mul");
}
int hyres_zero(void* p, long long bytes, hyres_stream_t s) {
    HY_REQUIRE(p || bytes == 0, HYRES_E_ARG, "zero: NULL");
    hipError_t e = hipMemsetAsync(p, 0, (size_t)bytes, as_stream(s));
    if (e != hipSuccess) return set_error((int)e, "zero: %s", hipGetErrorString(e));
    return ok();
}
int hyres_gdn_reparam_fwd(const float* beta, const float* gamma, float* bp, float* gp, int C, hyres_stream_t s) {
    HY_REQUIRE(beta && gamma && bp && gp, HYRES_E_ARG, "gdn_reparam_fwd: NULL");
    hipLaunchKernelGGL(gdn_reparam_fwd_kernel, dim3(grid_for((long long)C * C)), dim3(256), 0, as_stream(s), beta,
                       gamma, bp, gp, C);
    return HY_LAUNCH_CHECK("gdn_reparam_fwd");
}
int hyres_gdn_reparam_bwd(const float* beta, const float* gamma, const float* dbp, const float* dgp, float* db,
                          float* dg, int C, int accumulate, hyres_stream_t s) {
    HY_REQUIRE(beta && gamma && dbp && dgp && db && dg, HYRES_E_ARG, "gdn_reparam_bwd: NULL");
    hipLaunchKernelGGL(gdn_reparam_bwd_kernel, dim3(grid_for((long long)C * C)), dim3(256), 0, as_stream(s), beta,
                       gamma, dbp, dgp, db, dg, C, accumulate);
    return HY_LAUNCH_CHECK("gdn_reparam_bwd");
}
int hyres_gdn_dnorm(const float* g, const float* y, const float* n, float* dn, long long P, int C, int inverse,
                    hyres_stream_t s) {
    HY_REQUIRE(g && y && n && dn, HYRES_E_ARG, "gdn_dnorm: NULL");
    long long cnt = P * C;
    hipLaunchKernelGGL((gdn_dnorm_kernel<false, false>), dim3(grid_for(cnt)), dim3(256), 0, as_stream(s), g, y, n, dn,
                       cnt, inverse ? 0.5f : -0.5f);
    return HY_LAUNCH_CHECK("gdn_dnorm");
}
int hyres_gdn_dnorm_f16(const void* g, const void* y, const void* n, void* dn, long long P, int C, int inverse, int g16,
                        hyres_stream_t s) {
    HY_REQUIRE(g && y && n && dn, HYRES_E_ARG, "gdn_dnorm_f16: NULL");
    long long cnt = P * C;
    if (g16)
        hipLaunchKernelGGL((gdn_dnorm_kernel<true, true>), dim3(grid_for(cnt)), dim3(256), 0, as_stream(s),
                           (const float*)g, (const float*)y, (const float*)n, (float*)dn, cnt, inverse ? 0.5f : -0.5f);
    else
        hipLaunchKernelGGL((gdn_dnorm_kernel<true, false>), dim3(grid_for(cnt)), dim3(256), 0, as_stream(s),
                           (const float*)g, (const float*)y, (const float*)n, (float*)dn, cnt, inverse ? 0.5f : -0.5f);
    return HY_LAUNCH_CHECK("gdn_dnorm_f16");
}
int hyres_uniform_noise(float* out, long long n, unsigned long long seed, unsigned long long offset,
                        hyres_stream_t s) {
    HY_REQUIRE(out, HYRES_E_ARG, "uniform_noise: NULL");
    hipLaunchKernelGGL(uniform_noise_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), out, n, seed, offset);
    return HY_LAUNCH_CHECK("uniform_noise");
}

int hyres_uniform_noise_dev(float* out, long long n, unsigned long long* seed_dev, unsigned long long salt,
                            hyres_stream_t s) {
    HY_REQUIRE(out && seed_dev, HYRES_E_ARG, "uniform_noise_dev: NULL");
    hipLaunchKernelGGL(uniform_noise_dev_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), out, n,
                       (const unsigned long long*)seed_dev, salt);
    int rc = HY_LAUNCH_CHECK("uniform_noise_dev");
    if (rc) return rc;
    hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(64), 0, as_stream(s), seed_dev);
    return HY_LAUNCH_CHECK("seed_advance");
}

static int reduce2(void (*k)(const float*, long long, float*), const float* x, long long n, float* out, void* ws,
                   long long ws_bytes, hyres_stream_t s, const char* name) {
    int nb = grid_for(n, 4);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * 4, HYRES_E_WORKSPACE, "%s: workspace", name);
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, as_stream(s), x, n, (float*)ws);
    int rc = HY_LAUNCH_CHECK(name);
    if (rc) return rc;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, as_stream(s), (const float*)ws, nb, out, 0);
    return HY_LAUNCH_CHECK(name);
}
int hyres_sum_log(const float* x, long long n, float* out, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && out, HYRES_E_ARG, "sum_log: NULL");
    return reduce2(sum_log_kernel, x, n, out, ws, ws_bytes, s, "sum_log");
}
int hyres_sumsq(const float* x, long long n, double* out, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && out, HYRES_E_ARG, "sumsq: NULL");
    int nb = grid_for(n, 4);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * 8, HYRES_E_WORKSPACE, "sumsq: workspace");
    hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, as_stream(s), x, n, (double*)ws);
    int rc = HY_LAUNCH_CHECK("sumsq");
    if (rc) return rc;
    hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, as_stream(s), (const double*)ws, nb, out);
    return HY_LAUNCH_CHECK("sumsq");
}
int hyres_sum_sqdiff(const float* a, const float* b, long long n, float* out, void* ws, long long ws_bytes,
                     hyres_stream_t s) {
    HY_REQUIRE(a && b && out, HYRES_E_ARG, "sum_sqdiff: NULL");
    int nb = grid_for(n, 4);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * 4, HYRES_E_WORKSPACE, "sum_sqdiff: workspace");
    hipLaunchKernelGGL(sum_sqdiff_kernel, dim3(nb), dim3(256), 0, as_stream(s), a, b, n, (float*)ws);
    int rc = HY_LAUNCH_CHECK("sum_sqdiff");
    if (rc) return rc;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, as_stream(s), (const float*)ws, nb, out, 0);
    return HY_LAUNCH_CHECK("sum_sqdiff_final");
}
int hyres_scale_recip(const float* x, const float* coef, float scale, float* g, long long n, hyres_stream_t s) {
    HY_REQUIRE(x && coef && g, HYRES_E_ARG, "scale_recip: NULL");
    hipLaunchKernelGGL(scale_recip_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x, coef, scale, g, n);
    return HY_LAUNCH_CHECK("scale_recip");
}
int hyres_scale_diff(const float* a, const float* b, const float* coef, float scale, float* g, long long n,
                     hyres_stream_t s) {
    HY_REQUIRE(a && b && coef && g, HYRES_E_ARG, "scale_diff: NULL");
    hipLaunchKernelGGL(scale_diff_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), a, b, coef, scale, g, n);
    return HY_LAUNCH_CHECK("scale_diff");
}
int hyres_scale(const float* x, const float* coef, float scale, float* y, long long n, int accumulate,
                hyres_stream_t s) {
    HY_REQUIRE(x && y, HYRES_E_ARG, "scale: NULL");
    hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(s), x, coef, scale, y, n, accumulate);
    return HY_LAUNCH_CHECK("scale");
}
int hyres_rd_finalize(const float* sums, const float* jpeg_bpp, float lmbda, long long npx, long long nel,
                      float* const* out, hyres_stream_t s) {
    HY_REQUIRE(sums && out, HYRES_E_ARG, "rd_finalize: NULL");
    RdOut o;
    for (int i = 0; i < 6; ++i) {
        HY_REQUIRE(out[i], HYRES_E_ARG, "rd_finalize: NULL output %d", i);
        o.o[i] = out[i];
    }
    hipLaunchKernelGGL(rd_finalize_kernel, dim3(1), dim3(64), 0, as_stream(s), sums, jpeg_bpp, lmbda, (float)npx,
                       (float)nel, o);
    return HY_LAUNCH_CHECK("rd_finalize");
}
int hyres_rd_bwd_coef(const float* g0, const float* g1, const float* g2, const float* g3, const float* g4,
                      const float* g5, float lmbda, long long npx, long long nel, float* coef, hyres_stream_t s) {
    HY_REQUIRE(g0 && g1 && g2 && g3 && g4 && g5 && coef, HYRES_E_ARG, "rd_bwd_coef: NULL");
    hipLaunchKernelGGL(rd_bwd_coef_kernel, dim3(1), dim3(64), 0, as_stream(s), g0, g1, g2, g3, g4, g5, lmbda,
                       (float)npx, (float)nel, coef);
    return HY_LAUNCH_CHECK("rd_bwd_coef");
}
int hyres_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n, double lr,
                    double beta1, double beta2, double eps, float* step_dev, const double* sumsq, double max_norm,
                    const float* gscale, int skip, hyres_stream_t s) {
    HY_REQUIRE(param && grad && exp_avg && exp_avg_sq && step_dev, HYRES_E_ARG, "adam: NULL");
    HY_REQUIRE(skip >= 0 && skip <= 2 && (skip == 0 || sumsq), HYRES_E_ARG, "adam: skip mode %d needs sumsq", skip);
    AdamHyper h;
    h.lr = lr;
    h.beta1 = beta1;
    h.beta2 = beta2;
    h.eps = eps;
    h.max_norm = max_norm;
    h.omb1 = (float)(1.0 - beta1);
    h.omb2 = (float)(1.0 - beta2);
    h.epsf = (float)eps;
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 4)), dim3(256), 0, as_stream(s), param, grad, exp_avg,
                       exp_avg_sq, n, h, (const float*)step_dev, sumsq, gscale, skip);
    int rc = HY_LAUNCH_CHECK("adam");
    if (rc) return rc;
    hipLaunchKernelGGL(adam_finish_kernel, dim3(1), dim3(64), 0, as_stream(s), step_dev, sumsq, skip);
    return HY_LAUNCH_CHECK("adam_finish");
}
int hyres_grad_scaler_update(const double* sumsq, float* scale, float* inv_scale, int* growth_tracker,
                             double growth_factor, double backoff_factor, int growth_interval, hyres_stream_t s) {
    HY_REQUIRE(sumsq && scale && inv_scale && growth_tracker && growth_interval > 0, HYRES_E_ARG,
               "grad_scaler_update: bad args");
    hipLaunchKernelGGL(grad_scaler_update_kernel, dim3(1), dim3(64), 0, as_stream(s), sumsq, scale, inv_scale,
                       growth_tracker, (float)growth_factor, (float)backoff_factor, growth_interval);
    return HY_LAUNCH_CHECK("grad_scaler_update");
}

}  // extern "C"
