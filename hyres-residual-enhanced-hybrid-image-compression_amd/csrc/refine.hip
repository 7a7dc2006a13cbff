// MultiScaleRefine pieces (models/layers/enhancement.py) on gfx950: bilinear resampling with
// PyTorch's align_corners=False source-index rule, SEBlock, SpatialAttention (CBAM SA).
// Activations are NHWC; every kernel streams HBM with the channel index on the fastest lanes.
#include "common.h"

#include <cstdlib>

namespace hyres {

#define GRID_STRIDE(i, n) \
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

static inline int grid_for_r(long long n) {
    long long b = (n + 255) / 256;
    return (int)std::max<long long>(1, std::min<long long>(b, 8192));
}
// the PW_UNR-unrolled pointwise kernels: each thread takes PW_UNR float4 per pass, 8 blocks of 256 per CU resident
static inline int pw_grid(long long n4) {
    long long b = (n4 + 256LL * 4 - 1) / (256LL * 4);
    return (int)std::max<long long>(1, std::min<long long>(b, 2048));
}

constexpr int PW_UNR = 4;  // float4 per thread in flight in the pointwise kernels below
constexpr int SE_PRELU_PARTS = 2048;  // hyres_se_bwd_prelu's slope partials (<= pw_grid's 2048 blocks)

// torch area_pixel_compute_source_index (linear, align_corners=False): max(scale*(o+0.5)-0.5, 0)
__device__ __forceinline__ void src_index(float scale, int o, int in, int& i0, int& i1, float& l0, float& l1) {
    float src = scale * ((float)o + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    i0 = (int)src;
    if (i0 > in - 1) i0 = in - 1;
    i1 = i0 + ((i0 < in - 1) ? 1 : 0);
    l1 = src - (float)i0;
    l0 = 1.0f - l1;
}

// VEC channels per thread (4: float4 when C, ld % 4 == 0 and 16B-aligned pointers). One block row per
// output row (blockIdx.y = b*Ho + oh: the vertical stencil is block-uniform), threads over (ow, channel
// group) with 32-bit index math.
template <int VEC, bool H = false>
__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const float* x, int ldx, float* y, int ldy, int B, int Hi,
                                                           int Wi, int Ho, int Wo, int C, float sh, float sw, int acc) {
    // H: x and y fp16 in HBM (autocast inference), fp32 arithmetic, no accumulate
    const int CG = C / VEC;
    const int row = blockIdx.y;
    const int b = row / Ho, oh = row - b * Ho;
    int h0, h1;
    float lh0, lh1;
    src_index(sh, oh, Hi, h0, h1, lh0, lh1);
    const long long x0 = ((long long)b * Hi + h0) * Wi * ldx;  // element offsets of the two source rows
    const long long x1 = ((long long)b * Hi + h1) * Wi * ldx;
    const long long yr = (long long)row * Wo * ldy;
    const int n = Wo * CG;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int ow = i / CG;
        const int c = (i - ow * CG) * VEC;
        int w0, w1;
        float lw0, lw1;
        src_index(sw, ow, Wi, w0, w1, lw0, lw1);
        float* yp = y + yr + (long long)ow * ldy + c;
        if constexpr (VEC == 4) {
            const float4 a = ldv4<H>(x, x0 + w0 * ldx + c), bq = ldv4<H>(x, x0 + w1 * ldx + c);
            const float4 cq = ldv4<H>(x, x1 + w0 * ldx + c), d = ldv4<H>(x, x1 + w1 * ldx + c);
            float4 v;
            v.x = lh0 * (lw0 * a.x + lw1 * bq.x) + lh1 * (lw0 * cq.x + lw1 * d.x);
            v.y = lh0 * (lw0 * a.y + lw1 * bq.y) + lh1 * (lw0 * cq.y + lw1 * d.y);
            v.z = lh0 * (lw0 * a.z + lw1 * bq.z) + lh1 * (lw0 * cq.z + lw1 * d.z);
            v.w = lh0 * (lw0 * a.w + lw1 * bq.w) + lh1 * (lw0 * cq.w + lw1 * d.w);
            if constexpr (H) {
                stv4<true>(y, yr + (long long)ow * ldy + c, v);
            } else {
                if (acc) {
                    const float4 o = ld4(yp);
                    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
                }
                *reinterpret_cast<float4*>(yp) = v;
            }
        } else {
            static_assert(!H, "fp16 resampling on the float4 path only");
            const float* x0p = x + x0;
            const float* x1p = x + x1;
            const float v = lh0 * (lw0 * x0p[w0 * ldx + c] + lw1 * x0p[w1 * ldx + c]) +
                            lh1 * (lw0 * x1p[w0 * ldx + c] + lw1 * x1p[w1 * ldx + c]);
            *yp = acc ? *yp + v : v;
        }
    }
}

// gather-form backward: for input pixel (h,w) sum over outputs whose stencil touches it
__device__ __forceinline__ float bw_weight(float scale, int o, int in, int target) {
    int i0, i1;
    float l0, l1;
    src_index(scale, o, in, i0, i1, l0, l1);
    float w = 0.f;
    if (i0 == target) w += l0;
    if (i1 == target) w += l1;
    return w;
}

__device__ __forceinline__ void bw_range(float inv, int t, int in, int out, int& lo, int& hi) {
    // outputs o with src(o) in [t-1, t+1] : o in [(t-0.5)/s - 0.5, (t+1.5)/s - 0.5]
    lo = max(0, (int)floorf(((float)t - 0.5f) * inv - 0.5f) - 1);
    hi = min(out - 1, (int)ceilf(((float)t + 1.5f) * inv - 0.5f) + 1);
    if (t == 0) lo = 0;
    if (t == in - 1) hi = out - 1;
}

// one block row per input row (blockIdx.y = b*Hi + h): the vertical output range and weights are
// block-uniform; threads over (w, channel group)
// the bilinear PReLU fold's block partials (one per 256-thread block: 16,384 at 128^2 x 16) summed in a fixed order and
// ADDED to the slope gradient, 8 loads in flight per thread
__global__ __launch_bounds__(256) void slope_sum8_kernel(const float* part, int n, float* dst) {
    __shared__ float red[256];
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int i = threadIdx.x;
    for (; i + 7 * 256 < n; i += 8 * 256)
#pragma unroll
        for (int k = 0; k < 8; ++k) s8[k] += part[i + k * 256];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (i + k * 256 < n) s8[k] += part[i + k * 256];
    red[threadIdx.x] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) dst[0] += red[0];
}

// PM (round 6, VEC == 4, acc == 0): the PReLU backward of the layer that produced the up-sampled map folded in —
// MultiScaleRefine's scales 2 and 3 end in conv + PReLU before the up-sample (enhancement.py:89-95,98-103): gx =
// pre > 0 ? g : slope * g with g the (G: fp16-rounded) gather sum, as prelu_bwd4_kernel on the stored gradient, and this
// block's share of sum_{pre <= 0} pre * g in part[block] (PM = 1: pre fp32, 2: pre fp16)
template <int VEC, bool G = false, int PM = 0>  // G: gy / gx fp16 (AMP fp16 gradients), fp32 sums
__global__ __launch_bounds__(256) void bilinear_bwd_kernel(const float* gy, int ldgy, float* gx, int ldgx, int B,
                                                           int Hi, int Wi, int Ho, int Wo, int C, float sh, float sw,
                                                           int acc, const float* pre, int ldpre, const float* slope,
                                                           float* part) {
    static_assert(PM == 0 || VEC == 4, "the PReLU fold runs on the vector kernel");
    float pslope = 0.f;
    const float a = PM ? slope[0] : 0.f;
    const int CG = C / VEC;
    const int row = blockIdx.y;
    const int b = row / Hi, h = row - b * Hi;
    int oh_lo, oh_hi;
    bw_range(1.0f / sh, h, Hi, Ho, oh_lo, oh_hi);
    const float isw = 1.0f / sw;
    const long long gb = (long long)b * Ho * Wo * ldgy;  // element offsets (the pointers may hold fp16)
    const long long gr = (long long)row * Wi * ldgx;
    const int n = Wi * CG;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int w = i / CG;
        const int c = (i - w * CG) * VEC;
        int ow_lo, ow_hi;
        bw_range(isw, w, Wi, Wo, ow_lo, ow_hi);
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int oh = oh_lo; oh <= oh_hi; ++oh) {
            const float wh = bw_weight(sh, oh, Hi, h);
            if (wh == 0.f) continue;
            float4 rs = make_float4(0.f, 0.f, 0.f, 0.f);
            const long long gq = gb + (long long)oh * Wo * ldgy + c;
            for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                const float ww = bw_weight(sw, ow, Wi, w);
                if (ww == 0.f) continue;
                const long long q = gq + (long long)ow * ldgy;
                if constexpr (VEC == 4) {
                    const float4 v = ldv4<G>(gy, q);
                    rs.x += ww * v.x; rs.y += ww * v.y; rs.z += ww * v.z; rs.w += ww * v.w;
                } else {
                    rs.x += ww * ldv<G>(gy, q);
                }
            }
            s.x += wh * rs.x; s.y += wh * rs.y; s.z += wh * rs.z; s.w += wh * rs.w;
        }
        const long long gp = gr + (long long)w * ldgx + c;
        if constexpr (PM != 0) {
            if constexpr (G) {  // the unfused chain's stored fp16 gradient
                s = make_float4((float)(_Float16)s.x, (float)(_Float16)s.y, (float)(_Float16)s.z, (float)(_Float16)s.w);
            }
            const float4 pv4 = ldv4<PM == 2>(pre, (long long)row * Wi * ldpre + (long long)w * ldpre + c);
            const float pv[4] = {pv4.x, pv4.y, pv4.z, pv4.w};
            float o[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!(pv[k] > 0.f)) pslope += pv[k] * o[k];
                o[k] = pv[k] > 0.f ? o[k] : a * o[k];
            }
            stv4<G>(gx, gp, make_float4(o[0], o[1], o[2], o[3]));
        } else if constexpr (VEC == 4) {
            if (acc) {
                const float4 o = ldv4<G>(gx, gp);
                s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
            }
            stv4<G>(gx, gp, s);
        } else {
            stv<G>(gx, gp, acc ? ldv<G>(gx, gp) + s.x : s.x);
        }
    }
    if constexpr (PM != 0) {  // wave sums (xor shuffles, a fixed order), then the four waves': one barrier per block
        __shared__ float red[4];
        for (int off = 32; off > 0; off >>= 1) pslope += __shfl_xor(pslope, off);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pslope;
        __syncthreads();
        if (threadIdx.x == 0) part[(long long)blockIdx.y * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    }
}

// backward of an exact integer down-sampling (enhancement.py:96,101: F.interpolate(scale_factor=1/S),
// S = 2 or 4, H_in = S*H_out): with align_corners=False every output o averages input pixels
// S*o + (S-2)/2 and the next one with weights 1/2 (src = S*(o+0.5)-0.5 is exact in fp32), so each
// input-gradient element receives exactly one 0.25*gy term or nothing — a streaming kernel instead of
// the general gather (which evaluates every candidate stencil weight per element); the same fp32 result
// (0.5 * (0.5 * g) == 0.25 * g).
template <int S, bool G = false>
__global__ __launch_bounds__(256) void bilinear_down_bwd_kernel(const float* gy, int ldgy, float* gx, int ldgx, int Hi,
                                                                int Wi, int Ho, int Wo, int C, int acc) {
    constexpr int A0 = (S - 2) / 2;
    const int CG = C / 4;
    const int row = blockIdx.y;
    const int b = row / Hi, h = row - b * Hi;
    const int dh = h - A0;
    const bool hok = dh >= 0 && (dh % S) < 2;
    const long long gyr = ((long long)b * Ho + (hok ? dh / S : 0)) * Wo;
    const long long gr = (long long)row * Wi * ldgx;
    const int n = Wi * CG;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int w = i / CG;
        const int c = (i - w * CG) * 4;
        const int dw = w - A0;
        const bool ok = hok && dw >= 0 && (dw % S) < 2;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) {
            const float4 g = ldv4<G>(gy, (gyr + dw / S) * ldgy + c);
            v = make_float4(0.25f * g.x, 0.25f * g.y, 0.25f * g.z, 0.25f * g.w);
        }
        const long long gp = gr + (long long)w * ldgx + c;
        if (acc) {
            const float4 o = ldv4<G>(gx, gp);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        stv4<G>(gx, gp, v);
    }
}

// ---------------------------------------------------------------- SEBlock
// pool partial: grid (B, nchunk), block 256: thread handles channels c = tid % C-ish
__global__ void se_pool_kernel(const float* x, int HW, int C, int per, float* part) {
    const int b = blockIdx.x, ch = blockIdx.y;
    const int p0 = ch * per, p1 = min(HW, p0 + per);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int p = p0; p < p1; ++p) s += x[((long long)b * HW + p) * C + c];
        part[((long long)b * gridDim.y + ch) * C + c] = s;
    }
}
__global__ void se_fc_kernel(const float* part, int nch, const float* w1, const float* w2, float* pooled, float* hidden,
                             float* sgate, int HW, int C, int Cr) {
    const int b = blockIdx.x;
    extern __shared__ float sm[];
    float* pm = sm;        // [C]
    float* hd = sm + C;    // [Cr]
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < nch; ++k) s += part[((long long)b * nch + k) * C + c];
        float m = s / (float)HW;
        pm[c] = m;
        pooled[b * C + c] = m;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < Cr; j += blockDim.x) {
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += w1[j * C + c] * pm[c];
        s = fmaxf(s, 0.f);
        hd[j] = s;
        hidden[b * Cr + j] = s;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int j = 0; j < Cr; ++j) s += w2[c * Cr + j] * hd[j];
        sgate[b * C + c] = 1.0f / (1.0f + expf(-s));
    }
}
// fp16 activations (autocast inference): x, y fp16, 4 channels per thread
// y = x * gate[b][c], 4 channels per thread (C % 4 == 0), 32-bit indices (B * HW * C / 4 < 2^31, host), UNR in flight;
// H: x, y fp16 (autocast inference)
template <bool H>
__global__ __launch_bounds__(256) void se_scale4_kernel(const float* x, const float* sgate, float* y, int B, int HW,
                                                        int C) {
    const int C4 = C >> 2, HWC4 = HW * C4;
    const int n = B * HWC4;
    const int stride = gridDim.x * 256;
    for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * PW_UNR) {
        float4 v[PW_UNR];
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i < n) v[u] = ldv4<H>(x, 4LL * i);
        }
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i >= n) continue;
            const int b = i / HWC4;
            const int c = 4 * (i - (i / C4) * C4);
            const float4 gt = ld4(sgate + b * C + c);
            stv4<H>(y, 4LL * i, make_float4(v[u].x * gt.x, v[u].y * gt.y, v[u].z * gt.z, v[u].w * gt.w));
        }
    }
}
__global__ void se_scale_kernel(const float* x, const float* sgate, float* y, int B, int HW, int C) {
    const long long n = (long long)B * HW * C;
    GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        const int b = (int)(i / ((long long)HW * C));
        y[i] = x[i] * sgate[b * C + c];
    }
}
// float4 variants (C % 4 == 0, 256 % (C/4) == 0): 256 threads = (C/4 channel groups) x (pixel lanes),
// every thread busy, deterministic LDS fold over the pixel lanes. SQ: sum of gy*x (backward) instead of x.
template <bool PROD, bool H = false, bool GH = false>  // GH: gy fp16
__global__ __launch_bounds__(256) void se_pool4_kernel(const float* x, const float* gy, int HW, int C, int per,
                                                       float* part) {
    __shared__ float4 red[256];
    const int b = blockIdx.x, ch = blockIdx.y;
    const int G = C >> 2, PL = 256 / G;
    const int g = threadIdx.x % G, lane = threadIdx.x / G;
    const int p0 = ch * per, p1 = min(HW, p0 + per);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = p0 + lane; p < p1; p += PL) {
        const long long i = ((long long)b * HW + p) * C + 4 * g;
        float4 v = ldv4<H>(x, i);
        if constexpr (PROD) {
            const float4 q = ldv4<GH>(gy, i);
            v.x *= q.x; v.y *= q.y; v.z *= q.z; v.w *= q.w;
        }
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < G) {
        float4 t = red[threadIdx.x];
        for (int l = 1; l < PL; ++l) {
            const float4 u = red[l * G + threadIdx.x];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        *reinterpret_cast<float4*>(part + ((long long)b * gridDim.y + ch) * C + 4 * threadIdx.x) = t;
    }
}
// backward: partial sums of gy*x per (b,c)
template <bool H = false, bool G = false>
__global__ void se_bwd_pool_kernel(const float* x, const float* gy, int HW, int C, int per, float* part) {
    const int b = blockIdx.x, ch = blockIdx.y;
    const int p0 = ch * per, p1 = min(HW, p0 + per);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f;
        for (int p = p0; p < p1; ++p) {
            long long i = ((long long)b * HW + p) * C + c;
            s += ldv<G>(gy, i) * ldv<H>(x, i);
        }
        part[((long long)b * gridDim.y + ch) * C + c] = s;
    }
}
// single block: all images (deterministic weight-gradient sums)
__global__ void se_fc_bwd_kernel(const float* part, int nch, int B, const float* w1, const float* w2,
                                 const float* pooled, const float* hidden, const float* sgate, float* gpool,
                                 float* gw1, float* gw2, int HW, int C, int Cr) {
    extern __shared__ float sm[];
    float* ga2 = sm;              // [B*C]
    float* gh = sm + B * C;       // [B*Cr]
    for (int idx = threadIdx.x; idx < B * C; idx += blockDim.x) {
        const int b = idx / C, c = idx % C;
        float s = 0.f;
        for (int k = 0; k < nch; ++k) s += part[((long long)b * nch + k) * C + c];
        const float sg = sgate[idx];
        ga2[idx] = s * sg * (1.0f - sg);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < B * Cr; idx += blockDim.x) {
        const int b = idx / Cr, j = idx % Cr;
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += w2[c * Cr + j] * ga2[b * C + c];
        gh[idx] = hidden[idx] > 0.f ? s : 0.f;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < C * Cr; idx += blockDim.x) {
        const int c = idx / Cr, j = idx % Cr;  // w2[c][j]
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += ga2[b * C + c] * hidden[b * Cr + j];
        gw2[idx] += s;
    }
    for (int idx = threadIdx.x; idx < Cr * C; idx += blockDim.x) {
        const int j = idx / C, c = idx % C;  // w1[j][c]
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += gh[b * Cr + j] * pooled[b * C + c];
        gw1[idx] += s;
    }
    for (int idx = threadIdx.x; idx < B * C; idx += blockDim.x) {
        const int b = idx / C, c = idx % C;
        float s = 0.f;
        for (int j = 0; j < Cr; ++j) s += w1[j * C + c] * gh[b * Cr + j];
        gpool[idx] = s / (float)HW;
    }
}
// gx = gy * gate[b][c] + gpool[b][c], 4 channels per thread (as se_scale4_kernel)
template <bool G>
__global__ __launch_bounds__(256) void se_bwd_x4_kernel(const float* gy, const float* sgate, const float* gpool,
                                                        float* gx, int B, int HW, int C) {
    const int C4 = C >> 2, HWC4 = HW * C4;
    const int n = B * HWC4;
    const int stride = gridDim.x * 256;
    for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * PW_UNR) {
        float4 v[PW_UNR];
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i < n) v[u] = ldv4<G>(gy, 4LL * i);
        }
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i >= n) continue;
            const int b = i / HWC4;
            const int c = 4 * (i - (i / C4) * C4);
            const float4 gt = ld4(sgate + b * C + c), gp = ld4(gpool + b * C + c);
            stv4<G>(gx, 4LL * i, make_float4(v[u].x * gt.x + gp.x, v[u].y * gt.y + gp.y, v[u].z * gt.z + gp.z,
                                             v[u].w * gt.w + gp.w));
        }
    }
}
// the same with the producing PReLU's backward folded in (hyres_se_bwd_prelu, fp32): gx = PReLU'(pre) * (gy * gate + gpool)
// and this block's share of the slope gradient sum_{pre <= 0} pre * (gy * gate + gpool) in part[blockIdx.x], elements
// in the same order as prelu_bwd4_kernel's per-thread sums. Round 6, AMP: H = pre fp16 (fp16 activations), G = gy / gx
// fp16 (fp16 gradients: the gradient is rounded to fp16 first, the unfused chain's stored value)
template <bool H = false, bool G = false>
__global__ __launch_bounds__(256) void se_bwd_x4_prelu_kernel(const float* gy, const float* sgate, const float* gpool,
                                                              float* gx, int B, int HW, int C, const float* pre,
                                                              const float* slope, float* part) {
    const int C4 = C >> 2, HWC4 = HW * C4;
    const int n = B * HWC4;
    const int stride = gridDim.x * 256;
    const float a = slope[0];
    float ps = 0.f;
    for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * PW_UNR) {
        float4 v[PW_UNR], pv[PW_UNR];
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i < n) {
                v[u] = ldv4<G>(gy, 4LL * i);
                pv[u] = ldv4<H>(pre, 4LL * i);
            }
        }
#pragma unroll
        for (int u = 0; u < PW_UNR; ++u) {
            const int i = i0 + u * stride;
            if (i >= n) continue;
            const int b = i / HWC4;
            const int c = 4 * (i - (i / C4) * C4);
            const float4 gt = ld4(sgate + b * C + c), gp = ld4(gpool + b * C + c);
            float o[4] = {v[u].x * gt.x + gp.x, v[u].y * gt.y + gp.y, v[u].z * gt.z + gp.z, v[u].w * gt.w + gp.w};
            const float q[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (G) o[k] = (float)(_Float16)o[k];
                if (!(q[k] > 0.f)) ps += q[k] * o[k];
                o[k] = q[k] > 0.f ? o[k] : a * o[k];
            }
            stv4<G>(gx, 4LL * i, make_float4(o[0], o[1], o[2], o[3]));
        }
    }
    __shared__ float red[256];
    red[threadIdx.x] = ps;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ __launch_bounds__(256) void se_prelu_slope_sum_kernel(const float* part, int n, float* dst) {
    __shared__ float red[256];
    float v = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) v += part[i];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) dst[0] += red[0];
}
template <bool G = false>
__global__ void se_bwd_x_kernel(const float* gy, const float* sgate, const float* gpool, float* gx, int B, int HW,
                                int C) {
    const long long n = (long long)B * HW * C;
    GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        const int b = (int)(i / ((long long)HW * C));
        stv<G>(gx, i, ldv<G>(gy, i) * sgate[b * C + c] + gpool[b * C + c]);
    }
}

// ---------------------------------------------------------------- SpatialAttention
// One wave per pixel (C <= 256, C % 4 == 0: float4 per lane): channel mean, max and the first-occurrence
// argmax (torch.max(dim=1) on CPU keeps the first maximal index; the backward routes g_max there).
// channel mean / max (+ first argmax, torch.max semantics) per pixel: 16 lanes per pixel (4 pixels per wave,
// each lane a float4 stride over the channels), folded with 4 xor-shuffles
// NC > 0 (round 6: C = 64 * NC, MultiScaleRefine's 192): the lane's NC float4 loads are all issued before the first
// compare — the runtime-bounded loop waited on each in turn (191 us at 256^2 x 16 x 192 fp32, ~4.2 TB/s); the same
// order of sums and compares, bit-identical
template <bool H = false, int NC = 0>
__global__ __launch_bounds__(256) void sa_pool_kernel(const float* x, float* pooled2, int* amax, long long P, int C) {
    const int l16 = threadIdx.x & 15;
    const long long p = (long long)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool ok = p < P;
    const long long xp = (ok ? p : 0) * C;
    float s = 0.f, m = -INFINITY;
    int mi = 0x7fffffff;
    if constexpr (NC > 0) {
        if (ok) {
            float4 vv[NC];
#pragma unroll
            for (int k = 0; k < NC; ++k) vv[k] = ldv4<H>(x, xp + 4 * l16 + 64 * k);
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const int c = 4 * l16 + 64 * k;
                const float4 v = vv[k];
                s += (v.x + v.y) + (v.z + v.w);
                if (v.x > m) { m = v.x; mi = c; }
                if (v.y > m) { m = v.y; mi = c + 1; }
                if (v.z > m) { m = v.z; mi = c + 2; }
                if (v.w > m) { m = v.w; mi = c + 3; }
            }
        }
    } else if (ok) {
        for (int c = 4 * l16; c < C; c += 64) {
            const float4 v = ldv4<H>(x, xp + c);
            s += (v.x + v.y) + (v.z + v.w);
            if (v.x > m) { m = v.x; mi = c; }
            if (v.y > m) { m = v.y; mi = c + 1; }
            if (v.z > m) { m = v.z; mi = c + 2; }
            if (v.w > m) { m = v.w; mi = c + 3; }
        }
    }
    for (int off = 8; off > 0; off >>= 1) {
        s += __shfl_xor(s, off);
        const float om = __shfl_xor(m, off);
        const int oi = __shfl_xor(mi, off);
        if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
    }
    if (ok && l16 == 0) {
        pooled2[p * 2 + 0] = s / (float)C;
        pooled2[p * 2 + 1] = m;
        amax[p] = mi;
    }
}
// y = x * attn[p], float4 over channels (C % 4 == 0)
template <bool H = false>
__global__ void sa_mul_kernel(const float* x, const float* attn, float* y, long long P, int C) {
    const int C4 = C >> 2;
    const long long n = P * C4;
    GRID_STRIDE(i, n) {
        const long long p = i / C4;
        const float a = attn[p];
        float4 v = ldv4<H>(x, 4 * i);
        v.x *= a; v.y *= a; v.z *= a; v.w *= a;
        stv4<H>(y, 4 * i, v);
    }
}
// bwd 1: g_logit[p] = (sum_c gy*x) * a*(1-a)
template <bool H = false, bool G = false>
__global__ void sa_bwd_logit_kernel(const float* x, const float* gy, const float* attn, float* glogit, long long P,
                                    int C) {
    // 16 lanes per pixel (4 pixels per wave), 4 xor-shuffles
    const int l16 = threadIdx.x & 15;
    const long long p = (long long)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool ok = p < P;
    float s = 0.f;
    if (ok) {
        for (int c = 4 * l16; c < C; c += 64) {
            const float4 g = ldv4<G>(gy, p * C + c);
            const float4 v = ldv4<H>(x, p * C + c);
            s += (g.x * v.x + g.y * v.y) + (g.z * v.z + g.w * v.w);
        }
    }
    for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (ok && l16 == 0) {
        float a = attn[p];
        glogit[p] = s * a * (1.0f - a);
    }
}
// ---- SpatialAttention's 7x7 (2 -> 1) conv on 16 x 16 pixel tiles staged with their 3-pixel halo in LDS (the
// per-pixel kernels above gather every tap from global memory: 71 us forward / 179 us backward at 16 x 256^2).
constexpr int SA_T = 16, SA_L = SA_T + 6;
__device__ __forceinline__ void sa_tile_of(int B, int H, int W, int& b, int& h0, int& w0) {
    const int tw = (W + SA_T - 1) / SA_T, th = (H + SA_T - 1) / SA_T;
    int t = blockIdx.x;
    const int tx = t % tw; t /= tw;
    const int ty = t % th;
    b = t / th;
    h0 = ty * SA_T;
    w0 = tx * SA_T;
}
// forward: attn = sigmoid(sum_{ch, kh, kw} w * pooled2), the per-pixel kernel's summation order (bit-identical)
__global__ __launch_bounds__(256) void sa_conv_tiled_kernel(const float* pooled2, const float* w, float* attn, int B,
                                                            int H, int W) {
    __shared__ float ws[98];
    __shared__ float pl[2][SA_L][SA_L + 1];
    int b, h0, w0;
    sa_tile_of(B, H, W, b, h0, w0);
    const int tid = threadIdx.x;
    if (tid < 98) ws[tid] = w[tid];
    for (int e = tid; e < SA_L * SA_L; e += 256) {
        const int ly = e / SA_L, lx = e - ly * SA_L;
        const int ih = h0 - 3 + ly, iw = w0 - 3 + lx;
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const float2 v = ok ? *reinterpret_cast<const float2*>(pooled2 + (((long long)b * H + ih) * W + iw) * 2)
                            : make_float2(0.f, 0.f);
        pl[0][ly][lx] = v.x;
        pl[1][ly][lx] = v.y;
    }
    __syncthreads();
    const int ty = tid / SA_T, tx = tid % SA_T;
    const int hh = h0 + ty, ww = w0 + tx;
    if (hh >= H || ww >= W) return;
    float s = 0.f;
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
            const int ih = hh + kh - 3;
            if (ih < 0 || ih >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 7; ++kw) {
                const int iw = ww + kw - 3;
                if (iw < 0 || iw >= W) continue;
                s += ws[ch * 49 + kh * 7 + kw] * pl[ch][ty + kh][tx + kw];
            }
        }
    attn[((long long)b * H + hh) * W + ww] = 1.0f / (1.0f + expf(-s));
}
// backward: gpooled2 (the per-pixel kernel's order: bit-identical) and per-tile weight-gradient partials (98 taps x 2
// half-tiles of 8 rows, summed in a fixed order); C > 0: the mean's gradient stored divided by C (HYRES_EPI_SA_BWD)
__global__ __launch_bounds__(256) void sa_bwd_conv_tiled_kernel(const float* glogit, const float* pooled2,
                                                                const float* w, float* gpooled2, float* wpart, int B,
                                                                int H, int W, int C) {
    __shared__ float ws[98];
    __shared__ float gl[SA_L][SA_L + 1];
    __shared__ float pl[2][SA_L][SA_L + 1];
    __shared__ float half2s[98];
    int b, h0, w0;
    sa_tile_of(B, H, W, b, h0, w0);
    const int tid = threadIdx.x;
    if (tid < 98) ws[tid] = w[tid];
    for (int e = tid; e < SA_L * SA_L; e += 256) {
        const int ly = e / SA_L, lx = e - ly * SA_L;
        const int ih = h0 - 3 + ly, iw = w0 - 3 + lx;
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const long long p = ((long long)b * H + ih) * W + iw;
        const float2 v = ok ? *reinterpret_cast<const float2*>(pooled2 + p * 2) : make_float2(0.f, 0.f);
        gl[ly][lx] = ok ? glogit[p] : 0.f;
        pl[0][ly][lx] = v.x;
        pl[1][ly][lx] = v.y;
    }
    __syncthreads();
    {
        const int ty = tid / SA_T, tx = tid % SA_T;
        const int hh = h0 + ty, ww = w0 + tx;
        if (hh < H && ww < W) {
            float g0 = 0.f, g1 = 0.f;
#pragma unroll
            for (int kh = 0; kh < 7; ++kh)
#pragma unroll
                for (int kw = 0; kw < 7; ++kw) {
                    const float go = gl[ty + 6 - kh][tx + 6 - kw];  // output (hh - kh + 3, ww - kw + 3); 0 outside
                    g0 += ws[kh * 7 + kw] * go;
                    g1 += ws[49 + kh * 7 + kw] * go;
                }
            const long long i = ((long long)b * H + hh) * W + ww;
            gpooled2[i * 2 + 0] = C > 0 ? g0 / (float)C : g0;
            gpooled2[i * 2 + 1] = g1;
        }
    }
    // weight gradient: tap k = (ch, kh, kw) sums glogit[p] * pooled2[ch][p + (kh - 3, kw - 3)] over the tile's pixels
    // (glogit is 0 outside the image), rows [8 * hf, 8 * hf + 8) per half
    float acc = 0.f;
    const int k = tid % 98, hf = tid / 98;
    if (tid < 196) {
        const int ch = k / 49, kh = (k % 49) / 7, kw = k % 7;
        for (int ty = 8 * hf; ty < 8 * hf + 8; ++ty)
#pragma unroll
            for (int tx = 0; tx < SA_T; ++tx) acc += gl[ty + 3][tx + 3] * pl[ch][ty + kh][tx + kw];
        if (hf == 1) half2s[k] = acc;
    }
    __syncthreads();
    if (tid < 98) wpart[(long long)blockIdx.x * 98 + tid] = acc + half2s[tid];
}
// one block per weight tap: 256 threads fold the per-block partials (deterministic order)
__global__ void sa_bwd_wfinal_kernel(const float* wpart, int nb, float* gw) {
    __shared__ float red[256];
    const int k = blockIdx.x;
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += 256) s += wpart[(long long)b * 98 + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) gw[k] += red[0];
}
// bwd 3: gx = gy*a + g_avg/C + [c == argmax] * g_max     (float4 over channels; argmax saved by the pool)
template <bool G = false>
__global__ void sa_bwd_x_kernel(const float* gy, const float* attn, const float* gpooled2, const int* amax, float* gx,
                                long long P, int C) {
    const int C4 = C >> 2;
    const long long n = P * C4;
    GRID_STRIDE(i, n) {
        const long long p = i / C4;
        const int c = (int)(i - p * C4) * 4;
        const float a = attn[p];
        const float gavg = gpooled2[p * 2 + 0] / (float)C;
        const float gmax = gpooled2[p * 2 + 1];
        const int mi = amax[p];
        float4 v = ldv4<G>(gy, 4 * i);
        v.x = v.x * a + gavg + (c == mi ? gmax : 0.f);
        v.y = v.y * a + gavg + (c + 1 == mi ? gmax : 0.f);
        v.z = v.z * a + gavg + (c + 2 == mi ? gmax : 0.f);
        v.w = v.w * a + gavg + (c + 3 == mi ? gmax : 0.f);
        stv4<G>(gx, 4 * i, v);
    }
}

// ---- training with SpatialAttention's multiply folded into the fusion 1x1 (HYRES_EPI_ROWSCALE forward):
// h = PReLU(pre), pre = attn[p] * (W multi)[p] + b. Per pixel (16 lanes, a float4 of the C <= 64 channels each):
// gp = PReLU-backward(gy); gs = attn * gp (the fusion 1x1's weight- and input-gradient operand: d W = sum gs x multi,
// d multi = W^T gs, exactly the reference's gradients through multi * attn); glogit = (1 - attn) * sum_o gp (pre - b),
// which is attn (1 - attn) * sum_o gp z with attn z = pre - b (the gradient at the attention logit, no division by
// attn). Per-block partials of d bias (sum gp) and d slope (sum over pre <= 0 of gy pre, prelu_bwd4_kernel's order).
__global__ __launch_bounds__(256) void sa_fold_bwd_kernel(const float* pre, int ldpre, const float* gy, int ldg,
                                                          const float* attn, const float* bias, const float* slope,
                                                          float* gs, float* glogit, float* part, long long P, int C) {
    __shared__ float rb[16][68];
    __shared__ float rs[256];
    const float a = slope[0];
    const int l16 = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int c = 4 * l16;
    const bool cok = c < C;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = cok ? *reinterpret_cast<const float4*>(bias + c) : z4;
    float4 bs = z4;
    float ss = 0.f;
    // every lane of a 16-lane group walks the same pixels, so the group's xor-shuffles never mix groups
    for (long long p = (long long)blockIdx.x * 16 + grp; p < P; p += (long long)gridDim.x * 16) {
        const float4 pv = cok ? *reinterpret_cast<const float4*>(pre + p * ldpre + c) : z4;
        const float4 gv = cok ? *reinterpret_cast<const float4*>(gy + p * ldg + c) : z4;
        const float at = attn[p];
        const float4 gp = make_float4(pv.x > 0.f ? gv.x : a * gv.x, pv.y > 0.f ? gv.y : a * gv.y,
                                      pv.z > 0.f ? gv.z : a * gv.z, pv.w > 0.f ? gv.w : a * gv.w);
        if (!(pv.x > 0.f)) ss += pv.x * gv.x;
        if (!(pv.y > 0.f)) ss += pv.y * gv.y;
        if (!(pv.z > 0.f)) ss += pv.z * gv.z;
        if (!(pv.w > 0.f)) ss += pv.w * gv.w;
        bs.x += gp.x; bs.y += gp.y; bs.z += gp.z; bs.w += gp.w;
        float d = (gp.x * (pv.x - b.x) + gp.y * (pv.y - b.y)) + (gp.z * (pv.z - b.z) + gp.w * (pv.w - b.w));
        if (cok) *reinterpret_cast<float4*>(gs + p * C + c) = make_float4(at * gp.x, at * gp.y, at * gp.z, at * gp.w);
        for (int off = 8; off > 0; off >>= 1) d += __shfl_xor(d, off);
        if (l16 == 0) glogit[p] = d * (1.0f - at);
    }
    if (cok) *reinterpret_cast<float4*>(&rb[grp][c]) = bs;
    rs[threadIdx.x] = ss;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) rs[threadIdx.x] += rs[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x < C) {
        float t = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) t += rb[g][threadIdx.x];
        part[(long long)blockIdx.x * (C + 1) + threadIdx.x] = t;
    }
    if (threadIdx.x == 0) part[(long long)blockIdx.x * (C + 1) + C] = rs[0];
}
// The fp16-activation build (AMP training): 8 lanes per pixel, 8 channels (one 16-byte fp16 row piece) each — the
// 16-lane float4 mapping above moves fp16 rows as 8-byte pieces and measured 169 us at 256^2 x 16 (r7h). Same
// arithmetic per element, d summed over 8 lanes (xor 4, 2, 1), per-block partials in the same layout.
template <bool G>
__global__ __launch_bounds__(256) void sa_fold_bwd_h8_kernel(const float* pre, int ldpre, const float* gy, int ldg,
                                                             const float* attn, const float* bias, const float* slope,
                                                             float* gs, float* glogit, float* part, long long P,
                                                             int C) {
    typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
    __shared__ float rb[32][68];
    __shared__ float rs[256];
    const float a = slope[0];
    const int l8 = threadIdx.x & 7, grp = threadIdx.x >> 3;
    const int c = 8 * l8;
    const bool cok = c < C;
    float b[8], bs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        b[k] = cok ? bias[c + k] : 0.f;
        bs[k] = 0.f;
    }
    float ss = 0.f;
    const _Float16* preh = reinterpret_cast<const _Float16*>(pre);
    // every lane of an 8-lane group walks the same pixels, so the group's xor-shuffles never mix groups
    for (long long p = (long long)blockIdx.x * 32 + grp; p < P; p += (long long)gridDim.x * 32) {
        float pv[8], gv[8];
        if (cok) {
            const h8_t ph = *reinterpret_cast<const h8_t*>(preh + p * ldpre + c);
#pragma unroll
            for (int k = 0; k < 8; ++k) pv[k] = (float)ph[k];
            if constexpr (G) {
                const h8_t gh = *reinterpret_cast<const h8_t*>(reinterpret_cast<const _Float16*>(gy) + p * ldg + c);
#pragma unroll
                for (int k = 0; k < 8; ++k) gv[k] = (float)gh[k];
            } else {
                const float4 g0 = *reinterpret_cast<const float4*>(gy + p * ldg + c);
                const float4 g1 = *reinterpret_cast<const float4*>(gy + p * ldg + c + 4);
                gv[0] = g0.x; gv[1] = g0.y; gv[2] = g0.z; gv[3] = g0.w;
                gv[4] = g1.x; gv[5] = g1.y; gv[6] = g1.z; gv[7] = g1.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) pv[k] = gv[k] = 0.f;
        }
        const float at = attn[p];
        float gp[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            gp[k] = pv[k] > 0.f ? gv[k] : a * gv[k];
            if (!(pv[k] > 0.f)) ss += pv[k] * gv[k];
            bs[k] += gp[k];
        }
        // sa_fold_bwd_kernel's pairing within each float4, then the two halves
        float d = ((gp[0] * (pv[0] - b[0]) + gp[1] * (pv[1] - b[1])) + (gp[2] * (pv[2] - b[2]) + gp[3] * (pv[3] - b[3]))) +
                  ((gp[4] * (pv[4] - b[4]) + gp[5] * (pv[5] - b[5])) + (gp[6] * (pv[6] - b[6]) + gp[7] * (pv[7] - b[7])));
        if (cok) {
            if constexpr (G) {
                h8_t o;
#pragma unroll
                for (int k = 0; k < 8; ++k) o[k] = (_Float16)(at * gp[k]);
                *reinterpret_cast<h8_t*>(reinterpret_cast<_Float16*>(gs) + p * C + c) = o;
            } else {
                *reinterpret_cast<float4*>(gs + p * C + c) = make_float4(at * gp[0], at * gp[1], at * gp[2], at * gp[3]);
                *reinterpret_cast<float4*>(gs + p * C + c + 4) = make_float4(at * gp[4], at * gp[5], at * gp[6], at * gp[7]);
            }
        }
        for (int off = 4; off > 0; off >>= 1) d += __shfl_xor(d, off);
        if (l8 == 0) glogit[p] = d * (1.0f - at);
    }
    if (cok) {
#pragma unroll
        for (int k = 0; k < 8; ++k) rb[grp][c + k] = bs[k];
    }
    rs[threadIdx.x] = ss;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) rs[threadIdx.x] += rs[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x < C) {
        float t = 0.f;
#pragma unroll
        for (int g = 0; g < 32; ++g) t += rb[g][threadIdx.x];
        part[(long long)blockIdx.x * (C + 1) + threadIdx.x] = t;
    }
    if (threadIdx.x == 0) part[(long long)blockIdx.x * (C + 1) + C] = rs[0];
}
// one block per output (C bias channels, then the slope): the partials folded in a fixed order, ADDED to the gradient
__global__ __launch_bounds__(256) void sa_fold_final_kernel(const float* part, int nb, int C, float* dbias,
                                                            float* dslope) {
    __shared__ float red[256];
    const int k = blockIdx.x;
    float s = 0.f;
    for (int i = threadIdx.x; i < nb; i += 256) s += part[(long long)i * (C + 1) + k];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (k < C) dbias[k] += red[0];
        else dslope[0] += red[0];
    }
}

}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_bilinear_fwd(const float* x, int ldx, float* y, int ldy, int B, int Hi, int Wi, int Ho, int Wo, int C,
                       float scale_h, float scale_w, int accumulate, hyres_stream_t s) {
    HY_REQUIRE(x && y && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, HYRES_E_ARG, "bilinear_fwd: bad args");
    const bool vec = C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && aligned16(x) && aligned16(y);
    HY_REQUIRE((long long)B * Ho <= 65535 && (long long)Wo * C < (1LL << 30), HYRES_E_SHAPE, "bilinear_fwd: too large");
    const dim3 grid(ceil_div((long long)Wo * (vec ? C / 4 : C), 256), B * Ho);
    if (vec)
        hipLaunchKernelGGL(bilinear_fwd_kernel<4>, grid, dim3(256), 0, as_stream(s), x, ldx, y, ldy, B, Hi, Wi, Ho, Wo,
                           C, scale_h, scale_w, accumulate);
    else
        hipLaunchKernelGGL(bilinear_fwd_kernel<1>, grid, dim3(256), 0, as_stream(s), x, ldx, y, ldy, B, Hi, Wi, Ho, Wo,
                           C, scale_h, scale_w, accumulate);
    return HY_LAUNCH_CHECK("bilinear_fwd");
}
int hyres_bilinear_fwd_f16(const void* x, int ldx, void* y, int ldy, int B, int Hi, int Wi, int Ho, int Wo, int C,
                           float scale_h, float scale_w, hyres_stream_t s) {
    HY_REQUIRE(x && y && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, HYRES_E_ARG, "bilinear_fwd_f16: bad args");
    HY_REQUIRE(C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0 &&
                   (reinterpret_cast<uintptr_t>(y) & 7) == 0,
               HYRES_E_ALIGN, "bilinear_fwd_f16: C, ld %% 4 == 0 and 8B-aligned x/y required");
    HY_REQUIRE((long long)B * Ho <= 65535 && (long long)Wo * C < (1LL << 30), HYRES_E_SHAPE, "bilinear_fwd_f16: too large");
    const dim3 grid(ceil_div((long long)Wo * (C / 4), 256), B * Ho);
    hipLaunchKernelGGL((bilinear_fwd_kernel<4, true>), grid, dim3(256), 0, as_stream(s), (const float*)x, ldx, (float*)y,
                       ldy, B, Hi, Wi, Ho, Wo, C, scale_h, scale_w, 0);
    return HY_LAUNCH_CHECK("bilinear_fwd_f16");
}
extern "C++" {
template <bool G>
static int bilinear_bwd_impl(const float* gy, int ldgy, float* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo, int C,
                             float scale_h, float scale_w, int accumulate, hyres_stream_t s) {
    HY_REQUIRE(gy && gx, HYRES_E_ARG, "bilinear_bwd: NULL");
    const unsigned am = G ? 7u : 15u;  // 4-element vectors: 8 B (fp16) / 16 B (fp32)
    const bool vec = C % 4 == 0 && ldgy % 4 == 0 && ldgx % 4 == 0 && (reinterpret_cast<uintptr_t>(gy) & am) == 0 &&
                     (reinterpret_cast<uintptr_t>(gx) & am) == 0;
    HY_REQUIRE((long long)B * Hi <= 65535 && (long long)Wi * C < (1LL << 30), HYRES_E_SHAPE, "bilinear_bwd: too large");
    const dim3 grid(ceil_div((long long)Wi * (vec ? C / 4 : C), 256), B * Hi);
    for (int S = 2; S <= 4 && vec; S += 2) {
        if (scale_h != (float)S || scale_w != (float)S || Hi != S * Ho || Wi != S * Wo) continue;
        if (S == 2)
            hipLaunchKernelGGL((bilinear_down_bwd_kernel<2, G>), grid, dim3(256), 0, as_stream(s), gy, ldgy, gx, ldgx,
                               Hi, Wi, Ho, Wo, C, accumulate);
        else
            hipLaunchKernelGGL((bilinear_down_bwd_kernel<4, G>), grid, dim3(256), 0, as_stream(s), gy, ldgy, gx, ldgx,
                               Hi, Wi, Ho, Wo, C, accumulate);
        return HY_LAUNCH_CHECK("bilinear_down_bwd");
    }
    if (vec)
        hipLaunchKernelGGL((bilinear_bwd_kernel<4, G>), grid, dim3(256), 0, as_stream(s), gy, ldgy, gx, ldgx, B, Hi, Wi,
                           Ho, Wo, C, scale_h, scale_w, accumulate, nullptr, 0, nullptr, nullptr);
    else
        hipLaunchKernelGGL((bilinear_bwd_kernel<1, G>), grid, dim3(256), 0, as_stream(s), gy, ldgy, gx, ldgx, B, Hi, Wi,
                           Ho, Wo, C, scale_h, scale_w, accumulate, nullptr, 0, nullptr, nullptr);
    return HY_LAUNCH_CHECK("bilinear_bwd");
}
static dim3 bilinear_bwd_grid(int B, int Hi, int Wi, int C) { return dim3(ceil_div((long long)Wi * (C / 4), 256), B * Hi); }
}  // extern "C++"
long long hyres_bilinear_bwd_prelu_workspace_bytes(int B, int Hi, int Wi, int C) {
    const dim3 g = bilinear_bwd_grid(B, Hi, Wi, C);
    return (long long)g.x * g.y * 4;
}
int hyres_bilinear_bwd_prelu(const void* gy, int ldgy, void* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo, int C,
                             float scale_h, float scale_w, const void* pre, int ldpre, const float* slope, float* dslope,
                             void* ws, long long ws_bytes, int io, hyres_stream_t s) {
    HY_REQUIRE(gy && gx && pre && slope && dslope && ws && io >= 0 && io <= 3, HYRES_E_ARG, "bilinear_bwd_prelu: NULL / io");
    const bool G = io & 1, H = io & 2;
    const unsigned ag = G ? 7u : 15u, ap = H ? 7u : 15u;
    HY_REQUIRE(C % 4 == 0 && ldgy % 4 == 0 && ldgx % 4 == 0 && ldpre % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(gy) & ag) == 0 && (reinterpret_cast<uintptr_t>(gx) & ag) == 0 &&
                   (reinterpret_cast<uintptr_t>(pre) & ap) == 0,
               HYRES_E_ALIGN, "bilinear_bwd_prelu: C %% 4 == 0, aligned rows");
    HY_REQUIRE((long long)B * Hi <= 65535 && (long long)Wi * C < (1LL << 30), HYRES_E_SHAPE, "bilinear_bwd_prelu: too large");
    HY_REQUIRE(ws_bytes >= hyres_bilinear_bwd_prelu_workspace_bytes(B, Hi, Wi, C), HYRES_E_WORKSPACE,
               "bilinear_bwd_prelu: workspace");
    const dim3 grid = bilinear_bwd_grid(B, Hi, Wi, C);
    hipStream_t st = as_stream(s);
    const float* g = (const float*)gy;
    float* x = (float*)gx;
    const float* p = (const float*)pre;
    float* part = (float*)ws;
#define HY_BBP(GG, PMV)                                                                                                  \
    hipLaunchKernelGGL((bilinear_bwd_kernel<4, GG, PMV>), grid, dim3(256), 0, st, g, ldgy, x, ldgx, B, Hi, Wi, Ho, Wo, C, \
                       scale_h, scale_w, 0, p, ldpre, slope, part)
    if (G && H) {
        HY_BBP(true, 2);
    } else if (G) {
        HY_BBP(true, 1);
    } else if (H) {
        HY_BBP(false, 2);
    } else {
        HY_BBP(false, 1);
    }
#undef HY_BBP
    int rc = HY_LAUNCH_CHECK("bilinear_bwd_prelu");
    if (rc) return rc;
    hipLaunchKernelGGL(slope_sum8_kernel, dim3(1), dim3(256), 0, st, (const float*)part, (int)(grid.x * grid.y), dslope);
    return HY_LAUNCH_CHECK("bilinear_bwd_prelu_final");
}
int hyres_bilinear_bwd(const float* gy, int ldgy, float* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo, int C,
                       float scale_h, float scale_w, int accumulate, hyres_stream_t s) {
    return bilinear_bwd_impl<false>(gy, ldgy, gx, ldgx, B, Hi, Wi, Ho, Wo, C, scale_h, scale_w, accumulate, s);
}
int hyres_bilinear_bwd_f16(const void* gy, int ldgy, void* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo, int C,
                           float scale_h, float scale_w, int accumulate, hyres_stream_t s) {
    return bilinear_bwd_impl<true>((const float*)gy, ldgy, (float*)gx, ldgx, B, Hi, Wi, Ho, Wo, C, scale_h, scale_w,
                                   accumulate, s);
}

static int se_chunks(int HW) { return std::max(1, std::min(64, (HW + 1023) / 1024)); }

long long hyres_se_workspace_bytes(int B, int HW, int C) { return (long long)B * se_chunks(HW) * C * 4; }

int hyres_se_fwd(const float* x, const float* w1, const float* w2, float* y, float* pooled, float* hidden,
                 float* sgate, int B, int HW, int C, int Cr, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && w1 && w2 && y && pooled && hidden && sgate, HYRES_E_ARG, "se_fwd: NULL");
    const int nch = se_chunks(HW);
    HY_REQUIRE(ws && ws_bytes >= (long long)B * nch * C * 4, HYRES_E_WORKSPACE, "se_fwd: workspace");
    const int per = (HW + nch - 1) / nch;
    hipStream_t st = as_stream(s);
    if (C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0 && aligned16(x))
        hipLaunchKernelGGL(se_pool4_kernel<false>, dim3(B, nch), dim3(256), 0, st, x, (const float*)nullptr, HW, C,
                           per, (float*)ws);
    else
        hipLaunchKernelGGL(se_pool_kernel, dim3(B, nch), dim3(256), 0, st, x, HW, C, per, (float*)ws);
    int rc = HY_LAUNCH_CHECK("se_pool");
    if (rc) return rc;
    hipLaunchKernelGGL(se_fc_kernel, dim3(B), dim3(256), (C + Cr) * 4, st, (const float*)ws, nch, w1, w2, pooled,
                       hidden, sgate, HW, C, Cr);
    rc = HY_LAUNCH_CHECK("se_fc");
    if (rc) return rc;
    long long n = (long long)B * HW * C;
    if (C % 4 == 0 && aligned16(x) && aligned16(y) && n / 4 < (1LL << 31))
        hipLaunchKernelGGL(se_scale4_kernel<false>, dim3(pw_grid(n / 4)), dim3(256), 0, st, x, (const float*)sgate, y, B,
                           HW, C);
    else
        hipLaunchKernelGGL(se_scale_kernel, dim3(grid_for_r(n)), dim3(256), 0, st, x, (const float*)sgate, y, B, HW, C);
    return HY_LAUNCH_CHECK("se_scale");
}

int hyres_se_fwd_f16(const void* x, const float* w1, const float* w2, void* y, float* pooled, float* hidden,
                     float* sgate, int B, int HW, int C, int Cr, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && w1 && w2 && y && pooled && hidden && sgate, HYRES_E_ARG, "se_fwd_f16: NULL");
    HY_REQUIRE(C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0 &&
                   (reinterpret_cast<uintptr_t>(y) & 7) == 0,
               HYRES_E_ALIGN, "se_fwd_f16: C %% 4 == 0, 256 %% (C/4) == 0, 8B-aligned x/y required");
    const int nch = se_chunks(HW);
    HY_REQUIRE(ws && ws_bytes >= (long long)B * nch * C * 4, HYRES_E_WORKSPACE, "se_fwd_f16: workspace");
    const int per = (HW + nch - 1) / nch;
    hipStream_t st = as_stream(s);
    hipLaunchKernelGGL((se_pool4_kernel<false, true>), dim3(B, nch), dim3(256), 0, st, (const float*)x,
                       (const float*)nullptr, HW, C, per, (float*)ws);
    int rc = HY_LAUNCH_CHECK("se_pool_f16");
    if (rc) return rc;
    hipLaunchKernelGGL(se_fc_kernel, dim3(B), dim3(256), (C + Cr) * 4, st, (const float*)ws, nch, w1, w2, pooled,
                       hidden, sgate, HW, C, Cr);
    rc = HY_LAUNCH_CHECK("se_fc");
    if (rc) return rc;
    const long long n = (long long)B * HW * C / 4;
    HY_REQUIRE(n < (1LL << 31), HYRES_E_SHAPE, "se_fwd_f16: too large");
    hipLaunchKernelGGL(se_scale4_kernel<true>, dim3(pw_grid(n)), dim3(256), 0, st, (const float*)x, (const float*)sgate,
                       (float*)y, B, HW, C);
    return HY_LAUNCH_CHECK("se_scale_f16");
}

extern "C++" {
template <bool H, bool G>
static int se_bwd_impl(const float* x, const float* gy, const float* w1, const float* w2, const float* pooled,
                       const float* hidden, const float* sgate, float* gx, float* gw1, float* gw2, int B, int HW, int C,
                       int Cr, void* ws, long long ws_bytes, hyres_stream_t s, const float* pre = nullptr,
                       const float* slope = nullptr, float* dslope = nullptr) {
    HY_REQUIRE(x && gy && w1 && w2 && pooled && hidden && sgate && gx && gw1 && gw2, HYRES_E_ARG, "se_bwd: NULL");
    const int nch = se_chunks(HW);
    const long long need = (long long)B * nch * C * 4 + (long long)B * C * 4 + (pre ? SE_PRELU_PARTS * 4 : 0);
    HY_REQUIRE(ws && ws_bytes >= need, HYRES_E_WORKSPACE, "se_bwd: workspace");
    HY_REQUIRE((long long)B * (C + Cr) * 4 <= 60000, HYRES_E_SHAPE, "se_bwd: batch too large for LDS");
    const int per = (HW + nch - 1) / nch;
    float* part = (float*)ws;
    float* gpool = part + (long long)B * nch * C;
    hipStream_t st = as_stream(s);
    if (C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0 && aligned16(x) && aligned16(gy))
        hipLaunchKernelGGL((se_pool4_kernel<true, H, G>), dim3(B, nch), dim3(256), 0, st, x, gy, HW, C, per, part);
    else
        hipLaunchKernelGGL((se_bwd_pool_kernel<H, G>), dim3(B, nch), dim3(256), 0, st, x, gy, HW, C, per, part);
    int rc = HY_LAUNCH_CHECK("se_bwd_pool");
    if (rc) return rc;
    hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(1), dim3(256), (size_t)B * (C + Cr) * 4, st, (const float*)part, nch, B,
                       w1, w2, pooled, hidden, sgate, gpool, gw1, gw2, HW, C, Cr);
    rc = HY_LAUNCH_CHECK("se_fc_bwd");
    if (rc) return rc;
    long long n = (long long)B * HW * C;
    const unsigned am = G ? 7u : 15u;
    if (pre) {  // the PReLU-folded form (alignment checked by the entry points)
        float* pp = gpool + (long long)B * C;
        const int nb = std::min(pw_grid(n / 4), SE_PRELU_PARTS);
        hipLaunchKernelGGL((se_bwd_x4_prelu_kernel<H, G>), dim3(nb), dim3(256), 0, st, gy, sgate, (const float*)gpool, gx,
                           B, HW, C, pre, slope, pp);
        rc = HY_LAUNCH_CHECK("se_bwd_x4_prelu");
        if (rc) return rc;
        hipLaunchKernelGGL(se_prelu_slope_sum_kernel, dim3(1), dim3(256), 0, st, (const float*)pp, nb, dslope);
        return HY_LAUNCH_CHECK("se_prelu_slope_sum");
    }
    if (C % 4 == 0 && (reinterpret_cast<uintptr_t>(gy) & am) == 0 && (reinterpret_cast<uintptr_t>(gx) & am) == 0 &&
        n / 4 < (1LL << 31))
        hipLaunchKernelGGL(se_bwd_x4_kernel<G>, dim3(pw_grid(n / 4)), dim3(256), 0, st, gy, sgate, (const float*)gpool,
                           gx, B, HW, C);
    else
        hipLaunchKernelGGL(se_bwd_x_kernel<G>, dim3(grid_for_r(n)), dim3(256), 0, st, gy, sgate, (const float*)gpool, gx,
                           B, HW, C);
    return HY_LAUNCH_CHECK("se_bwd_x");
}
}  // extern "C++"
int hyres_se_bwd(const float* x, const float* gy, const float* w1, const float* w2, const float* pooled,
                 const float* hidden, const float* sgate, float* gx, float* gw1, float* gw2, int B, int HW, int C,
                 int Cr, void* ws, long long ws_bytes, hyres_stream_t s) {
    return se_bwd_impl<false, false>(x, gy, w1, w2, pooled, hidden, sgate, gx, gw1, gw2, B, HW, C, Cr, ws, ws_bytes, s);
}
int hyres_se_bwd_prelu(const float* x, const float* gy, const float* w1, const float* w2, const float* pooled,
                       const float* hidden, const float* sgate, float* gx, float* gw1, float* gw2, int B, int HW, int C,
                       int Cr, const float* pre, const float* slope, float* dslope, void* ws, long long ws_bytes,
                       hyres_stream_t s) {
    HY_REQUIRE(pre && slope && dslope && C % 4 == 0 && aligned16(gy) && aligned16(gx) && aligned16(pre) &&
                   (long long)B * HW * C / 4 < (1LL << 31),
               HYRES_E_ARG, "se_bwd_prelu: needs pre / slope / dslope, C %% 4 == 0, 16B-aligned gy / gx / pre");
    return se_bwd_impl<false, false>(x, gy, w1, w2, pooled, hidden, sgate, gx, gw1, gw2, B, HW, C, Cr, ws, ws_bytes, s,
                                     pre, slope, dslope);
}
int hyres_se_bwd_prelu_f16(const void* x, const void* gy, const float* w1, const float* w2, const float* pooled,
                           const float* hidden, const float* sgate, void* gx, float* gw1, float* gw2, int B, int HW, int C,
                           int Cr, const void* pre, const float* slope, float* dslope, void* ws, long long ws_bytes,
                           int g16, hyres_stream_t s) {
    const unsigned ag = g16 ? 7u : 15u;
    HY_REQUIRE(pre && slope && dslope && C % 4 == 0 && (reinterpret_cast<uintptr_t>(gy) & ag) == 0 &&
                   (reinterpret_cast<uintptr_t>(gx) & ag) == 0 && (reinterpret_cast<uintptr_t>(pre) & 7u) == 0 &&
                   (long long)B * HW * C / 4 < (1LL << 31),
               HYRES_E_ARG, "se_bwd_prelu_f16: needs pre / slope / dslope, C %% 4 == 0, aligned gy / gx / pre");
    if (g16)
        return se_bwd_impl<true, true>((const float*)x, (const float*)gy, w1, w2, pooled, hidden, sgate, (float*)gx, gw1,
                                       gw2, B, HW, C, Cr, ws, ws_bytes, s, (const float*)pre, slope, dslope);
    return se_bwd_impl<true, false>((const float*)x, (const float*)gy, w1, w2, pooled, hidden, sgate, (float*)gx, gw1,
                                    gw2, B, HW, C, Cr, ws, ws_bytes, s, (const float*)pre, slope, dslope);
}
int hyres_se_bwd_f16(const void* x, const void* gy, const float* w1, const float* w2, const float* pooled,
                     const float* hidden, const float* sgate, void* gx, float* gw1, float* gw2, int B, int HW, int C,
                     int Cr, void* ws, long long ws_bytes, int g16, hyres_stream_t s) {
    if (g16)
        return se_bwd_impl<true, true>((const float*)x, (const float*)gy, w1, w2, pooled, hidden, sgate, (float*)gx, gw1,
                                       gw2, B, HW, C, Cr, ws, ws_bytes, s);
    return se_bwd_impl<true, false>((const float*)x, (const float*)gy, w1, w2, pooled, hidden, sgate, (float*)gx, gw1,
                                    gw2, B, HW, C, Cr, ws, ws_bytes, s);
}

static int sa_bwd_blocks(long long n) {  // >= 4 pixels per thread: the 98-tap weight fold is amortised
    return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 1024));
}

static long long sa_tiles(int B, int H, int W) {
    return (long long)B * ((H + SA_T - 1) / SA_T) * ((W + SA_T - 1) / SA_T);
}

long long hyres_spatial_attn_workspace_bytes(int B, int H, int W) {
    long long n = (long long)B * H * W;
    const long long nb = std::max<long long>(sa_bwd_blocks(n), sa_tiles(B, H, W));
    return nb * 98 * 4 + n * 4 + n * 2 * 4 + 1024;
}

int hyres_spatial_attn_fwd(const float* x, const float* w, float* pooled2, int* argmax, float* attn, float* y, int B,
                           int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(x && w && pooled2 && argmax && attn, HYRES_E_ARG, "spatial_attn_fwd: NULL");  // y NULL: map only
    HY_REQUIRE(C % 4 == 0 && C <= 1024 && aligned16(x) && (!y || aligned16(y)), HYRES_E_ALIGN,
               "spatial_attn: C %% 4 == 0 and 16B-aligned x/y required");
    long long P = (long long)B * H * W;
    hipStream_t st = as_stream(s);
    HY_REQUIRE(C % 4 == 0 && aligned16(x), HYRES_E_ALIGN, "spatial_attn_fwd: C %% 4 and 16B-aligned x needed");
    if (C == 192)
        hipLaunchKernelGGL((sa_pool_kernel<false, 3>), dim3((unsigned)((P + 15) / 16)), dim3(256), 0, st, x, pooled2, argmax,
                           P, C);
    else
        hipLaunchKernelGGL(sa_pool_kernel<false>, dim3((unsigned)((P + 15) / 16)), dim3(256), 0, st, x, pooled2, argmax, P,
                           C);
    int rc = HY_LAUNCH_CHECK("sa_pool");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_conv_tiled_kernel, dim3((unsigned)sa_tiles(B, H, W)), dim3(256), 0, st, (const float*)pooled2,
                       w, attn, B, H, W);
    rc = HY_LAUNCH_CHECK("sa_conv");
    if (rc) return rc;
    if (!y) return ok();  // the attention map only (the multiply folded into the consumer: HYRES_EPI_ROWSCALE)
    hipLaunchKernelGGL(sa_mul_kernel<false>, dim3(grid_for_r(P * C / 4)), dim3(256), 0, st, x, (const float*)attn, y, P, C);
    return HY_LAUNCH_CHECK("sa_mul");
}

int hyres_spatial_attn_fwd_f16(const void* x, const float* w, float* pooled2, int* argmax, float* attn, void* y, int B,
                               int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(x && w && pooled2 && argmax && attn, HYRES_E_ARG, "spatial_attn_fwd_f16: NULL");  // y NULL: map only
    HY_REQUIRE(C % 4 == 0 && C <= 1024 && (reinterpret_cast<uintptr_t>(x) & 7) == 0 &&
                   (reinterpret_cast<uintptr_t>(y) & 7) == 0,
               HYRES_E_ALIGN, "spatial_attn_fwd_f16: C %% 4 == 0 and 8B-aligned x/y required");
    const long long P = (long long)B * H * W;
    hipStream_t st = as_stream(s);
    if (C == 192)
        hipLaunchKernelGGL((sa_pool_kernel<true, 3>), dim3((unsigned)((P + 15) / 16)), dim3(256), 0, st, (const float*)x,
                           pooled2, argmax, P, C);
    else
        hipLaunchKernelGGL(sa_pool_kernel<true>, dim3((unsigned)((P + 15) / 16)), dim3(256), 0, st, (const float*)x,
                           pooled2, argmax, P, C);
    int rc = HY_LAUNCH_CHECK("sa_pool_f16");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_conv_tiled_kernel, dim3((unsigned)sa_tiles(B, H, W)), dim3(256), 0, st, (const float*)pooled2,
                       w, attn, B, H, W);
    rc = HY_LAUNCH_CHECK("sa_conv");
    if (rc) return rc;
    if (!y) return ok();  // the attention map only
    hipLaunchKernelGGL(sa_mul_kernel<true>, dim3(grid_for_r(P * C / 4)), dim3(256), 0, st, (const float*)x,
                       (const float*)attn, (float*)y, P, C);
    return HY_LAUNCH_CHECK("sa_mul_f16");
}

extern "C++" {
template <bool HF, bool G>
static int spatial_attn_bwd_impl(const float* x, const float* w, const float* pooled2, const int* argmax,
                                 const float* attn, const float* gy, float* gx, float* gw, int B, int H, int W, int C,
                                 void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(x && w && pooled2 && argmax && attn && gy && gx && gw, HYRES_E_ARG, "spatial_attn_bwd: NULL");
    const unsigned am = G ? 7u : 15u;
    HY_REQUIRE(C % 4 == 0 && C <= 1024 && (reinterpret_cast<uintptr_t>(x) & 7) == 0 &&
                   (reinterpret_cast<uintptr_t>(gy) & am) == 0 && (reinterpret_cast<uintptr_t>(gx) & am) == 0,
               HYRES_E_ALIGN, "spatial_attn: C %% 4 == 0 and aligned x/gy/gx required");
    long long P = (long long)B * H * W;
    HY_REQUIRE(ws && ws_bytes >= hyres_spatial_attn_workspace_bytes(B, H, W), HYRES_E_WORKSPACE,
               "spatial_attn_bwd: workspace");
    float* glogit = (float*)ws;
    float* gp2 = glogit + P;
    float* wpart = gp2 + 2 * P;
    hipStream_t st = as_stream(s);
    hipLaunchKernelGGL((sa_bwd_logit_kernel<HF, G>), dim3((unsigned)((P + 15) / 16)), dim3(256), 0, st, x, gy, attn,
                       glogit, P, C);
    int rc = HY_LAUNCH_CHECK("sa_bwd_logit");
    if (rc) return rc;
    const int nb = (int)sa_tiles(B, H, W);
    hipLaunchKernelGGL(sa_bwd_conv_tiled_kernel, dim3(nb), dim3(256), 0, st, (const float*)glogit, pooled2, w, gp2,
                       wpart, B, H, W, 0);
    rc = HY_LAUNCH_CHECK("sa_bwd_conv");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_bwd_wfinal_kernel, dim3(98), dim3(256), 0, st, (const float*)wpart, nb, gw);
    rc = HY_LAUNCH_CHECK("sa_bwd_wfinal");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_bwd_x_kernel<G>, dim3(grid_for_r(P * C / 4)), dim3(256), 0, st, gy, attn, (const float*)gp2,
                       argmax, gx, P, C);
    return HY_LAUNCH_CHECK("sa_bwd_x");
}
}  // extern "C++"
static int sa_fold_blocks(long long P) { return (int)std::max<long long>(1, std::min<long long>((P + 63) / 64, 1024)); }

long long hyres_sa_fold_workspace_bytes(long long P, int C) { return (long long)sa_fold_blocks(P) * (C + 1) * 4 + 256; }

int hyres_sa_fold_bwd(const float* pre, int ldpre, const float* gy, int ldg, const float* attn, const float* bias,
                      const float* slope, float* gs, float* glogit, float* dbias, float* dslope, long long P, int C,
                      void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(pre && gy && attn && bias && slope && gs && glogit && dbias && dslope && P > 0, HYRES_E_ARG,
               "sa_fold_bwd: NULL");
    HY_REQUIRE(C % 4 == 0 && C > 0 && C <= 64 && ldpre % 4 == 0 && ldg % 4 == 0 && aligned16(pre) && aligned16(gy) &&
                   aligned16(gs) && aligned16(bias),
               HYRES_E_ALIGN, "sa_fold_bwd: C %% 4 == 0, C <= 64, 16B-aligned rows");
    HY_REQUIRE(ws && ws_bytes >= hyres_sa_fold_workspace_bytes(P, C), HYRES_E_WORKSPACE, "sa_fold_bwd: workspace");
    const int nb = sa_fold_blocks(P);
    hipStream_t st = as_stream(s);
    hipLaunchKernelGGL(sa_fold_bwd_kernel, dim3(nb), dim3(256), 0, st, pre, ldpre, gy, ldg, attn, bias, slope, gs, glogit,
                       (float*)ws, P, C);
    int rc = HY_LAUNCH_CHECK("sa_fold_bwd");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_fold_final_kernel, dim3(C + 1), dim3(256), 0, st, (const float*)ws, nb, C, dbias, dslope);
    return HY_LAUNCH_CHECK("sa_fold_final");
}

int hyres_sa_fold_bwd_f16(const void* pre, int ldpre, const void* gy, int ldg, const float* attn, const float* bias,
                          const float* slope, void* gs, float* glogit, float* dbias, float* dslope, long long P, int C,
                          void* ws, long long ws_bytes, int g16, hyres_stream_t s) {
    HY_REQUIRE(pre && gy && attn && bias && slope && gs && glogit && dbias && dslope && P > 0, HYRES_E_ARG,
               "sa_fold_bwd_f16: NULL");
    HY_REQUIRE(C % 8 == 0 && C > 0 && C <= 64 && ldpre % 8 == 0 && ldg % 8 == 0 && aligned16(pre) && aligned16(gy) &&
                   aligned16(gs),
               HYRES_E_ALIGN, "sa_fold_bwd_f16: C %% 8 == 0, C <= 64, 16B-aligned rows");
    HY_REQUIRE(ws && ws_bytes >= hyres_sa_fold_workspace_bytes(P, C), HYRES_E_WORKSPACE, "sa_fold_bwd_f16: workspace");
    const int nb = sa_fold_blocks(P);
    hipStream_t st = as_stream(s);
    if (g16)
        hipLaunchKernelGGL(sa_fold_bwd_h8_kernel<true>, dim3(nb), dim3(256), 0, st, (const float*)pre, ldpre,
                           (const float*)gy, ldg, attn, bias, slope, (float*)gs, glogit, (float*)ws, P, C);
    else
        hipLaunchKernelGGL(sa_fold_bwd_h8_kernel<false>, dim3(nb), dim3(256), 0, st, (const float*)pre, ldpre,
                           (const float*)gy, ldg, attn, bias, slope, (float*)gs, glogit, (float*)ws, P, C);
    int rc = HY_LAUNCH_CHECK("sa_fold_bwd_f16");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_fold_final_kernel, dim3(C + 1), dim3(256), 0, st, (const float*)ws, nb, C, dbias, dslope);
    return HY_LAUNCH_CHECK("sa_fold_final");
}

int hyres_spatial_attn_bwd_map(const float* glogit, const float* pooled2, const float* w, float* gpooled2, float* gw,
                               int B, int H, int W, int C, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(glogit && pooled2 && w && gpooled2 && gw && C > 0, HYRES_E_ARG, "spatial_attn_bwd_map: NULL");
    HY_REQUIRE(ws && ws_bytes >= hyres_spatial_attn_workspace_bytes(B, H, W), HYRES_E_WORKSPACE,
               "spatial_attn_bwd_map: workspace");
    const long long P = (long long)B * H * W;
    float* wpart = (float*)ws;
    const int nb = (int)sa_tiles(B, H, W);
    (void)P;
    hipStream_t st = as_stream(s);
    hipLaunchKernelGGL(sa_bwd_conv_tiled_kernel, dim3(nb), dim3(256), 0, st, glogit, pooled2, w, gpooled2, wpart, B, H,
                       W, C);
    int rc = HY_LAUNCH_CHECK("sa_bwd_conv");
    if (rc) return rc;
    hipLaunchKernelGGL(sa_bwd_wfinal_kernel, dim3(98), dim3(256), 0, st, (const float*)wpart, nb, gw);
    return HY_LAUNCH_CHECK("sa_bwd_wfinal");
}

int hyres_spatial_attn_bwd(const float* x, const float* w, const float* pooled2, const int* argmax, const float* attn,
                           const float* gy, float* gx, float* gw, int B, int H, int W, int C, void* ws,
                           long long ws_bytes, hyres_stream_t s) {
    return spatial_attn_bwd_impl<false, false>(x, w, pooled2, argmax, attn, gy, gx, gw, B, H, W, C, ws, ws_bytes, s);
}
int hyres_spatial_attn_bwd_f16(const void* x, const float* w, const float* pooled2, const int* argmax,
                               const float* attn, const void* gy, void* gx, float* gw, int B, int H, int W, int C,
                               void* ws, long long ws_bytes, int g16, hyres_stream_t s) {
    if (g16)
        return spatial_attn_bwd_impl<true, true>((const float*)x, w, pooled2, argmax, attn, (const float*)gy, (float*)gx,
                                                 gw, B, H, W, C, ws, ws_bytes, s);
    return spatial_attn_bwd_impl<true, false>((const float*)x, w, pooled2, argmax, attn, (const float*)gy, (float*)gx, gw,
                                              B, H, W, C, ws, ws_bytes, s);
}

}  // extern "C"
