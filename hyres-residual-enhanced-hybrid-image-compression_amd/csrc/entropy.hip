// Quantisation, checkerboard two-pass context split/merge, GaussianConditional and
// EntropyBottleneck likelihoods (forward + backward) for the HyRES hot path on gfx950.
//
// Reference semantics (paths relative to the reference repo):
//   * anchor set = {(h,w) : (h+w) even}  — models/checkerboard.py:106-112 (bit-exact index parity)
//   * Quantizer "ste": round(t) - t + t, op order kept — models/utils/quantization.py:11-12
//   * GaussianConditional (compressai 1.2.6): v = |y_q - mu|, s = max(scales, 0.11),
//     lik = max(Phi((.5-v)/s) - Phi((-.5-v)/s), 1e-9), Phi(x) = .5 erfc(-x/sqrt2)
//   * EntropyBottleneck: per-channel MLP 1-3-3-3-3-1 with softplus weights and tanh gates,
//     lik = max(sigmoid(L(v+.5)) - sigmoid(L(v-.5)), 1e-9)
// Layout: all activations NHWC; y/scales/means are [B,H,W,C] with C = M (192).
#include "common.h"

namespace hyres {

#define GRID_STRIDE(i, n) \
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

static inline int grid_for_e(long long n) {
    long long b = (n + 255) / 256;
    return (int)std::max<long long>(1, std::min<long long>(b, 8192));
}

__device__ __forceinline__ float ste_round(float t) {
    // torch.round(t) - t.detach() + t  (half-to-even; evaluated left to right in fp32)
    float r = rintf(t);
    float d = r - t;
    return d + t;
}
__device__ __forceinline__ bool is_anchor(long long pix, int H, int W) {
    int w = (int)(pix % W);
    int h = (int)((pix / W) % H);
    return ((h + w) & 1) == 0;
}

__global__ void quantize_kernel(const float* x, int mode, float* y, long long n) {
    GRID_STRIDE(i, n) y[i] = mode == 0 ? ste_round(x[i]) : rintf(x[i]);
}

__global__ void ckbd_anchor_fwd_kernel(const float* y, const float* means_a, int ldm, const float* noise,
                                       float* out, int B, int H, int W, int C) {
    const long long n = (long long)B * H * W * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        float ya = is_anchor(p, H, W) ? y[i] : 0.f;
        float v;
        if (noise) {
            v = ya + noise[i];
        } else {
            float m = means_a[p * ldm + c];
            v = ste_round(ya - m) + m;
        }
        out[i] = v;
    }
}

__device__ __forceinline__ float std_cum(float x) {
    // compressai _standardized_cumulative: 0.5 * erfc(-(2^-0.5) * x)
    return 0.5f * erfcf(-0.70710678118654752f * x);
}
__device__ __forceinline__ float std_pdf(float x) { return 0.39894228040143268f * expf(-0.5f * x * x); }

__global__ void ckbd_nonanchor_gc_fwd_kernel(const float* y, const float* ya_hat, const float* pa, int lda,
                                             const float* pn, int ldn, const float* noise_q, const float* noise_gc,
                                             float* y_hat, float* scales, float* means, float* y_q, float* lik,
                                             int B, int H, int W, int C) {
    const long long n = (long long)B * H * W * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        const float yv = y[i];
        const float sa = pa[p * lda + c], ma = pa[p * lda + C + c];
        const float sn = pn[p * ldn + c], mn = pn[p * ldn + C + c];
        const float yna = is_anchor(p, H, W) ? 0.f : yv;
        float yna_hat = noise_q ? (yna + noise_q[i]) : (ste_round(yna - mn) + mn);
        y_hat[i] = ya_hat[i] + yna_hat;
        const float sc = sa + sn;
        const float mu = ma + mn;
        scales[i] = sc;
        means[i] = mu;
        float q;
        if (noise_gc) q = yv + noise_gc[i];
        else q = rintf(yv - mu) + mu;
        y_q[i] = q;
        const float v = fabsf(q - mu);
        const float s = fmaxf(sc, 0.11f);
        const float up = std_cum((0.5f - v) / s);
        const float lo = std_cum((-0.5f - v) / s);
        lik[i] = fmaxf(up - lo, 1e-9f);
    }
}

// Backward of the non-anchor quantiser + combine + GaussianConditional.
//   g_y            = g_yhat (+ GC term when training)             (all positions; anchor positions
//                    also get the ctx-path gradient later via ckbd_anchor_bwd)
//   g_params[...]  = [g_scales | g_means] written to both param-aggregation gradient buffers
__global__ void ckbd_gc_bwd_kernel(const float* y_q, const float* scales, const float* means, const float* g_lik,
                                   const float* g_yhat, int training, float* g_y, float* gpa, int lda, float* gpn,
                                   int ldn, int B, int H, int W, int C) {
    const long long n = (long long)B * H * W * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        int c = (int)(i - p * C);
        const float mu = means[i];
        const float sc = scales[i];
        const float d = y_q[i] - mu;
        const float v = fabsf(d);
        const float s = fmaxf(sc, 0.11f);
        const float a_up = (0.5f - v) / s, a_lo = (-0.5f - v) / s;
        const float raw = std_cum(a_up) - std_cum(a_lo);
        float gl = g_lik ? g_lik[i] : 0.f;
        // likelihood LowerBound(1e-9)
        if (!(raw >= 1e-9f || gl < 0.f)) gl = 0.f;
        const float pu = std_pdf(a_up), pl = std_pdf(a_lo);
        const float dv = gl * (pl - pu) / s;               // d lik / d v
        float ds = gl * (-a_up * pu + a_lo * pl) / s;      // d lik / d s'
        if (!(sc >= 0.11f || ds < 0.f)) ds = 0.f;          // scale LowerBound(0.11)
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        const float gd = dv * sgn;                          // d / d (y_q - mu)
        // training: y_q = y + noise  -> d/dy = gd, d/dmu = -gd ; eval: y_q - mu = round(y-mu): no grad
        const float gy_gc = training ? gd : 0.f;
        const float gmu = training ? -gd : 0.f;
        g_y[i] = g_yhat[i] + gy_gc;
        gpa[p * lda + c] = ds;
        gpa[p * lda + C + c] = gmu;
        gpn[p * ldn + c] = ds;
        gpn[p * ldn + C + c] = gmu;
    }
}

__global__ void ckbd_anchor_bwd_kernel(const float* g_ya, float* g_y, int B, int H, int W, int C) {
    const long long n = (long long)B * H * W * C;
    GRID_STRIDE(i, n) {
        long long p = i / C;
        if (is_anchor(p, H, W)) g_y[i] += g_ya[i];
    }
}

// ---------------------------------------------------------------- EntropyBottleneck
// packed per-channel record (HYRES_EB_REC floats):
constexpr int EB_M0 = 0, EB_B0 = 3, EB_F0 = 6;    // softplus(M0)[3x1], b0[3], tanh(f0)[3]
constexpr int EB_M1 = 9, EB_B1 = 18, EB_F1 = 21;  // [3x3], [3], [3]
constexpr int EB_M2 = 24, EB_B2 = 33, EB_F2 = 36;
constexpr int EB_M3 = 39, EB_B3 = 48, EB_F3 = 51;
constexpr int EB_M4 = 54, EB_B4 = 57;             // [1x3], [1]
constexpr int EB_MED = 58;
constexpr int EB_NP = 59;

struct EbFwdState {
    float h[4][3];  // pre-gate activations of layers 0..3
    float a[4][3];  // post-gate activations
};

__device__ __forceinline__ float eb_logits(const float* r, float v, EbFwdState& st) {
    // layer 0: 1 -> 3
    float in[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float h = r[EB_M0 + j] * v + r[EB_B0 + j];
        st.h[0][j] = h;
        float a = h + r[EB_F0 + j] * tanhf(h);
        st.a[0][j] = a;
        in[j] = a;
    }
#pragma unroll
    for (int L = 1; L < 4; ++L) {
        const int mo = EB_M1 + (L - 1) * 15, bo = mo + 9, fo = mo + 12;
        float out[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            // torch.matmul(softplus(M), logits): sum_k M[j][k] * in[k]
            float h = r[mo + 3 * j + 0] * in[0] + r[mo + 3 * j + 1] * in[1] + r[mo + 3 * j + 2] * in[2];
            h = h + r[bo + j];
            st.h[L][j] = h;
            float a = h + r[fo + j] * tanhf(h);
            st.a[L][j] = a;
            out[j] = a;
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) in[j] = out[j];
    }
    float o = r[EB_M4 + 0] * in[0] + r[EB_M4 + 1] * in[1] + r[EB_M4 + 2] * in[2];
    return o + r[EB_B4];
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void eb_fwd_kernel(const float* z, const float* packed, const float* noise, int training, float* z_q,
                              float* lik, float* z_hat_ste, long long P, int C) {
    const long long n = P * C;
    GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        const float* r = packed + (long long)c * HYRES_EB_REC;
        const float zv = z[i];
        const float med = r[EB_MED];
        float v = training ? (zv + noise[i]) : (rintf(zv - med) + med);
        z_q[i] = v;
        EbFwdState st;
        float lo = eb_logits(r, v - 0.5f, st);
        float up = eb_logits(r, v + 0.5f, st);
        lik[i] = fmaxf(sigm(up) - sigm(lo), 1e-9f);
        if (z_hat_ste) z_hat_ste[i] = ste_round(zv - med) + med;
    }
}

// backprop d(logit)/d(params, v) scaled by gout, accumulating param grads into gp[EB_NP]
__device__ __forceinline__ float eb_logits_bwd(const float* r, float v, float gout, float* gp) {
    EbFwdState st;
    (void)eb_logits(r, v, st);
    // output layer
    gp[EB_B4] += gout;
    float ga[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        gp[EB_M4 + k] += gout * st.a[3][k];
        ga[k] = gout * r[EB_M4 + k];
    }
#pragma unroll
    for (int L = 3; L >= 1; --L) {
        const int mo = EB_M1 + (L - 1) * 15, bo = mo + 9, fo = mo + 12;
        float gh[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float th = tanhf(st.h[L][j]);
            gp[fo + j] += ga[j] * th;
            gh[j] = ga[j] * (1.0f + r[fo + j] * (1.0f - th * th));
            gp[bo + j] += gh[j];
        }
        float gin[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                gp[mo + 3 * j + k] += gh[j] * st.a[L - 1][k];
                gin[k] += gh[j] * r[mo + 3 * j + k];
            }
#pragma unroll
        for (int k = 0; k < 3; ++k) ga[k] = gin[k];
    }
    float gv = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float th = tanhf(st.h[0][j]);
        gp[EB_F0 + j] += ga[j] * th;
        float gh = ga[j] * (1.0f + r[EB_F0 + j] * (1.0f - th * th));
        gp[EB_B0 + j] += gh;
        gp[EB_M0 + j] += gh * v;
        gv += gh * r[EB_M0 + j];
    }
    return gv;
}

// grid (C, nb): block handles channel c, elements [b*per, (b+1)*per) of the P pixels
__global__ __launch_bounds__(256) void eb_bwd_kernel(const float* z_q, const float* packed, const float* lik,
                                                     const float* g_lik, const float* g_zhat, int training,
                                                     int noisequant, float* g_z, float* gws, long long P, int C,
                                                     int per) {
    const int c = blockIdx.x;
    const float* r = packed + (long long)c * HYRES_EB_REC;
    __shared__ float rs[HYRES_EB_REC];
    if (threadIdx.x < HYRES_EB_REC) rs[threadIdx.x] = r[threadIdx.x];
    __syncthreads();
    float gp[EB_NP];
#pragma unroll
    for (int k = 0; k < EB_NP; ++k) gp[k] = 0.f;
    const long long p0 = (long long)blockIdx.y * per;
    const long long p1 = min((long long)P, p0 + per);
    for (long long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const long long i = p * C + c;
        const float v = z_q[i];
        float gl = g_lik ? g_lik[i] : 0.f;
        EbFwdState st;
        const float lo = eb_logits(rs, v - 0.5f, st);
        const float up = eb_logits(rs, v + 0.5f, st);
        const float su = sigm(up), sl = sigm(lo);
        const float raw = su - sl;
        if (!(raw >= 1e-9f || gl < 0.f)) gl = 0.f;
        float gv = 0.f;
        if (gl != 0.f) {
            gv += eb_logits_bwd(rs, v + 0.5f, gl * su * (1.0f - su), gp);
            gv += eb_logits_bwd(rs, v - 0.5f, -gl * sl * (1.0f - sl), gp);
        }
        // v = z + noise (train) -> dz = gv ; v = round(z-med)+med (eval) -> dmed = gv
        float gz = training ? gv : 0.f;
        if (!training) gp[EB_MED] += gv;
        // z_hat path: STE (noisequant=False): dz = g ; noisequant: z_hat = v -> train dz = g, eval dmed = g
        const float gzh = g_zhat ? g_zhat[i] : 0.f;
        if (!noisequant || training) gz += gzh;
        else gp[EB_MED] += gzh;
        g_z[i] = gz;
    }
    // block reduction of gp[0..EB_NP)
    __shared__ float red[256];
    float* out = gws + ((long long)blockIdx.y * C + c) * HYRES_EB_REC;
    for (int k = 0; k < EB_NP; ++k) {
        red[threadIdx.x] = gp[k];
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[k] = red[0];
        __syncthreads();
    }
}

struct EbPtrs {
    const float* m[5];
    const float* b[5];
    const float* f[4];
    float* gm[5];
    float* gb[5];
    float* gf[4];
};

__device__ __forceinline__ float softplus_t(float x) {
    // torch F.softplus(beta=1, threshold=20)
    return x > 20.f ? x : log1pf(expf(x));
}

__global__ void eb_pack_kernel(const EbPtrs ptr, const float* quantiles, float* packed, int C) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float* r = packed + (long long)c * HYRES_EB_REC;
    const int fin[5] = {1, 3, 3, 3, 3}, fout[5] = {3, 3, 3, 3, 1};
    const int mo[5] = {EB_M0, EB_M1, EB_M2, EB_M3, EB_M4};
    const int bo[5] = {EB_B0, EB_B1, EB_B2, EB_B3, EB_B4};
    const int fo[4] = {EB_F0, EB_F1, EB_F2, EB_F3};
    for (int L = 0; L < 5; ++L) {
        const int nm = fin[L] * fout[L];
        for (int k = 0; k < nm; ++k) r[mo[L] + k] = softplus_t(ptr.m[L][(long long)c * nm + k]);
        for (int k = 0; k < fout[L]; ++k) r[bo[L] + k] = ptr.b[L][(long long)c * fout[L] + k];
        if (L < 4)
            for (int k = 0; k < 3; ++k) r[fo[L] + k] = tanhf(ptr.f[L][(long long)c * 3 + k]);
    }
    r[EB_MED] = quantiles[(long long)c * 3 + 1];
    for (int k = EB_NP; k < HYRES_EB_REC; ++k) r[k] = 0.f;
}

__global__ void eb_unpack_grad_kernel(const float* gws, int nb, const EbPtrs ptr, float* g_quant, int C, int acc) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float g[EB_NP];
    for (int k = 0; k < EB_NP; ++k) {
        float s = 0.f;
        for (int b = 0; b < nb; ++b) s += gws[((long long)b * C + c) * HYRES_EB_REC + k];
        g[k] = s;
    }
    const int fin[5] = {1, 3, 3, 3, 3}, fout[5] = {3, 3, 3, 3, 1};
    const int mo[5] = {EB_M0, EB_M1, EB_M2, EB_M3, EB_M4};
    const int bo[5] = {EB_B0, EB_B1, EB_B2, EB_B3, EB_B4};
    const int fo[4] = {EB_F0, EB_F1, EB_F2, EB_F3};
    for (int L = 0; L < 5; ++L) {
        const int nm = fin[L] * fout[L];
        for (int k = 0; k < nm; ++k) {
            long long idx = (long long)c * nm + k;
            float x = ptr.m[L][idx];
            // d softplus / dx (threshold 20): sigmoid(x) or 1
            float d = x > 20.f ? 1.f : 1.0f / (1.0f + expf(-x));
            float v = g[mo[L] + k] * d;
            ptr.gm[L][idx] = acc ? ptr.gm[L][idx] + v : v;
        }
        for (int k = 0; k < fout[L]; ++k) {
            long long idx = (long long)c * fout[L] + k;
            float v = g[bo[L] + k];
            ptr.gb[L][idx] = acc ? ptr.gb[L][idx] + v : v;
        }
        if (L < 4)
            for (int k = 0; k < 3; ++k) {
                long long idx = (long long)c * 3 + k;
                float t = tanhf(ptr.f[L][idx]);
                float v = g[fo[L] + k] * (1.0f - t * t);
                ptr.gf[L][idx] = acc ? ptr.gf[L][idx] + v : v;
            }
    }
    if (g_quant) {
        float v = g[EB_MED];
        long long idx = (long long)c * 3 + 1;
        g_quant[idx] = acc ? g_quant[idx] + v : v;
    }
}

// aux loss: sum_c sum_k |L_c(q[c][k]) - target[k]| with the MLP detached; gradient wrt quantiles only
__global__ void eb_aux_kernel(const float* packed, const float* quantiles, const float* target, float* loss,
                              float* g_q, int C) {
    __shared__ float red[1024];
    float s = 0.f;
    for (int idx = threadIdx.x; idx < C * 3; idx += blockDim.x) {
        const int c = idx / 3, k = idx % 3;
        const float* r = packed + (long long)c * HYRES_EB_REC;
        const float q = quantiles[idx];
        EbFwdState st;
        const float l = eb_logits(r, q, st);
        const float d = l - target[k];
        s += fabsf(d);
        if (g_q) {
            float gp[EB_NP];
#pragma unroll
            for (int j = 0; j < EB_NP; ++j) gp[j] = 0.f;
            const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            g_q[idx] = eb_logits_bwd(r, q, sg, gp);
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = blockDim.x / 2; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = red[0];
}

}  // namespace hyres

namespace hyres {

// ---------------------------------------------------------------- entropy-coding symbolisation
// (compress/decompress). Symbols and CDF indexes are produced in NCHW order per image —
// compressai's per-image string order (symbols[i].reshape(-1)) — from the NHWC activations.
__device__ __forceinline__ bool ckbd_keep(int parity, int h, int w) {
    return parity < 0 || (((h + w) & 1) == parity);
}

// GaussianConditional: sym = round(y*keep - mean) (compressai quantize "symbols"), idx = build_indexes(
// max(scale, 0.11)) = (nt-1) - #{k < nt-1 : scale <= table[k]}.  y == NULL: indexes only.
__global__ void gc_symbols_kernel(const float* y, int ldy, const float* params, int ldp, int M, int B, int H, int W,
                                  int parity, const float* table, int nt, int* sym, int* idx) {
    const long long n = (long long)B * M * H * W;
    GRID_STRIDE(i, n) {
        const int w = (int)(i % W);
        const long long r = i / W;
        const int h = (int)(r % H);
        const long long r2 = r / H;
        const int c = (int)(r2 % M);
        const int b = (int)(r2 / M);
        const long long pix = ((long long)b * H + h) * W + w;
        const float scale = fmaxf(params[pix * ldp + c], 0.11f);
        int k = nt - 1;
        for (int t = 0; t < nt - 1; ++t) k -= (scale <= table[t]) ? 1 : 0;
        idx[i] = k;
        if (y) {
            const float mean = params[pix * ldp + M + c];
            const float yv = ckbd_keep(parity, h, w) ? y[pix * ldy + c] : 0.f;
            sym[i] = (int)rintf(yv - mean);
        }
    }
}

// y_hat (+)= sym + mean (compressai dequantize), NHWC out
__global__ void gc_dequant_kernel(const int* sym, const float* params, int ldp, int M, int B, int H, int W,
                                  float* out, int ldo, int acc) {
    const long long n = (long long)B * M * H * W;
    GRID_STRIDE(i, n) {
        const int w = (int)(i % W);
        const long long r = i / W;
        const int h = (int)(r % H);
        const long long r2 = r / H;
        const int c = (int)(r2 % M);
        const int b = (int)(r2 / M);
        const long long pix = ((long long)b * H + h) * W + w;
        const float v = (float)sym[i] + params[pix * ldp + M + c];
        float* o = out + pix * ldo + c;
        *o = acc ? *o + v : v;
    }
}

// EntropyBottleneck: sym = round(z - median_c) (dequant: sym + median_c), NCHW symbols, NHWC tensors
__global__ void eb_symbols_kernel(const float* z, int ldz, const float* med, int B, int H, int W, int C, int* sym,
                                  float* zhat, int ldo, int dequant) {
    const long long n = (long long)B * C * H * W;
    GRID_STRIDE(i, n) {
        const int w = (int)(i % W);
        const long long r = i / W;
        const int h = (int)(r % H);
        const long long r2 = r / H;
        const int c = (int)(r2 % C);
        const int b = (int)(r2 / C);
        const long long pix = ((long long)b * H + h) * W + w;
        if (dequant) {
            zhat[pix * ldo + c] = (float)sym[i] + med[c];
        } else {
            sym[i] = (int)rintf(z[pix * ldz + c] - med[c]);
        }
    }
}

}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_quantize(const float* x, int mode, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(x && y && (mode == 0 || mode == 1), HYRES_E_ARG, "quantize: bad args");
    hipLaunchKernelGGL(quantize_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), x, mode, y, n);
    return HY_LAUNCH_CHECK("quantize");
}

int hyres_ckbd_anchor_fwd(const float* y, const float* means_a, int ldm, const float* noise, float* y_a_hat, int B,
                          int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(y && y_a_hat && (noise || means_a), HYRES_E_ARG, "ckbd_anchor_fwd: NULL");
    long long n = (long long)B * H * W * C;
    hipLaunchKernelGGL(ckbd_anchor_fwd_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), y, means_a, ldm,
                       noise, y_a_hat, B, H, W, C);
    return HY_LAUNCH_CHECK("ckbd_anchor_fwd");
}

int hyres_ckbd_nonanchor_gc_fwd(const float* y, const float* y_a_hat, const float* params_a, int lda,
                                const float* params_na, int ldn, const float* noise_q, const float* noise_gc,
                                float* y_hat, float* scales, float* means, float* y_q, float* lik, int B, int H,
                                int W, int C, hyres_stream_t s) {
    HY_REQUIRE(y && y_a_hat && params_a && params_na && y_hat && scales && means && y_q && lik, HYRES_E_ARG,
               "ckbd_nonanchor_gc_fwd: NULL");
    long long n = (long long)B * H * W * C;
    hipLaunchKernelGGL(ckbd_nonanchor_gc_fwd_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), y, y_a_hat,
                       params_a, lda, params_na, ldn, noise_q, noise_gc, y_hat, scales, means, y_q, lik, B, H, W, C);
    return HY_LAUNCH_CHECK("ckbd_nonanchor_gc_fwd");
}

int hyres_ckbd_gc_bwd(const float* y_q, const float* scales, const float* means, const float* g_lik,
                      const float* g_yhat, int training, float* g_y, float* g_params_a, int lda,
                      float* g_params_na, int ldn, int B, int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(y_q && scales && means && g_yhat && g_y && g_params_a && g_params_na, HYRES_E_ARG,
               "ckbd_gc_bwd: NULL");
    long long n = (long long)B * H * W * C;
    hipLaunchKernelGGL(ckbd_gc_bwd_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), y_q, scales, means,
                       g_lik, g_yhat, training, g_y, g_params_a, lda, g_params_na, ldn, B, H, W, C);
    return HY_LAUNCH_CHECK("ckbd_gc_bwd");
}

int hyres_ckbd_anchor_bwd(const float* g_ya_ctx, float* g_y, int B, int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(g_ya_ctx && g_y, HYRES_E_ARG, "ckbd_anchor_bwd: NULL");
    long long n = (long long)B * H * W * C;
    hipLaunchKernelGGL(ckbd_anchor_bwd_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), g_ya_ctx, g_y, B, H,
                       W, C);
    return HY_LAUNCH_CHECK("ckbd_anchor_bwd");
}

int hyres_eb_pack(const float* const* mats, const float* const* biases, const float* const* factors,
                  const float* quantiles, float* packed, int C, hyres_stream_t s) {
    HY_REQUIRE(mats && biases && factors && quantiles && packed, HYRES_E_ARG, "eb_pack: NULL");
    EbPtrs p{};
    for (int i = 0; i < 5; ++i) { p.m[i] = mats[i]; p.b[i] = biases[i]; }
    for (int i = 0; i < 4; ++i) p.f[i] = factors[i];
    hipLaunchKernelGGL(eb_pack_kernel, dim3((C + 127) / 128), dim3(128), 0, as_stream(s), p, quantiles, packed, C);
    return HY_LAUNCH_CHECK("eb_pack");
}

int hyres_eb_fwd(const float* z, const float* packed, const float* noise, int training, float* z_q, float* lik,
                 float* z_hat_ste, long long P, int C, hyres_stream_t s) {
    HY_REQUIRE(z && packed && z_q && lik && (!training || noise), HYRES_E_ARG, "eb_fwd: NULL");
    long long n = P * C;
    hipLaunchKernelGGL(eb_fwd_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), z, packed, noise, training,
                       z_q, lik, z_hat_ste, P, C);
    return HY_LAUNCH_CHECK("eb_fwd");
}

long long hyres_eb_workspace_bytes(long long P, int C) {
    int per = 1024;
    long long nb = (P + per - 1) / per;
    return nb * C * HYRES_EB_REC * 4;
}

int hyres_eb_bwd(const float* z_q, const float* packed, const float* lik, const float* g_lik, const float* g_zhat,
                 int training, int noisequant, float* g_z, float* g_packed_ws, long long P, int C,
                 hyres_stream_t s) {
    HY_REQUIRE(z_q && packed && g_z && g_packed_ws, HYRES_E_ARG, "eb_bwd: NULL");
    int per = 1024;
    int nb = (int)((P + per - 1) / per);
    hipLaunchKernelGGL(eb_bwd_kernel, dim3(C, nb), dim3(256), 0, as_stream(s), z_q, packed, lik, g_lik, g_zhat,
                       training, noisequant, g_z, g_packed_ws, P, C, per);
    return HY_LAUNCH_CHECK("eb_bwd");
}

int hyres_eb_unpack_grad(const float* g_packed_ws, int nblocks, const float* const* mats, const float* const* factors,
                         float* const* g_mats, float* const* g_biases, float* const* g_factors, float* g_quantiles,
                         int C, int accumulate, hyres_stream_t s) {
    HY_REQUIRE(g_packed_ws && mats && factors && g_mats && g_biases && g_factors, HYRES_E_ARG, "eb_unpack: NULL");
    EbPtrs p{};
    for (int i = 0; i < 5; ++i) { p.m[i] = mats[i]; p.gm[i] = g_mats[i]; p.gb[i] = g_biases[i]; }
    for (int i = 0; i < 4; ++i) { p.f[i] = factors[i]; p.gf[i] = g_factors[i]; }
    hipLaunchKernelGGL(eb_unpack_grad_kernel, dim3((C + 127) / 128), dim3(128), 0, as_stream(s), g_packed_ws, nblocks,
                       p, g_quantiles, C, accumulate);
    return HY_LAUNCH_CHECK("eb_unpack_grad");
}

int hyres_eb_aux_loss(const float* packed, const float* quantiles, const float* target, float* loss,
                      float* g_quantiles, int C, hyres_stream_t s) {
    HY_REQUIRE(packed && quantiles && target && loss, HYRES_E_ARG, "eb_aux_loss: NULL");
    hipLaunchKernelGGL(eb_aux_kernel, dim3(1), dim3(512), 0, as_stream(s), packed, quantiles, target, loss,
                       g_quantiles, C);
    return HY_LAUNCH_CHECK("eb_aux_loss");
}


int hyres_gc_symbols(const float* y, int ldy, const float* params, int ldp, int M, int B, int H, int W, int parity,
                     const float* scale_table, int nt, int* sym, int* idx, hyres_stream_t s) {
    HY_REQUIRE(params && scale_table && idx && nt >= 1 && (!y || sym), HYRES_E_ARG, "gc_symbols: bad args");
    const long long n = (long long)B * M * H * W;
    hipLaunchKernelGGL(gc_symbols_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), y, ldy, params, ldp, M, B,
                       H, W, parity, scale_table, nt, sym, idx);
    return HY_LAUNCH_CHECK("gc_symbols");
}

int hyres_gc_dequant(const int* sym, const float* params, int ldp, int M, int B, int H, int W, float* out, int ldo,
                     int accumulate, hyres_stream_t s) {
    HY_REQUIRE(sym && params && out, HYRES_E_ARG, "gc_dequant: NULL");
    const long long n = (long long)B * M * H * W;
    hipLaunchKernelGGL(gc_dequant_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), sym, params, ldp, M, B, H,
                       W, out, ldo, accumulate);
    return HY_LAUNCH_CHECK("gc_dequant");
}

int hyres_eb_symbols(const float* z, int ldz, const float* medians, int B, int H, int W, int C, int* sym,
                     float* zhat, int ldo, int dequant, hyres_stream_t s) {
    HY_REQUIRE(medians && sym && (dequant ? zhat != nullptr : z != nullptr), HYRES_E_ARG, "eb_symbols: NULL");
    const long long n = (long long)B * C * H * W;
    hipLaunchKernelGGL(eb_symbols_kernel, dim3(grid_for_e(n)), dim3(256), 0, as_stream(s), z, ldz, medians, B, H, W, C,
                       sym, zhat, ldo, dequant);
    return HY_LAUNCH_CHECK("eb_symbols");
}

}  // extern "C"
