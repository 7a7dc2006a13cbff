// VGG16 perceptual-loss pieces (src/losses/vgg16.py: VGGLoss, used by src/losses/rd_loss.py:40 when
// alpha > 0) on gfx950.  The 13 convolutions run on the implicit-GEMM conv kernels (conv.hip); this file
// has the rest of the feature pipeline, NHWC:
//   * torchvision Normalize(mean, std): y = (x - mean_c) / std_c (+ backward g / std_c);
//   * ReLU forward at a slice boundary (a slice ends on a conv's pre-activation, vgg16.py:29-33);
//   * MaxPool2d(2, 2): first maximum in (0,0),(0,1),(1,0),(1,1) order wins (torch's rule), argmax kept
//     for the backward scatter;
//   * the per-slice L1 term mean|fx - fy| (two-pass deterministic sum) and its backward
//     coef * sign(fx - fy) / n.
#include "common.h"

namespace hyres {

#define VGG_GRID_STRIDE(i, n) \
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

static inline int vgg_grid(long long n) {
    long long b = (n + 255) / 256;
    return (int)std::max<long long>(1, std::min<long long>(b, 8192));
}

struct ChanAffine {
    float mean[4], std[4];
};

__global__ void normalize_fwd_kernel(const float* x, float* y, long long n, int C, ChanAffine a) {
    VGG_GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        y[i] = (x[i] - a.mean[c]) / a.std[c];
    }
}
__global__ void normalize_bwd_kernel(const float* g, float* gx, long long n, int C, ChanAffine a, int acc) {
    VGG_GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        const float v = g[i] / a.std[c];
        gx[i] = acc ? gx[i] + v : v;
    }
}
__global__ void relu_fwd_kernel(const float* x, float* y, long long n) {
    VGG_GRID_STRIDE(i, n) y[i] = fmaxf(x[i], 0.f);
}

// NHWC 2x2/2 max pool: one thread per (b, i, j, c)
__global__ void maxpool2_fwd_kernel(const float* x, float* y, unsigned char* arg, int B, int H, int W, int C) {
    const int Ho = H / 2, Wo = W / 2;
    const long long n = (long long)B * Ho * Wo * C;
    VGG_GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        long long p = i / C;
        const int j = (int)(p % Wo);
        p /= Wo;
        const int r = (int)(p % Ho);
        const int b = (int)(p / Ho);
        const float* src = x + (((long long)b * H + 2 * r) * W + 2 * j) * C + c;
        const float v[4] = {src[0], src[C], src[(long long)W * C], src[(long long)W * C + C]};
        float m = v[0];
        int k = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
            if (v[q] > m || isnan(v[q])) { m = v[q]; k = q; }
        y[i] = m;
        arg[i] = (unsigned char)k;
    }
}
// backward: each input element takes g of its window iff it was the argmax (gather form, no atomics)
__global__ void maxpool2_bwd_kernel(const float* g, const unsigned char* arg, float* gx, int B, int H, int W, int C,
                                    int acc) {
    const long long n = (long long)B * H * W * C;
    const int Ho = H / 2, Wo = W / 2;
    VGG_GRID_STRIDE(i, n) {
        const int c = (int)(i % C);
        long long p = i / C;
        const int w = (int)(p % W);
        p /= W;
        const int h = (int)(p % H);
        const int b = (int)(p / H);
        float v = 0.f;
        if (h / 2 < Ho && w / 2 < Wo) {
            const long long o = (((long long)b * Ho + h / 2) * Wo + w / 2) * C + c;
            if (arg[o] == (unsigned char)((h & 1) * 2 + (w & 1))) v = g[o];
        }
        gx[i] = acc ? gx[i] + v : v;
    }
}

__device__ __forceinline__ float vgg_block_sum(float v, float* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    return red[0];
}
__global__ void absdiff_partial_kernel(const float* a, const float* b, long long n, float* part) {
    __shared__ float red[256];
    float s = 0.f;
    VGG_GRID_STRIDE(i, n) s += fabsf(a[i] - b[i]);
    const float r = vgg_block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}
// out[0] (+)= scale * sum(part[0..nb))
__global__ void absdiff_final_kernel(const float* part, int nb, float scale, float* out, int acc) {
    __shared__ float red[256];
    float s = 0.f;
    for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
    const float r = vgg_block_sum(s, red);
    if (threadIdx.x == 0) out[0] = acc ? out[0] + r * scale : r * scale;
}
__global__ void absdiff_bwd_kernel(const float* a, const float* b, const float* coef, float scale, float* ga,
                                   long long n, int acc) {
    const float c = coef[0] * scale;
    VGG_GRID_STRIDE(i, n) {
        const float d = a[i] - b[i];
        const float v = c * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
        ga[i] = acc ? ga[i] + v : v;
    }
}

}  // namespace hyres

using namespace hyres;

extern "C" {

static ChanAffine chan_affine(const float* mean, const float* stdv, int C) {
    ChanAffine a{};
    for (int c = 0; c < C; ++c) {
        a.mean[c] = mean[c];
        a.std[c] = stdv[c];
    }
    return a;
}

int hyres_normalize_fwd(const float* x, float* y, long long P, int C, const float* mean, const float* stdv,
                        hyres_stream_t s) {
    HY_REQUIRE(x && y && mean && stdv && C >= 1 && C <= 4, HYRES_E_ARG, "normalize_fwd: bad args");
    const long long n = P * C;
    hipLaunchKernelGGL(normalize_fwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), x, y, n, C,
                       chan_affine(mean, stdv, C));
    return HY_LAUNCH_CHECK("normalize_fwd");
}
int hyres_normalize_bwd(const float* g, float* gx, long long P, int C, const float* mean, const float* stdv,
                        int accumulate, hyres_stream_t s) {
    HY_REQUIRE(g && gx && mean && stdv && C >= 1 && C <= 4, HYRES_E_ARG, "normalize_bwd: bad args");
    const long long n = P * C;
    hipLaunchKernelGGL(normalize_bwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), g, gx, n, C,
                       chan_affine(mean, stdv, C), accumulate);
    return HY_LAUNCH_CHECK("normalize_bwd");
}
int hyres_relu_fwd(const float* x, float* y, long long n, hyres_stream_t s) {
    HY_REQUIRE(x && y, HYRES_E_ARG, "relu_fwd: NULL");
    hipLaunchKernelGGL(relu_fwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), x, y, n);
    return HY_LAUNCH_CHECK("relu_fwd");
}
int hyres_maxpool2_fwd(const float* x, float* y, unsigned char* argmax, int B, int H, int W, int C, hyres_stream_t s) {
    HY_REQUIRE(x && y && argmax && H >= 2 && W >= 2, HYRES_E_ARG, "maxpool2_fwd: bad args");
    const long long n = (long long)B * (H / 2) * (W / 2) * C;
    hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), x, y, argmax, B, H, W, C);
    return HY_LAUNCH_CHECK("maxpool2_fwd");
}
int hyres_maxpool2_bwd(const float* g, const unsigned char* argmax, float* gx, int B, int H, int W, int C,
                       int accumulate, hyres_stream_t s) {
    HY_REQUIRE(g && argmax && gx, HYRES_E_ARG, "maxpool2_bwd: NULL");
    const long long n = (long long)B * H * W * C;
    hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), g, argmax, gx, B, H, W, C,
                       accumulate);
    return HY_LAUNCH_CHECK("maxpool2_bwd");
}
long long hyres_absdiff_workspace_bytes(long long n) { return (long long)vgg_grid(n) * 4 + 256; }
int hyres_absdiff_mean(const float* a, const float* b, long long n, float* out, int accumulate, void* ws,
                       long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(a && b && out && n > 0, HYRES_E_ARG, "absdiff_mean: bad args");
    const int nb = vgg_grid(n);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * 4, HYRES_E_WORKSPACE, "absdiff_mean: workspace");
    hipLaunchKernelGGL(absdiff_partial_kernel, dim3(nb), dim3(256), 0, as_stream(s), a, b, n, (float*)ws);
    int rc = HY_LAUNCH_CHECK("absdiff_partial");
    if (rc) return rc;
    hipLaunchKernelGGL(absdiff_final_kernel, dim3(1), dim3(256), 0, as_stream(s), (const float*)ws, nb,
                       (float)(1.0 / (double)n), out, accumulate);
    return HY_LAUNCH_CHECK("absdiff_final");
}
int hyres_absdiff_bwd(const float* a, const float* b, const float* coef, long long n, float* ga, int accumulate,
                      hyres_stream_t s) {
    HY_REQUIRE(a && b && coef && ga && n > 0, HYRES_E_ARG, "absdiff_bwd: bad args");
    hipLaunchKernelGGL(absdiff_bwd_kernel, dim3(vgg_grid(n)), dim3(256), 0, as_stream(s), a, b, coef,
                       (float)(1.0 / (double)n), ga, n, accumulate);
    return HY_LAUNCH_CHECK("absdiff_bwd");
}

}  // extern "C"
