// Fused ResidualUnit / ResidualBottleneckBlock forward for autocast inference (fp16 activations, f16 MFMA).
//
//   ResidualUnit (models/layers/attention.py:11-30):   y = relu(x + W3 * relu(W2 (*) relu(W1 * x + b1) + b2) + b3)
//   ResidualBottleneckBlock (compressai, g_a.2 / g_s.2 / g_s.6 via models/checkerboard.py:38,42,51,56):
//                                                       y =      x + W3 * relu(W2 (*) relu(W1 * x + b1) + b2) + b3
//
// with N = 128 (W1: 1x1 128 -> 64, W2: 3x3 64 -> 64, W3: 1x1 64 -> 128). The unfused autocast path runs three convs and
// moves x, t1 (write + read), t2 (write + read), x again (residual) and y through HBM: 5 N-channel-equivalents of
// traffic per pixel. Here one persistent 512-thread block per CU walks 4-row x 64-pixel output tiles and keeps t1 and t2
// on chip, so HBM sees x once (the halo re-reads and the residual re-read hit L2) and y once: 2 of the 5.
//
// Per tile (8 waves, transposed products C^T = W X^T as conv3x3_wres_f16_kernel, fp32 accumulation, f16 operands):
//   1. t1 over the 6 x 66-pixel halo (396 pixels, padded to 13 blocks of 32): x streams through LDS in 32-channel
//      chunks (fp16, 40-half rows, two buffers); W1's fragments for the wave's 32-channel output block stay in
//      registers for the whole launch. Epilogue: + b1, ReLU, zero outside the image (the 3x3's zero padding applies to
//      t1), fp16 into LDS as two 32-channel chunks — the layout conv3x3_wres_f16_kernel reads its halo in.
//   2. t2 = the 3x3 on t1 with W2 (fp16, LDS-resident for the launch: 92 KB), exactly wres16's inner loop;
//      + b2, ReLU, fp16 into LDS (the t1 buffers are free by then).
//   3. y = W3 t2 + b3 + x (ReLU for the ResidualUnit), W3's fragments in registers, the residual read as fp16,
//      y stored fp16. The next tile's first x chunk is loaded into registers during this phase.
// Training (AMP, t1 / t2 outputs given): the same launch also writes t1 (each tile's own pixels) and t2 to HBM — the
// backward needs them (weight-gradient operands, ReLU masks) — and the three convs' backward closures are recorded
// as usual (hyres_hip.ops.residual_unit_fused): only the re-reads of t1, t2 and x disappear.
// The fp16 rounding points are the unfused autocast path's (t1, t2 stored fp16; every GEMM on fp16 operands), so the
// results agree with it up to fp32 summation order (tests/test_ru_fused_gpu.py).
#include "common.h"
#include "conv_common.h"

namespace hyres {

namespace {

constexpr int RU_N = 128, RU_M = 64;               // block width N, bottleneck N / 2
constexpr int RU_R = 4, RU_TW = 64;                 // output tile: 4 rows x 64 pixels
constexpr int RU_HH = RU_R + 2, RU_HW = RU_TW + 2;  // t1 halo tile 6 x 66
constexpr int RU_HNPX = RU_HH * RU_HW;              // 396
constexpr int RU_PB1 = (RU_HNPX + 31) / 32;         // 13 pixel blocks of 32 in phase 1
constexpr int RU_PH = 40;                           // halves per staged 32-channel row (80 B: conflict-free b128)
constexpr int RU_TBUF = RU_PB1 * 32 * RU_PH;        // one staging buffer: 416 rows x 40 halves
constexpr int RU_W2 = 2 * 9 * RU_M * RU_PH;         // W2 [chunk][tap][co][40]
constexpr int RU_XE = RU_HNPX * 8;                  // x chunk: 396 pixels x 8 half4 (32 channels)
constexpr int RU_XV = (RU_XE + 511) / 512;          // half4 loads per thread per chunk (7)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ half8 ld_w8(const float* p) {  // 8 consecutive fp32 weights -> f16 fragment
    const float4 a = ld4(p), b = ld4(p + 4);
    return half8{(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
                 (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
}

}  // namespace

struct RuArgs {
    const _Float16* x;  // [B][H][W][128] fp16
    _Float16* y;        // [B][H][W][128] fp16
    const float *w1, *b1, *w2, *b2, *w3, *b3;  // PyTorch layouts: w1 [64][128], w2 [64][64][3][3], w3 [128][64]
    _Float16 *t1, *t2;  // training (AMP): the intermediates [B][H][W][64] fp16 for the backward, or NULL
    int B, H, W, ntiles, final_relu;
};

// GUARD: the whole VGPR file of its SIMDs (2 waves x 256; the code needs 228). With the compiler's 232 a 48-VGPR hole
// per SIMD let another stream's waves share them, and a side-stream bilinear then lost loaded values (round 5,
// scripts/bf6_interference_repro.hip ru: 20 of 20 runs wrong; DESIGN §4 "Cross-kernel interference"). No cost: the
// 158.7 KB of LDS already limits the CU to one block. GUARD = false only for that diagnosis (hyres_conv_tuning key 9 = 0).
template <bool GUARD>
__global__ __launch_bounds__(512, 1) void ru_fused_f16_kernel(const RuArgs a) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[RU_W2 + 2 * RU_TBUF];
    if constexpr (GUARD) asm volatile("" ::: "v255");
    _Float16* const W2s = lds;
    _Float16* const T = lds + RU_W2;  // two buffers: x chunks (phase 1), t1 chunks (phase 2), t2 chunks (phase 3)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    const int H = a.H, W = a.W;
    const int nrt = (H + RU_R - 1) / RU_R, nct = W / RU_TW;
    // tiles walked XCD-contiguously (hardware XCD = blockIdx.x % 8; gridDim.x % 8 == 0): vertically adjacent tiles share
    // two halo rows of x
    const int xcd = blockIdx.x & 7, nx = gridDim.x >> 3, jx = blockIdx.x >> 3;
    const int q = a.ntiles >> 3, r8 = a.ntiles & 7;
    const int tbeg = xcd * q + min(xcd, r8), tcnt = q + (xcd < r8 ? 1 : 0);
    const int mytiles = jx < tcnt ? (tcnt - 1 - jx) / nx + 1 : 0;
    auto tile_of = [&](int k, int& b, int& i0, int& j0) {
        int l = tbeg + jx + k * nx;
        const int rt = l % nrt;
        l /= nrt;
        const int ct = l % nct;
        b = l / nct;
        i0 = rt * RU_R;
        j0 = ct * RU_TW;
    };

    // ---- weights: W2 -> LDS fp16 [c][t][co][40] (ci = 32c + k); W1 / W3 fragments -> registers (launch-resident)
    for (int f = tid; f < RU_M * RU_M * 9; f += 512) {  // w2[co][ci][t], linear over the PyTorch layout
        const int co = f / (RU_M * 9), rem = f - co * (RU_M * 9), ci = rem / 9, t = rem - ci * 9;
        W2s[(((ci >> 5) * 9 + t) * RU_M + co) * RU_PH + (ci & 31)] = (_Float16)a.w2[f];
    }
    const int cb1 = wave & 1;  // phase 1: t1 output-channel block of this wave
    half8 w1f[8];               // W1[32 cb1 + lr][16 s + 8 lh .. +7], s = 0..7 (K = 128)
#pragma unroll
    for (int s = 0; s < 8; ++s) w1f[s] = ld_w8(a.w1 + (32 * cb1 + lr) * RU_N + 16 * s + 8 * lh);
    const int cb3 = wave & 3;  // phase 3: y output-channel block of this wave
    half8 w3f[4];               // W3[32 cb3 + lr][16 s + 8 lh .. +7], s = 0..3 (K = 64)
#pragma unroll
    for (int s = 0; s < 4; ++s) w3f[s] = ld_w8(a.w3 + (32 * cb3 + lr) * RU_M + 16 * s + 8 * lh);

    const long long img = (long long)H * W * RU_N;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, (short)0, (int)std::min<long long>((long long)a.B * img * 2, 0x7FFFFFF0LL), 0x00020000);
    half4_t xreg[RU_XV];
    auto xload = [&](int k, int c) {  // x chunk c (channels 32c..32c+31) of tile k's halo -> registers
        int b, i0, j0;
        tile_of(k, b, i0, j0);
        const int base = b * (int)img;
#pragma unroll
        for (int v = 0; v < RU_XV; ++v) {
            const int e = tid + 512 * v;
            const int px = e >> 3, c4 = e & 7;
            const int hr = px / RU_HW, hc = px - hr * RU_HW;
            const int ih = i0 - 1 + hr, iw = j0 - 1 + hc;
            const bool ok = e < RU_XE && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            const int off = ok ? (base + (ih * W + iw) * RU_N + 32 * c + 4 * c4) * 2 : (int)0x80000000;
            xreg[v] = __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
        }
    };
    auto xstore = [&](_Float16* buf) {
#pragma unroll
        for (int v = 0; v < RU_XV; ++v) {
            const int e = tid + 512 * v;
            if (e < RU_XE) *reinterpret_cast<half4_t*>(&buf[(e >> 3) * RU_PH + 4 * (e & 7)]) = xreg[v];
        }
    };

    // phase 1 pixel blocks of this wave: 2 output-channel blocks x 13 pixel blocks over 8 waves
    const int pbase = wave >> 1;  // pixel blocks pbase, pbase + 4, pbase + 8, pbase + 12 (< 13)
    const int orow = wave & 3, wn = wave >> 2;  // phase 2: output row, t2 channel half
    const int pb3 = wave >> 2;  // phase 3: pixel blocks pb3, +2, +4, +6

    if (mytiles > 0) {
        xload(0, 0);
        xstore(T);
        xload(0, 1);
    }
    __syncthreads();
    for (int k = 0; k < mytiles; ++k) {
        int b, i0, j0;
        tile_of(k, b, i0, j0);
        // ---------------- phase 1: t1 = relu(W1 x + b1) over the halo
        floatx16 acc1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc1[i][r] = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const _Float16* X = T + (c & 1) * RU_TBUF;
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const half8 af = w1f[2 * c + ss];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int pb = pbase + 4 * i;
                    if (pb < RU_PB1) {
                        const half8 bf = *reinterpret_cast<const half8*>(&X[(32 * pb + lr) * RU_PH + 16 * ss + 8 * lh]);
                        acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc1[i], 0, 0, 0);
                    }
                }
            }
            if (c + 1 < 4) {
                xstore(T + ((c + 1) & 1) * RU_TBUF);  // chunk c + 1 (its buffer held chunk c - 1: done at the barrier)
                if (c + 2 < 4) xload(k, c + 2);
            }
            __syncthreads();
        }
        // t1 epilogue -> T as [chunk = cb1][halo pixel][40] (zero outside the image)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pb = pbase + 4 * i;
            if (pb >= RU_PB1) continue;
            const int px = 32 * pb + lr;
            const int hr = px / RU_HW, hc = px - hr * RU_HW;
            const int ih = i0 - 1 + hr, iw = j0 - 1 + hc;
            const bool inside = px < RU_HNPX && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            // training: the tile's own (center) pixels of t1 also go to HBM — every pixel is the center of one tile
            const bool center = a.t1 != nullptr && inside && hr >= 1 && hr <= RU_R && hc >= 1 && hc <= RU_TW;
            const long long tpix = ((long long)b * H + ih) * W + iw;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int co = 8 * qd + 4 * lh;  // within the 32-channel block cb1
                const float4 bb = ld4(a.b1 + 32 * cb1 + co);
                const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
                half4_t h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (_Float16)(inside ? fmaxf(acc1[i][4 * qd + r] + bv[r], 0.f) : 0.f);
                *reinterpret_cast<half4_t*>(&T[cb1 * RU_TBUF + px * RU_PH + co]) = h;
                if (center) *reinterpret_cast<half4_t*>(&a.t1[tpix * RU_M + 32 * cb1 + co]) = h;
            }
        }
        __syncthreads();
        // ---------------- phase 2: t2 = relu(W2 (*) t1 + b2), conv3x3_wres_f16_kernel's loop
        floatx16 acc2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc2[i][r] = 0.f;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const _Float16* Hc = T + c * RU_TBUF;
            const _Float16* Bc = W2s + c * 9 * RU_M * RU_PH;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int dh = t / 3 - 1, dw = t % 3 - 1;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const half8 bf = *reinterpret_cast<const half8*>(&Bc[(t * RU_M + wn * 32 + lr) * RU_PH + 16 * ks + 8 * lh]);
#pragma unroll
                    for (int at = 0; at < 2; ++at) {
                        const int px = (orow + 1 + dh) * RU_HW + at * 32 + lr + 1 + dw;
                        const half8 af = *reinterpret_cast<const half8*>(&Hc[px * RU_PH + 16 * ks + 8 * lh]);
                        acc2[at] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf, af, acc2[at], 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();  // every wave is done reading t1
        // t2 epilogue -> T as [chunk = wn][output pixel (orow*64 + 32 at + lr)][40]
#pragma unroll
        for (int at = 0; at < 2; ++at) {
            const int px = orow * RU_TW + 32 * at + lr;
            const bool store = a.t2 != nullptr && i0 + orow < H;
            const long long tpix = ((long long)b * H + i0 + orow) * W + j0 + 32 * at + lr;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int co = 8 * qd + 4 * lh;
                const float4 bb = ld4(a.b2 + 32 * wn + co);
                const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
                half4_t h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (_Float16)fmaxf(acc2[at][4 * qd + r] + bv[r], 0.f);
                *reinterpret_cast<half4_t*>(&T[wn * RU_TBUF + px * RU_PH + co]) = h;
                if (store) *reinterpret_cast<half4_t*>(&a.t2[tpix * RU_M + 32 * wn + co]) = h;
            }
        }
        __syncthreads();
        // next tile's first x chunk into registers while phase 3 computes
        if (k + 1 < mytiles) xload(k + 1, 0);
        // ---------------- phase 3: y = (relu)(W3 t2 + b3 + x)
        floatx16 acc3[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc3[i][r] = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const _Float16* Tc = T + (s >> 1) * RU_TBUF;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int px = 32 * (pb3 + 2 * i) + lr;
                const half8 bf = *reinterpret_cast<const half8*>(&Tc[px * RU_PH + 16 * (s & 1) + 8 * lh]);
                acc3[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w3f[s], bf, acc3[i], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int px = 32 * (pb3 + 2 * i) + lr;
            const int row = px >> 6, col = px & 63;
            const int ii = i0 + row;
            if (ii >= H) continue;
            const long long pix = ((long long)b * H + ii) * W + j0 + col;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int co = 32 * cb3 + 8 * qd + 4 * lh;
                const float4 bb = ld4(a.b3 + co);
                const float4 xv = ldv4<true>(reinterpret_cast<const float*>(a.x), pix * RU_N + co);
                float4 v = make_float4(acc3[i][4 * qd] + bb.x + xv.x, acc3[i][4 * qd + 1] + bb.y + xv.y,
                                       acc3[i][4 * qd + 2] + bb.z + xv.z, acc3[i][4 * qd + 3] + bb.w + xv.w);
                if (a.final_relu) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                stv4<true>(reinterpret_cast<float*>(a.y), pix * RU_N + co, v);
            }
        }
        if (k + 1 < mytiles) {
            __syncthreads();  // every wave is done reading t2
            xstore(T);
            xload(k + 1, 1);
            __syncthreads();
        }
    }
}

}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_ru_fused_f16_ok(int B, int H, int W, int N) {
    return N == RU_N && B > 0 && H > 0 && W > 0 && W % RU_TW == 0 && (long long)B * H * W * RU_N * 2 < 0x7FFFFFF0LL;
}

int hyres_ru_fused_f16(const void* x, void* y, int B, int H, int W, int N, const float* w1, const float* b1,
                       const float* w2, const float* b2, const float* w3, const float* b3, int final_relu,
                       void* t1, void* t2, hyres_stream_t s) {
    HY_REQUIRE(x && y && w1 && b1 && w2 && b2 && w3 && b3 && x != y, HYRES_E_ARG, "ru_fused_f16: NULL or in place");
    HY_REQUIRE((t1 == nullptr) == (t2 == nullptr) && (!t1 || (aligned16(t1) && aligned16(t2))), HYRES_E_ARG,
               "ru_fused_f16: t1 and t2 both NULL (inference) or both 16-byte aligned outputs (training)");
    HY_REQUIRE(hyres_ru_fused_f16_ok(B, H, W, N), HYRES_E_SHAPE,
               "ru_fused_f16: N = 128, W %% 64 == 0 and a batch < 2 GB needed (B %d H %d W %d N %d)", B, H, W, N);
    HY_REQUIRE(aligned16(x) && aligned16(y) && aligned16(w1) && aligned16(w3) && aligned16(b1) && aligned16(b2) &&
                   aligned16(b3),
               HYRES_E_ALIGN, "ru_fused_f16: 16-byte aligned operands needed");
    RuArgs a;
    a.x = (const _Float16*)x;
    a.y = (_Float16*)y;
    a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.w3 = w3; a.b3 = b3;
    a.t1 = (_Float16*)t1;
    a.t2 = (_Float16*)t2;
    a.B = B; a.H = H; a.W = W;
    a.ntiles = B * ((H + RU_R - 1) / RU_R) * (W / RU_TW);
    a.final_relu = final_relu ? 1 : 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus < 8)
        cus = 256;
    // one block per CU, at most one per tile, a multiple of 8 (XCD-contiguous tile ranges)
    const int blocks = std::max(8, (std::min(cus, a.ntiles) + 7) & ~7);
    if (g_tune[9] == 0)  // diagnostic only (DESIGN §4 "Cross-kernel interference")
        hipLaunchKernelGGL(ru_fused_f16_kernel<false>, dim3(blocks), dim3(512), 0, as_stream(s), a);
    else
        hipLaunchKernelGGL(ru_fused_f16_kernel<true>, dim3(blocks), dim3(512), 0, as_stream(s), a);
    return HY_LAUNCH_CHECK("ru_fused_f16_kernel");
}

}  // extern "C"
