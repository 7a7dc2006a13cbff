// Implicit-GEMM convolutions for the HyRES hot path on CDNA4 (gfx950), fp32 in / fp32 accumulate.
//
// Every Conv2d / ConvTranspose2d / GDN contraction of the reference (models/checkerboard.py:35-88,
// models/layers/attention.py, models/layers/enhancement.py, compressai GDN / RBB) and their
// input-gradients run through ONE kernel family:
//     Y[b, i*osh+oph, j*osw+opw, co] = epi( sum_{t in taps(phase)} sum_ci X[b, i*ish+dh_t, j*isw+dw_t, ci] * W2[co][t][ci] )
// GEMM view: M = output pixels of one phase (NHWC rows), N = output channels, K = taps x Ci.
//   * operands are staged HBM -> registers -> LDS in 32-deep K chunks (the next chunk's global
//     loads are issued before the current chunk's MFMAs: issue-early / write-late);
//   * the MFMA is v_mfma_f32_32x32x2_f32 (exact fp32, 64 FLOP/clk/SIMD = the fp32 peak);
//   * both LDS tiles are stored K-contiguous ([row][k], +4 float pad) and the K order inside a chunk
//     is permuted so that lane-half h consumes k = 16h + s at MFMA step s: one ds_read_b128 feeds four
//     consecutive MFMA steps (conflict-free with the 36-float row pitch).
// Weight gradients use a second kernel (P^T Q over pixels, split-K slabs + deterministic reduce).
#include "conv_common.h"

namespace hyres {

constexpr int PADK = 36;  // LDS row pitch (floats)

struct ConvArgs {
    hyres_conv_geom g;
    const float* x;
    const float* w2;
    int ldw;
    float* y;
    hyres_epilogue e;
    int M;       // B*Hq*Wq
    int nsplit;  // split-K factor (1 = fused epilogue)
    int cps;     // K chunks per split
    float* slab; // [nsplit][nphase][M][Co] partials when nsplit > 1
    int vec4;    // every epilogue operand 16B aligned with ld % 4 == 0 and Co % 4 == 0
    int w_bytes; // bytes of W2 (buffer-resource range)
    int xcd;     // 1: grid.x = M tiles x N tiles in XCD-aware order (grid.y = 1)
    int prio;    // 1: raise the wave priority while it issues its MFMA cluster (s_setprio)
    int x_bytes; // conv1x1_stream_kernel: bytes of X (buffer-resource range)
    int rsrc_ok; // every epilogue operand / output spans < 2 GB: the epilogues may address them by buffer resources
    int b6sw;    // bf16x6 implicit GEMM: 64-B LDS rows with the 16-B slot XOR-swizzled by row bits 2..3 (round 6,
                 // hyres_conv_tuning key 19, default 1) instead of 80-B padded rows
};

// Buffer resource of an epilogue operand: an absent operand (p == NULL) gets an empty resource, so its loads return
// 0 without a branch (a load behind a branch is waited on at the join: the epilogue's loads would serialise)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t opnd_rsrc(const void* p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, p ? (int)std::min<long long>(bytes, 0x7FFFFFF0LL) : 0,
                                             0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ half4_t bload4h(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ float4 h2f4(half4_t h) { return make_float4((float)h.x, (float)h.y, (float)h.z, (float)h.w); }


struct EpiChannel {
    float bias, slope;
};

__device__ __forceinline__ EpiChannel epi_channel(const hyres_epilogue& e, int n) {
    EpiChannel c;
    c.bias = e.bias ? e.bias[n] : 0.f;
    c.slope = (e.act == HYRES_ACT_PRELU) ? e.slope[0] : 0.f;
    return c;
}

// Saved-activation operand of a backward epilogue (the ReLU mask's y, GDN-backward's x and norm): fp16 when
// the whole epilogue is fp16 (H) or, with fp32 X/Y, when io_f16 carries HYRES_IO_AUX16 (AMP training keeps
// its activations fp16 and its gradients fp32). A uniform kernel-argument branch.
template <bool H>
__device__ __forceinline__ float ld_aux(const hyres_epilogue& e, const float* p, long long i) {
    if constexpr (H) return ldv<true>(p, i);
    else return (e.io_f16 & HYRES_IO_AUX16) ? ldv<true>(p, i) : p[i];
}
template <bool H>
__device__ __forceinline__ float4 ld_aux4(const hyres_epilogue& e, const float* p, long long i) {
    if constexpr (H) return ldv4<true>(p, i);
    else return (e.io_f16 & HYRES_IO_AUX16) ? ldv4<true>(p, i) : ld4(p + i);
}

// Apply the epilogue to one GEMM result v for output pixel ``pix`` / channel n and store it
// (H: y and the activation operands res / aux0 / out2 are fp16 in HBM).
// SAB: the HYRES_EPI_SA_BWD case compiled in (only conv_fwd_body, the one kernel family the launcher routes that
// epilogue to: every other caller keeps its register allocation — the case cost the weight-resident f16 kernels a spill)
template <bool H = false, bool SAB = false>
__device__ __forceinline__ void epi_store(const hyres_epilogue& e, float* y, int ldy, long long pix, int n, float v,
                                          const EpiChannel& c) {
    switch (e.kind) {
        case HYRES_EPI_ROWSCALE:  // the product scaled per output pixel first (aux1[pix * ld1]), then as BIAS
            v *= e.aux1[pix * e.ld1];
            [[fallthrough]];
        case HYRES_EPI_BIAS: {
            v += c.bias;
            if (e.res) v += ldv<H>(e.res, pix * e.ldres + n);
            if (e.out2) stv<H>(e.out2, pix * e.ldo2 + n, v);  // pre-activation (PReLU backward)
            if (e.act == HYRES_ACT_RELU) v = fmaxf(v, 0.f);
            else if (e.act == HYRES_ACT_PRELU) v = v >= 0.f ? v : c.slope * v;
            else if (e.act == HYRES_ACT_RELU_MASK) v = ld_aux<H>(e, e.aux0, pix * e.ld0 + n) > 0.f ? v : 0.f;
            break;
        }
        case HYRES_EPI_GDN:
        case HYRES_EPI_IGDN: {
            const float nv = v + c.bias;
            const float xv = ldv<H>(e.aux0, pix * e.ld0 + n);
            stv<H>(e.out2, pix * e.ldo2 + n, nv);
            v = (e.kind == HYRES_EPI_GDN) ? xv * (1.0f / sqrtf(nv)) : xv * sqrtf(nv);
            break;
        }
        case HYRES_EPI_SA_BWD: {  // SpatialAttention's mean / max backward: + d mean / C, + d max at the argmax
            if constexpr (SAB) {
                const float* gm = e.aux0 + pix * e.ld0;
                v = v + gm[0] + (n == reinterpret_cast<const int*>(e.aux2)[pix] ? gm[1] : 0.f);
            }
            break;
        }
        case HYRES_EPI_GDN_BWD:
        case HYRES_EPI_IGDN_BWD: {  // H (AMP fp16 gradients): x, the incoming gradient and the norm all fp16
            const float xv = ld_aux<H>(e, e.aux0, pix * e.ld0 + n);
            const float gv = ldv<H>(e.aux1, pix * e.ld1 + n);
            const float nv = ld_aux<H>(e, e.aux2, pix * e.ld2 + n);
            const float f = (e.kind == HYRES_EPI_GDN_BWD) ? (1.0f / sqrtf(nv)) : sqrtf(nv);
            v = 2.0f * xv * v + gv * f;
            break;
        }
        default: break;
    }
    if constexpr (H) {
        if (e.accumulate) v += ldv<true>(y, pix * ldy + n);  // fp16 gradient accumulation (AMP): fp32 add
        stv<true>(y, pix * ldy + n, v);
    } else {
        float* yp = y + pix * ldy + n;
        if (e.accumulate) v += *yp;
        *yp = v;
    }
}

__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// float4 variant of epi_store for channels n..n+3 (all operands 16B aligned).
template <bool H = false, bool SAB = false>
__device__ __forceinline__ void epi_store4(const hyres_epilogue& e, float* y, int ldy, long long pix, int n, float4 v,
                                           float slope, bool use_pre = false,
                                           float4 rpre = make_float4(0.f, 0.f, 0.f, 0.f)) {
    float o[4] = {v.x, v.y, v.z, v.w};
    switch (e.kind) {
        case HYRES_EPI_ROWSCALE: {
            const float sc = e.aux1[pix * e.ld1];
#pragma unroll
            for (int c = 0; c < 4; ++c) o[c] *= sc;
        }
            [[fallthrough]];
        case HYRES_EPI_BIAS: {
            if (e.bias) { const float4 b = ld4(e.bias + n); o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w; }
            if (e.res) {  // rpre: the residual already loaded by the caller (same value, same order; passed by value:
                          // a pointer into the caller's register array put that array in scratch memory)
                const float4 r = use_pre ? rpre : ldv4<H>(e.res, pix * e.ldres + n);
                o[0] += r.x; o[1] += r.y; o[2] += r.z; o[3] += r.w;
            }
            if (e.out2) stv4<H>(e.out2, pix * e.ldo2 + n, make_float4(o[0], o[1], o[2], o[3]));
            if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
            } else if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                for (int c = 0; c < 4; ++c) o[c] = o[c] >= 0.f ? o[c] : slope * o[c];
            } else if (e.act == HYRES_ACT_RELU_MASK) {
                const float4 y = ld_aux4<H>(e, e.aux0, pix * e.ld0 + n);
                o[0] = y.x > 0.f ? o[0] : 0.f;
                o[1] = y.y > 0.f ? o[1] : 0.f;
                o[2] = y.z > 0.f ? o[2] : 0.f;
                o[3] = y.w > 0.f ? o[3] : 0.f;
            }
            break;
        }
        case HYRES_EPI_GDN:
        case HYRES_EPI_IGDN: {
            const float4 b = e.bias ? ld4(e.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 x = ldv4<H>(e.aux0, pix * e.ld0 + n);
            const float nv[4] = {o[0] + b.x, o[1] + b.y, o[2] + b.z, o[3] + b.w};
            const float xv[4] = {x.x, x.y, x.z, x.w};
            stv4<H>(e.out2, pix * e.ldo2 + n, make_float4(nv[0], nv[1], nv[2], nv[3]));
#pragma unroll
            for (int c = 0; c < 4; ++c)
                o[c] = (e.kind == HYRES_EPI_GDN) ? xv[c] * (1.0f / sqrtf(nv[c])) : xv[c] * sqrtf(nv[c]);
            break;
        }
        case HYRES_EPI_SA_BWD: {  // as in epi_store: (acc + d mean / C) + (channel == argmax ? d max : 0)
            if constexpr (SAB) {
                const float* gm = e.aux0 + pix * e.ld0;
                const float ga = gm[0], gx = gm[1];
                const int mi = reinterpret_cast<const int*>(e.aux2)[pix];
#pragma unroll
                for (int c = 0; c < 4; ++c) o[c] = o[c] + ga + (n + c == mi ? gx : 0.f);
            }
            break;
        }
        case HYRES_EPI_GDN_BWD:
        case HYRES_EPI_IGDN_BWD: {
            const float4 x = ld_aux4<H>(e, e.aux0, pix * e.ld0 + n);
            const float4 gg = ldv4<H>(e.aux1, pix * e.ld1 + n);
            const float4 nn = ld_aux4<H>(e, e.aux2, pix * e.ld2 + n);
            const float xv[4] = {x.x, x.y, x.z, x.w}, gv[4] = {gg.x, gg.y, gg.z, gg.w}, nv[4] = {nn.x, nn.y, nn.z, nn.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float f = (e.kind == HYRES_EPI_GDN_BWD) ? (1.0f / sqrtf(nv[c])) : sqrtf(nv[c]);
                o[c] = 2.0f * xv[c] * o[c] + gv[c] * f;
            }
            break;
        }
        default: break;
    }
    if constexpr (H) {
        if (e.accumulate) {
            const float4 p = ldv4<true>(y, pix * ldy + n);
            o[0] += p.x; o[1] += p.y; o[2] += p.z; o[3] += p.w;
        }
        stv4<true>(y, pix * ldy + n, make_float4(o[0], o[1], o[2], o[3]));
    } else {
        float* yp = y + pix * ldy + n;
        if (e.accumulate) {
            const float4 p = ld4(yp);
            o[0] += p.x; o[1] += p.y; o[2] += p.z; o[3] += p.w;
        }
        st4(yp, make_float4(o[0], o[1], o[2], o[3]));
    }
}

// bf16x8_t / bf16x4_t, bf6_split4, bf6_mfma: conv_common.h (shared with the bf16x6 weight gradients)

template <int TM, int TN, int WAVES_M, int WAVES_N, int MODE, bool SPLITK, bool F16, int IO, bool B6 = false,
          bool DB = false>
__device__ __forceinline__ void conv_fwd_body(const ConvArgs& a) {
    // MODE 0: Ci % 32 == 0 (float4 loads); 1: same + square A (GDN); 2: generic scalar (small Ci).
    // F16: operands rounded to fp16 when staged into LDS ([row][32 halves], pitch PADH halves) and
    // consumed by v_mfma_f32_32x32x16_f16 (lane r,h holds row r, k = 8h..8h+7), fp32 accumulation.
    // IO (fp16 activations in HBM, autocast inference): bit 0 X is fp16 (8-byte loads of 4 channels),
    // bit 1 Y / res / aux0 / out2 are fp16; arithmetic stays fp32 (F16: fp16 MFMA operands as before).
    // B6: fp32 operands split into three bf16 planes when staged ([plane][row][32], pitch PADH), products to fp32
    // accuracy on v_mfma_f32_32x32x16_bf16 (bf6_mfma; hyres_conv_tuning key 7, conv3x3_wres_bf6_kernel's numerics)
    static_assert(!F16 || MODE != 2, "fp16 operands on the Ci % 32 == 0 paths only");
    static_assert(!B6 || (!F16 && IO == 0 && MODE != 2), "bf16x6: fp32 operands on the vector path");
    static_assert(!(IO & 1) || MODE != 2, "fp16 X on the Ci % 32 == 0 paths only");
    // DB (round 6, bf16x6 only): two LDS buffers of swizzled 64-B rows, one barrier per K chunk — chunk k + 1 is split
    // and stored into the other buffer right after chunk k's MFMAs, while other waves may still read chunk k
    static_assert(!DB || B6, "double-buffered staging: the bf16x6 path");
    constexpr bool XH = (IO & 1) != 0, YH = (IO & 2) != 0;
    constexpr int XES = XH ? 2 : 4;  // X element bytes
    constexpr int PADH = 40;
    constexpr int BM = 32 * TM * WAVES_M;
    constexpr int BN = 32 * TN * WAVES_N;
    constexpr int SOP = DB ? 2 * 3 * (BM + BN) * 32 / 2 : B6 ? 3 * (BM + BN) * PADH / 2 : (BM + BN) * PADK;  // staging (floats)
    constexpr int SMEM = (SOP > BM * (32 * WAVES_N + 8)) ? SOP : BM * (32 * WAVES_N + 8);
    __shared__ __attribute__((aligned(16))) float smem[SMEM];
    float* const As = smem;
    float* const Bs = smem + BM * PADK;
    _Float16* const Ah = reinterpret_cast<_Float16*>(smem);
    _Float16* const Bh = Ah + BM * PADH;
    __bf16* const Pb0 = reinterpret_cast<__bf16*>(smem);  // B6: plane p = Pb0 + p * PLANE, A rows then B (DB: + buffer)
    // B6 row layout (round 6): b6sw = 1 (default) 32-half rows, 16-B slot s of row r stored at slot s ^ ((r >> 2) & 3):
    // the split stores (ds_write_b64, 16-lane groups = two consecutive rows, banks mod 32) then fill complementary
    // halves of the 32 banks, and every ds_read_b128 lane group (16 rows, banks mod 64) meets 16 distinct slots.
    // b6sw = 0: the 40-half padded rows (reads conflict-free, the stores 2-way: SQ_LDS_BANK_CONFLICT 0.33 of the LDS
    // cycles at 32^2, profiles/r6f_pmc_families.txt). Same products in the same order either way.
    const int b6p = (DB || (B6 && a.b6sw)) ? 32 : PADH;
    const int PLANE = (BM + BN) * b6p;

    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    const int nsplit = SPLITK ? a.nsplit : 1;
    const int phase = blockIdx.z / nsplit;
    const int split = blockIdx.z - phase * nsplit;
    // XCD-aware tile order (a.xcd): hardware block b runs on XCD b % 8, so XCD x gets the contiguous
    // logical range [x*q + min(x, r), ...) of the nb = q*8 + r tiles (a bijection for any nb); within
    // it the N tiles of one M tile are adjacent. Neighbouring pixel tiles (the 3x3/5x5 halo rows) and
    // the N tiles sharing an A tile then hit one L2 instead of being spread over all eight.
    int m0, n0;
    if (a.xcd) {
        const int nb = gridDim.x, hw = blockIdx.x;
        const int q = nb >> 3, r = nb & 7, x = hw & 7;
        const int l = x * q + min(x, r) + (hw >> 3);
        const int ntn = (g.Co + BN - 1) / BN;
        m0 = (l / ntn) * BM;
        n0 = (l - (l / ntn) * ntn) * BN;
    } else {
        m0 = blockIdx.x * BM;
        n0 = blockIdx.y * BN;
    }
    const int HqWq = g.Hq * g.Wq;
    const int ntap = g.ntap[phase];
    const int tap0 = g.tap0[phase];
    const int Ci = g.Ci;

    constexpr int A_V = (MODE == 2) ? (BM * KT / 256) : (BM / 32);
    constexpr int B_V = (MODE == 2) ? (BN * KT / 256) : (BN / 32);

    // ---- per-thread A rows (pixel decode once)
    int a_b[A_V], a_i[A_V], a_j[A_V];
    bool a_ok[A_V];
#pragma unroll
    for (int q = 0; q < A_V; ++q) {
        int row = (MODE == 2) ? ((tid + 256 * q) / KT) : (tid / 8 + 32 * q);
        int m = m0 + row;
        a_ok[q] = m < a.M;
        int mm = a_ok[q] ? m : 0;
        a_b[q] = mm / HqWq;
        int r = mm - a_b[q] * HqWq;
        a_i[q] = r / g.Wq;
        a_j[q] = r - a_i[q] * g.Wq;
    }
    const int c4 = tid & 7;

    int nk;
    if constexpr (MODE == 2) nk = (ntap * Ci + KT - 1) / KT;
    else nk = ntap * (Ci / KT);

    float4 ra[MODE == 2 || XH ? 1 : A_V], rb[MODE == 2 ? 1 : B_V];
    // fp16 X: the raw halves stay in registers until the LDS store (converting at the load would make the
    // prefetch of the next chunk wait for its data before this chunk's MFMAs)
    half4_t rah[XH ? A_V : 1];
    float sa[MODE == 2 ? A_V : 1], sb[MODE == 2 ? B_V : 1];
    static_assert(!XH || F16, "fp16 X is staged for the f16 MFMA");

    // vector path: raw buffer loads (out-of-range offset -> 0, no branches). The X resource starts at
    // the block's first image so 32-bit byte offsets suffice (host checks 3 images < 2 GB).
    const int b0 = m0 / HqWq;
    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const long long xrem = ((long long)g.B - b0) * img * XES;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(a.x) + (long long)b0 * img * XES), (short)0,
        (int)(xrem < 0x7FFFFFF0LL ? xrem : 0x7FFFFFF0LL), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, a.w_bytes, 0x00020000);
    int a_base[A_V];  // element offset of image row 0 of this row's image, rel. to b0
#pragma unroll
    for (int q = 0; q < A_V; ++q) {
        a_base[q] = (int)((a_b[q] - b0) * img);
        a_i[q] *= g.ish;
        a_j[q] *= g.isw;
    }
    // tap offsets of this phase in LDS (uniform broadcast reads instead of indexed kernarg loads)
    __shared__ int2 tapoff[HYRES_MAX_TAPS];
    for (int i = tid; i < ntap; i += 256) tapoff[i] = make_int2(g.dh[tap0 + i], g.dw[tap0 + i]);
    __syncthreads();
    // (tap, channel) of the next chunk to load, advanced incrementally (no division per chunk)
    int ld_t = 0, ld_c = 0;

    auto load_chunk = [&](int kc) {
        if constexpr (MODE != 2) {
            const int2 o = tapoff[ld_t];
            const int c0 = ld_c + 4 * c4;
            const int gt = tap0 + ld_t;
#pragma unroll
            for (int q = 0; q < A_V; ++q) {
                const int ih = a_i[q] + o.x, iw = a_j[q] + o.y;
                const bool ok = a_ok[q] && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
                const int off = ok ? (a_base[q] + (ih * g.Wi + iw) * g.ldx + c0) * XES : (int)0x80000000;
                if constexpr (XH) {
                    rah[q] = __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
                } else {
                    float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
                    if constexpr (MODE == 1) { v.x *= v.x; v.y *= v.y; v.z *= v.z; v.w *= v.w; }
                    ra[q] = v;
                }
            }
#pragma unroll
            for (int q = 0; q < B_V; ++q) {
                const int co = n0 + tid / 8 + 32 * q;
                const int off = co < g.Co ? (co * a.ldw + gt * Ci + c0) * 4 : (int)0x80000000;
                rb[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
            }
            ld_c += KT;
            if (ld_c == Ci) { ld_c = 0; ++ld_t; }
        } else {
            // generic K = ntap*Ci (small Ci): a thread's k is the same for all its rows (256 % KT == 0),
            // so the (tap, channel) decode happens once per chunk; branch-free raw buffer loads
            const int K = ntap * Ci;
            const int k = kc * KT + (tid % KT);
            const bool kok = k < K;
            const int t = kok ? k / Ci : 0;
            const int ci = k - t * Ci;
            const int2 o = tapoff[t];
#pragma unroll
            for (int q = 0; q < A_V; ++q) {
                const int ih = a_i[q] + o.x, iw = a_j[q] + o.y;
                const bool okq = kok && a_ok[q] && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
                const int off = okq ? (a_base[q] + (ih * g.Wi + iw) * g.ldx + ci) * 4 : (int)0x80000000;
                sa[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
            }
#pragma unroll
            for (int q = 0; q < B_V; ++q) {
                const int co = n0 + (tid + 256 * q) / KT;
                const int off = (co < g.Co && kok) ? (co * a.ldw + tap0 * Ci + k) * 4 : (int)0x80000000;
                sb[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, off, 0, 0));
            }
        }
    };
    auto store_chunk = [&](int buf = 0) {
        if constexpr (B6) {
            __bf16* const Pb = Pb0 + buf * 3 * PLANE;
            const int sx = b6p == 32 ? (((c4 >> 1) ^ ((tid >> 5) & 3)) << 3) + 4 * (c4 & 1) : 4 * c4;  // row bits 2..3 = tid bits 5..6
#pragma unroll
            for (int q = 0; q < A_V; ++q) {
                bf16x4_t h, m, l;
                bf6_split4(ra[q], h, m, l);
                const int o = (tid / 8 + 32 * q) * b6p + sx;
                *reinterpret_cast<bf16x4_t*>(&Pb[o]) = h;
                *reinterpret_cast<bf16x4_t*>(&Pb[PLANE + o]) = m;
                *reinterpret_cast<bf16x4_t*>(&Pb[2 * PLANE + o]) = l;
            }
#pragma unroll
            for (int q = 0; q < B_V; ++q) {
                bf16x4_t h, m, l;
                bf6_split4(rb[q], h, m, l);
                const int o = (BM + tid / 8 + 32 * q) * b6p + sx;
                *reinterpret_cast<bf16x4_t*>(&Pb[o]) = h;
                *reinterpret_cast<bf16x4_t*>(&Pb[PLANE + o]) = m;
                *reinterpret_cast<bf16x4_t*>(&Pb[2 * PLANE + o]) = l;
            }
        } else if constexpr (F16) {
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int q = 0; q < A_V; ++q) {
                half4 h;
                if constexpr (XH && MODE == 1) {  // GDN norm: x^2 of the fp16 x, rounded for the MFMA
                    const half4_t r = rah[q];
                    const float4 v = make_float4((float)r.x * (float)r.x, (float)r.y * (float)r.y,
                                                 (float)r.z * (float)r.z, (float)r.w * (float)r.w);
                    h = half4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
                } else if constexpr (XH) {
                    h = __builtin_bit_cast(half4, rah[q]);
                } else {
                    h = half4{(_Float16)ra[q].x, (_Float16)ra[q].y, (_Float16)ra[q].z, (_Float16)ra[q].w};
                }
                *reinterpret_cast<half4*>(&Ah[(tid / 8 + 32 * q) * PADH + 4 * c4]) = h;
            }
#pragma unroll
            for (int q = 0; q < B_V; ++q) {
                const half4 h = {(_Float16)rb[q].x, (_Float16)rb[q].y, (_Float16)rb[q].z, (_Float16)rb[q].w};
                *reinterpret_cast<half4*>(&Bh[(tid / 8 + 32 * q) * PADH + 4 * c4]) = h;
            }
        } else if constexpr (MODE != 2) {
#pragma unroll
            for (int q = 0; q < A_V; ++q)
                *reinterpret_cast<float4*>(&As[(tid / 8 + 32 * q) * PADK + 4 * c4]) = ra[q];
#pragma unroll
            for (int q = 0; q < B_V; ++q)
                *reinterpret_cast<float4*>(&Bs[(tid / 8 + 32 * q) * PADK + 4 * c4]) = rb[q];
        } else {
#pragma unroll
            for (int q = 0; q < A_V; ++q) {
                int e = tid + 256 * q;
                As[(e / KT) * PADK + (e % KT)] = sa[q];
            }
#pragma unroll
            for (int q = 0; q < B_V; ++q) {
                int e = tid + 256 * q;
                Bs[(e / KT) * PADK + (e % KT)] = sb[q];
            }
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int lr = lane & 31, lh = lane >> 5;

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int kbeg = SPLITK ? min(nk, split * a.cps) : 0;
    const int kend = SPLITK ? min(nk, kbeg + a.cps) : nk;
    if constexpr (MODE != 2) {
        const int cpt = Ci / KT;
        ld_t = kbeg / cpt;
        ld_c = (kbeg - ld_t * cpt) * KT;
    }
    auto b6_compute = [&](int buf) {
        const __bf16* const Pb = Pb0 + buf * 3 * PLANE;
            if (a.prio) __builtin_amdgcn_s_setprio(1);
            const int rx = b6p == 32 ? (lr >> 2) & 3 : 0;  // the row's slot swizzle (tile bases are multiples of 32 rows)
#pragma unroll
            for (int s16 = 0; s16 < 2; ++s16) {
                bf16x8_t af[TM][3], bf[TN][3];
                const int ko = ((2 * s16 + lh) ^ rx) << 3;
#pragma unroll
                for (int p = 0; p < 3; ++p) {
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
                        af[tm][p] = *reinterpret_cast<const bf16x8_t*>(
                            &Pb[p * PLANE + (wm * TM * 32 + tm * 32 + lr) * b6p + ko]);
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        bf[tn][p] = *reinterpret_cast<const bf16x8_t*>(
                            &Pb[p * PLANE + (BM + wn * TN * 32 + tn * 32 + lr) * b6p + ko]);
                }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = bf6_mfma(af[tm], bf[tn], acc[tm][tn]);
            }
            if (a.prio) __builtin_amdgcn_s_setprio(0);
    };
    if constexpr (DB) {
        if (kbeg < kend) {
            load_chunk(kbeg);
            store_chunk(0);
        }
        __syncthreads();
        int cur = 0;
        for (int kc = kbeg; kc < kend; ++kc) {
            const bool nxt = kc + 1 < kend;  // block-uniform
            if (nxt) load_chunk(kc + 1);
            b6_compute(cur);
            if (nxt) store_chunk(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
    } else {
    if (kbeg < kend) load_chunk(kbeg);
    for (int kc = kbeg; kc < kend; ++kc) {
        __syncthreads();
        store_chunk();
        __syncthreads();
        if (kc + 1 < kend) load_chunk(kc + 1);
        if constexpr (B6) {
            b6_compute(0);
            continue;
        }
        if constexpr (F16) {
            typedef _Float16 half8 __attribute__((ext_vector_type(8)));
            if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s16 = 0; s16 < 2; ++s16) {
                half8 af[TM], bf[TN];
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
                    af[tm] = *reinterpret_cast<const half8*>(
                        &Ah[(wm * TM * 32 + tm * 32 + lr) * PADH + 16 * s16 + 8 * lh]);
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    bf[tn] = *reinterpret_cast<const half8*>(
                        &Bh[(wn * TN * 32 + tn * 32 + lr) * PADH + 16 * s16 + 8 * lh]);
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
            }
            if (a.prio) __builtin_amdgcn_s_setprio(0);
            continue;
        }
        if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float4 af[TM], bf[TN];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
                af[tm] = *reinterpret_cast<const float4*>(
                    &As[(wm * TM * 32 + tm * 32 + lr) * PADK + lh * 16 + 4 * u]);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                bf[tn] = *reinterpret_cast<const float4*>(
                    &Bs[(wn * TN * 32 + tn * 32 + lr) * PADK + lh * 16 + 4 * u]);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) {
                        float av = e == 0 ? af[tm].x : e == 1 ? af[tm].y : e == 2 ? af[tm].z : af[tm].w;
                        float bv = e == 0 ? bf[tn].x : e == 1 ? bf[tn].y : e == 2 ? bf[tn].z : bf[tn].w;
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[tm][tn], 0, 0, 0);
                    }
        }
        if (a.prio) __builtin_amdgcn_s_setprio(0);
    }
    }

    // ---- epilogue: stage the accumulators through LDS one TN column slice at a time (static register
    // indices), then apply the epilogue row-major: consecutive threads cover consecutive channels of
    // one NHWC pixel row (float4 when every operand is 16B aligned), each row decoded once.
    constexpr int CW = 32 * WAVES_N, CP = CW + 8;  // +8: the two lane halves hit disjoint banks
    float* Cs = smem;
    constexpr bool split_k = SPLITK;
    float* slab = split_k ? a.slab + ((long long)(split * g.nphase + phase) * a.M) * g.Co : nullptr;
    const bool linear = g.nphase == 1 && g.osh == 1 && g.osw == 1 && g.Ho == g.Hq && g.Wo == g.Wq;
    const int oph = g.oph[phase], opw = g.opw[phase];
    const float slope = (a.e.act == HYRES_ACT_PRELU) ? a.e.slope[0] : 0.f;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        __syncthreads();
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                Cs[(wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * CP + wn * 32 + lr] = acc[tm][tn][r];
        __syncthreads();
        if constexpr (!split_k) {
            // fast path (BIAS epilogue, float4 operands): the bias / residual / old-y / ReLU-mask loads of U
            // iterations are issued before any of them is consumed. Per-lane validity goes into the buffer offset
            // (out of range -> 0, no divergent branch: a load behind one is waited on where the branches join);
            // an absent operand is skipped by a uniform branch around all U of its loads
            if (a.vec4 && a.rsrc_ok && a.e.kind == HYRES_EPI_BIAS) {
                constexpr int ITER = BM * (CW / 4) / 256;
                constexpr int U = ITER >= 4 ? 4 : ITER;
                static_assert(ITER % U == 0, "epilogue tiling");
                const hyres_epilogue& e = a.e;
                constexpr int ES = YH ? 2 : 4;  // residual / fp16-storage element bytes
                const long long npo = (long long)g.B * g.Ho * g.Wo;
                const bool mask = e.act == HYRES_ACT_RELU_MASK;
                const bool m16 = YH || (e.io_f16 & HYRES_IO_AUX16);
                const __amdgpu_buffer_rsrc_t r_bias = opnd_rsrc(e.bias, (long long)g.Co * 4);
                const __amdgpu_buffer_rsrc_t r_res = opnd_rsrc(e.res, npo * e.ldres * ES);
                const __amdgpu_buffer_rsrc_t r_m32 = opnd_rsrc(mask && !m16 ? e.aux0 : nullptr, npo * e.ld0 * 4);
                const __amdgpu_buffer_rsrc_t r_m16 = opnd_rsrc(mask && m16 ? e.aux0 : nullptr, npo * e.ld0 * 2);
                const __amdgpu_buffer_rsrc_t r_old = opnd_rsrc(e.accumulate ? a.y : nullptr, npo * g.ldy * ES);
                constexpr int OOR = (int)0x80000000;
                for (int it0 = 0; it0 < ITER; it0 += U) {
                    float4 v[U], yo[U], mk[U], bs[U];
                    std::conditional_t<YH, half4_t, float4> rs[U];
                    half4_t mh[U];
                    long long px[U];
                    int nn[U];
                    bool ok[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int idx = tid + 256 * (it0 + u);
                        const int row = idx / (CW / 4);
                        const int col = 4 * (idx - row * (CW / 4));
                        const int m = m0 + row;
                        const int n = n0 + (col >> 5) * TN * 32 + tn * 32 + (col & 31);
                        ok[u] = m < a.M && n < g.Co;
                        nn[u] = n;
                        v[u] = *reinterpret_cast<const float4*>(&Cs[row * CP + col]);
                        long long pix = m;
                        if (!linear) {
                            const int b = m / HqWq;
                            const int rr = m - b * HqWq;
                            const int i = rr / g.Wq;
                            const int j = rr - i * g.Wq;
                            pix = (long long)(b * g.Ho + i * g.osh + oph) * g.Wo + j * g.osw + opw;
                        }
                        px[u] = pix;
                    }
                    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int u = 0; u < U; ++u) { bs[u] = z4; yo[u] = z4; mk[u] = z4; }
                    if (e.bias) {
#pragma unroll
                        for (int u = 0; u < U; ++u) bs[u] = bload4(r_bias, ok[u] ? nn[u] * 4 : OOR);
                    }
                    if (e.res) {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int orr = ok[u] ? (int)((px[u] * e.ldres + nn[u]) * ES) : OOR;
                            if constexpr (YH) rs[u] = bload4h(r_res, orr);
                            else rs[u] = bload4(r_res, orr);
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            if constexpr (YH) rs[u] = half4_t{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
                            else rs[u] = z4;
                        }
                    }
                    if (e.accumulate) {  // YH: fp16 gradient accumulation (AMP)
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int oo = ok[u] ? (int)((px[u] * g.ldy + nn[u]) * ES) : OOR;
                            if constexpr (YH) yo[u] = h2f4(bload4h(r_old, oo));
                            else yo[u] = bload4(r_old, oo);
                        }
                    }
                    if (mask && m16) {
#pragma unroll
                        for (int u = 0; u < U; ++u) mh[u] = bload4h(r_m16, ok[u] ? (int)((px[u] * e.ld0 + nn[u]) * 2) : OOR);
                    } else if (mask) {
#pragma unroll
                        for (int u = 0; u < U; ++u) mk[u] = bload4(r_m32, ok[u] ? (int)((px[u] * e.ld0 + nn[u]) * 4) : OOR);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (!ok[u]) continue;
                        float4 r4;
                        if constexpr (YH) r4 = h2f4(rs[u]);
                        else r4 = rs[u];
                        float o[4] = {v[u].x + bs[u].x + r4.x, v[u].y + bs[u].y + r4.y,
                                      v[u].z + bs[u].z + r4.z, v[u].w + bs[u].w + r4.w};
                        if (e.out2) stv4<YH>(e.out2, px[u] * e.ldo2 + nn[u], make_float4(o[0], o[1], o[2], o[3]));
                        if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
                        } else if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) o[c] = o[c] >= 0.f ? o[c] : slope * o[c];
                        } else if (mask) {
                            const float4 q = m16 ? h2f4(mh[u]) : mk[u];
                            o[0] = q.x > 0.f ? o[0] : 0.f;
                            o[1] = q.y > 0.f ? o[1] : 0.f;
                            o[2] = q.z > 0.f ? o[2] : 0.f;
                            o[3] = q.w > 0.f ? o[3] : 0.f;
                        }
                        stv4<YH>(a.y, px[u] * g.ldy + nn[u],
                                 make_float4(o[0] + yo[u].x, o[1] + yo[u].y, o[2] + yo[u].z, o[3] + yo[u].w));
                    }
                }
                continue;
            }
        }
        for (int idx = tid; idx < BM * (CW / 4); idx += 256) {
            const int row = idx / (CW / 4);
            const int col = 4 * (idx - row * (CW / 4));
            const int m = m0 + row;
            const int n = n0 + (col >> 5) * TN * 32 + tn * 32 + (col & 31);
            if (m >= a.M || n >= g.Co) continue;
            const float4 v = *reinterpret_cast<const float4*>(&Cs[row * CP + col]);
            if constexpr (split_k) {
                float* sp = slab + (long long)m * g.Co + n;
                if (a.vec4) {
                    *reinterpret_cast<float4*>(sp) = v;
                } else {
                    sp[0] = v.x;
                    if (n + 1 < g.Co) sp[1] = v.y;
                    if (n + 2 < g.Co) sp[2] = v.z;
                    if (n + 3 < g.Co) sp[3] = v.w;
                }
                continue;
            }
            long long pix = m;
            if (!linear) {
                const int b = m / HqWq;
                const int rr = m - b * HqWq;
                const int i = rr / g.Wq;
                const int j = rr - i * g.Wq;
                pix = (long long)(b * g.Ho + i * g.osh + oph) * g.Wo + j * g.osw + opw;
            }
            if (a.vec4) {
                epi_store4<YH, true>(a.e, a.y, g.ldy, pix, n, v, slope);
            } else {
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (n + c < g.Co) epi_store<YH, true>(a.e, a.y, g.ldy, pix, n + c, vv[c], epi_channel(a.e, n + c));
            }
        }
    }
}

// waves per SIMD the register allocation must allow: 4 (<= 128 VGPRs: 4 blocks per CU) for the vector-load tiles with
// at most two accumulator tiles per wave — left to itself the compiler gave the 64x128 / 128x64 tiles 144 registers
// (3 blocks per CU); with the bound they fit in 109-127 with no spill — and 3 (<= 168) for the 128x128 tiles (176-212
// -> 142-154, 3 blocks per CU instead of 2; AMP step -0.5 %, fp32 neutral: profiles/r3aa_conv_wpe3_ab.txt). The
// scalar-load path (MODE 2, the 3-channel image side) would spill: the compiler's choice there. -DHYRES_CONV_WPE4=0
// builds the unbounded variant (A/B).
#ifndef HYRES_CONV_WPE4
#define HYRES_CONV_WPE4 1
#endif
template <int TM, int TN, int MODE>
constexpr int conv_wpe() { return (HYRES_CONV_WPE4 && MODE != 2) ? (TM * TN <= 2 ? 4 : 3) : 1; }

template <int TM, int TN, int WAVES_M, int WAVES_N, int MODE, bool SPLITK, bool F16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(conv_wpe<TM, TN, MODE>())))
void conv_fwd_kernel(const ConvArgs a) {
    conv_fwd_body<TM, TN, WAVES_M, WAVES_N, MODE, SPLITK, F16, 0>(a);
}

// fp32 operands, bf16x6 products (hyres_conv_tuning key 7): the compiler's register allocation (the three-plane
// fragments do not fit the 4-waves-per-SIMD bound of conv_fwd_kernel)
template <int TM, int TN, int WAVES_M, int WAVES_N, int MODE, bool SPLITK>
__global__ __launch_bounds__(256) void conv_fwd_b6_kernel(const ConvArgs a) {
    conv_fwd_body<TM, TN, WAVES_M, WAVES_N, MODE, SPLITK, false, 0, true>(a);
}
// the same with double-buffered staging (conv_fwd_body DB; round 6, the 64x64 tile only: hyres_conv_tuning key 20)
template <int TM, int TN, int WAVES_M, int WAVES_N, int MODE, bool SPLITK>
__global__ __launch_bounds__(256) void conv_fwd_b6db_kernel(const ConvArgs a) {
    conv_fwd_body<TM, TN, WAVES_M, WAVES_N, MODE, SPLITK, false, 0, true, true>(a);
}

// fp16 activations in HBM (IO = 1: X fp16, 2: Y fp16, 3: both); fp16 MFMA operands except on the
// small-Ci scalar path (MODE 2: the fp32 image in, fp16 features out)
template <int TM, int TN, int WAVES_M, int WAVES_N, int MODE, bool SPLITK, int IO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(conv_wpe<TM, TN, MODE>())))
void conv_fwd_h_kernel(const ConvArgs a) {
    conv_fwd_body<TM, TN, WAVES_M, WAVES_N, MODE, SPLITK, MODE != 2, IO>(a);
}

// ------------------------------------------------------------------------------------------------
// Halo-staged f16 3x3 conv (autocast; the dominant AMP kernel).  The implicit-GEMM kernel above gathers the
// A operand once per tap from L2: for a 3x3 64->64 layer at 128^2 that is ~1 GB of L2->CU traffic per launch
// (PMC: TCC hits+misses ~7.9 M requests, 84 % hit) for 134 MB of HBM traffic, and its one-chunk register
// prefetch cannot cover that latency with the 4 f16 MFMAs a 32-deep chunk gives each wave (SQ_WAIT_ANY 48 %
// of wave-cycles).  Here a block computes a 4-row x 64-pixel x 64-channel output tile: the 6 x 66-pixel
// input halo of one 32-channel chunk is staged ONCE in LDS as fp16 (2 buffers: the next chunk's halo loads
// are issued in three parts between the taps of the current chunk), and all 9 taps read their A fragments
// from it (ds_read_b128, 80-B pixel pitch: conflict-free); the B fragments (weights, fp32 W2 converted in
// registers) come straight from L2 in MFMA layout, one tap ahead.  L2->CU bytes per output pixel drop from
// ~3.4 KB to ~1.5 KB.  Taps: any 9 offsets within [-1, 1]^2 (the conv and its input-gradient), stride 1,
// same-size output, Ci % 32 == 0, Co % 64 == 0, Wo % 64 == 0.  IO: bit 0 X fp16, bit 1 Y/res/aux fp16.
constexpr int HALO_R = 4, HALO_TW = 64, HALO_HR = HALO_R + 2, HALO_HW = HALO_TW + 2;
constexpr int HALO_NPX = HALO_HR * HALO_HW;  // 396 halo pixels
constexpr int HALO_PH = 40;                   // halves per staged pixel (32 channels + 8 pad: 80-B pitch)
constexpr int HALO_E = HALO_NPX * 8;          // float4 elements of one 32-channel halo chunk
constexpr int HALO_PE = (HALO_E + 2) / 3;     // per staging part (3 parts per chunk)
constexpr int HALO_PV = (HALO_PE + 255) / 256;

template <int IO>
__global__ __launch_bounds__(256, 2) void conv3x3_halo_f16_kernel(const ConvArgs a) {
    constexpr bool XH = (IO & 1) != 0, YH = (IO & 2) != 0;
    constexpr int XES = XH ? 2 : 4;
    constexpr int HBUF = HALO_NPX * HALO_PH;  // halves per buffer
    constexpr int CP = 64 + 4;                // epilogue staging pitch (floats)
    static_assert(2 * 64 * CP * 4 <= 2 * HBUF * 2, "epilogue staging fits in the halo buffers");
    __shared__ __attribute__((aligned(16))) _Float16 hal[2 * HBUF];
    __shared__ int2 tapoff[9];
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));

    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    // tile decode, XCD-aware (conv_fwd_body): N tiles fastest, then row tiles (vertical neighbours share
    // two of the six halo rows through one L2), column tiles, images
    const int nnt = g.Co / 64, nrt = (g.Ho + HALO_R - 1) / HALO_R, nct = g.Wo / HALO_TW;
    int l;
    {
        const int nb = gridDim.x, hw = blockIdx.x;
        const int q = nb >> 3, r = nb & 7, x = hw & 7;
        l = x * q + min(x, r) + (hw >> 3);
    }
    const int nt = l % nnt; l /= nnt;
    const int rt = l % nrt; l /= nrt;
    const int ct = l % nct;
    const int b = l / nct;
    const int n0 = nt * 64, i0 = rt * HALO_R, j0 = ct * HALO_TW;
    const int Ci = g.Ci, nch = Ci / 32;
    if (tid < 9) tapoff[tid] = make_int2(g.dh[tid], g.dw[tid]);

    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const long long xrem = img * XES;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(a.x) + (long long)b * img * XES), (short)0,
        (int)(xrem < 0x7FFFFFF0LL ? xrem : 0x7FFFFFF0LL), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, a.w_bytes, 0x00020000);

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;  // rows 2wm, 2wm+1; channels n0 + 32wn ..
    const int lr = lane & 31, lh = lane >> 5;

    // ---- halo staging (part p of chunk c: elements [p*PE, (p+1)*PE) of the 396 px x 8 float4)
    std::conditional_t<XH, half4_t, float4> hreg[HALO_PV];  // fp16 X: raw halves until the LDS store
    auto hload = [&](int part, int c) {
        const int ci0 = c * 32;
#pragma unroll
        for (int q = 0; q < HALO_PV; ++q) {
            const int e = part * HALO_PE + tid + 256 * q;
            const int px = e >> 3, c4 = e & 7;
            const int hr = px / HALO_HW, hc = px - hr * HALO_HW;
            const int ih = i0 - 1 + hr, iw = j0 - 1 + hc;
            const bool ok = e < (part + 1) * HALO_PE && e < HALO_E && (unsigned)ih < (unsigned)g.Hi &&
                            (unsigned)iw < (unsigned)g.Wi;
            const int off = ok ? ((ih * g.Wi + iw) * g.ldx + ci0 + 4 * c4) * XES : (int)0x80000000;
            if constexpr (XH) {
                hreg[q] = __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
            } else {
                hreg[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            }
        }
    };
    auto hstore = [&](int part, int buf) {
#pragma unroll
        for (int q = 0; q < HALO_PV; ++q) {
            const int e = part * HALO_PE + tid + 256 * q;
            if (e < (part + 1) * HALO_PE && e < HALO_E) {
                const int px = e >> 3, c4 = e & 7;
                half4_t h;
                if constexpr (XH) h = hreg[q];
                else h = half4_t{(_Float16)hreg[q].x, (_Float16)hreg[q].y, (_Float16)hreg[q].z, (_Float16)hreg[q].w};
                *reinterpret_cast<half4_t*>(&hal[buf * HBUF + px * HALO_PH + 4 * c4]) = h;
            }
        }
    };
    // ---- B fragments of one tap (both 16-deep k-steps of the chunk): W2[co][t][ci], fp32 -> fp16
    const int co = n0 + wn * 32 + lr;
    float4 bnx[4];
    auto bload = [&](int t, int c) {
        const int base = (co * a.ldw + t * Ci + c * 32 + 8 * lh) * 4;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bnx[2 * ks] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, base + 64 * ks, 0, 0));
            bnx[2 * ks + 1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wr, base + 64 * ks + 16, 0, 0));
        }
    };

    floatx16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

#pragma unroll
    for (int part = 0; part < 3; ++part) {
        hload(part, 0);
        hstore(part, 0);
    }
    bload(0, 0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        const _Float16* H = hal + (c & 1) * HBUF;
        const bool more = c + 1 < nch;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            half8 bf[2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const float4 u = bnx[2 * ks], v = bnx[2 * ks + 1];
                bf[ks] = half8{(_Float16)u.x, (_Float16)u.y, (_Float16)u.z, (_Float16)u.w,
                               (_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
            }
            if (t < 8) bload(t + 1, c);
            else if (more) bload(0, c + 1);
            if (more && t % 3 == 0) hload(t / 3, c + 1);
            const int2 o = tapoff[t];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                for (int at = 0; at < 4; ++at) {
                    const int orow = 2 * wm + (at >> 1);  // output row within the tile
                    const int px = (orow + 1 + o.x) * HALO_HW + (at & 1) * 32 + lr + 1 + o.y;
                    const half8 af = *reinterpret_cast<const half8*>(&H[px * HALO_PH + 16 * ks + 8 * lh]);
                    acc[at] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[ks], acc[at], 0, 0, 0);
                }
            }
            if (more && t % 3 == 2) hstore(t / 3, (c + 1) & 1);
        }
        __syncthreads();
    }

    // ---- epilogue in two passes of 2 output rows (rows p and 2 + p), staged through the halo buffers
    float* Cs = reinterpret_cast<float*>(hal);
    const float slope = (a.e.act == HYRES_ACT_PRELU) ? a.e.slope[0] : 0.f;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        if (p) __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                Cs[(wm * 64 + h * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * CP + wn * 32 + lr] = acc[2 * p + h][r];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int idx = tid + 256 * k;
            const int c4 = idx & 15, px = (idx >> 4) & 63, rr = idx >> 10;
            const int i = i0 + 2 * rr + p, j = j0 + px;
            if (i < g.Ho) {
                const float4 v = *reinterpret_cast<const float4*>(&Cs[(rr * 64 + px) * CP + 4 * c4]);
                const long long pix = ((long long)b * g.Ho + i) * g.Wo + j;
                epi_store4<YH>(a.e, a.y, g.ldy, pix, n0 + 4 * c4, v, slope);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Weight-resident persistent f16 3x3 conv, Ci = 64 (the 64-channel 3x3 convs of every ResidualUnit / RBB
// / MultiScaleRefine scale at 64^2..256^2, forward and input-gradient).  conv3x3_halo_f16_kernel above still
// re-reads the B operand (all 576 x 64 weights, fp32) from L2 once per wave and 256-pixel tile: 147 KB per
// 32-channel chunk per block against 51 KB of halo, ~400 GB/s per CU of L2->CU traffic, 2-3x what a CU gets
// from L2 (MI355X_MICROARCH.md "Indexed rows": 66-73 GB/s per CU from L2) — so it measured no faster than the
// implicit-GEMM kernel.  Here one 512-thread block per CU converts the layer's weights of its 64-channel
// output slice to fp16 ONCE into LDS (9 taps x 64 co x 64 ci, 80-B rows: 92 KB) and then walks its share of
// the 4-row x 64-pixel tiles; per tile and 32-channel chunk only the 6 x 66-pixel halo moves (fp32 -> fp16,
// 7 float4 per thread issued one chunk ahead, 2 LDS buffers: 63 KB), and every A and B fragment is a
// conflict-free ds_read_b128.  Per CU that is ~22 B per cycle at the MFMA rate, below the L2 rate; the
// epilogue is applied from the accumulators directly (per-lane scalar epi_store: the LDS is full).
// 8 waves = 4 output rows x 2 co halves, 2 A tiles (64 px) each; tiles are walked XCD-contiguously.
constexpr int WRES_LDS_B = 2 * 9 * 64 * HALO_PH;  // halves: [chunk][tap][co][40]
constexpr int WRES_HV = (HALO_E + 511) / 512;     // halo float4 per thread per chunk (7)

template <int IO>
__global__ __launch_bounds__(512, 2) void conv3x3_wres_f16_kernel(const ConvArgs a, int ntiles, int groups) {
    constexpr bool XH = (IO & 1) != 0, YH = (IO & 2) != 0;
    constexpr int XES = XH ? 2 : 4;
    constexpr int HBUF = HALO_NPX * HALO_PH;
    __shared__ __attribute__((aligned(16))) _Float16 lds[WRES_LDS_B + 2 * HBUF];
    __shared__ int2 tapoff[9];
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    _Float16* const Bs = lds;
    _Float16* const Hs = lds + WRES_LDS_B;
    // whole VGPR file (as conv3x3_wres_bf6_kernel, DESIGN §4 "Cross-kernel interference"): IO 1 allocated 248 and left
    // a 16-VGPR hole beside its two waves per SIMD; the others already allocate 256 (and the clobber made IO 3 spill)
    if constexpr (IO == 1) asm volatile("" ::: "v255");

    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    const int nrt = (g.Ho + HALO_R - 1) / HALO_R, nct = g.Wo / HALO_TW;
    // block -> (output-channel group, share of the tiles): the blocks of one XCD (b % 8) take one contiguous
    // range of tiles, interleaved, so that vertically adjacent tiles (two shared halo rows) run together on it
    // group-major block order with nb % 8 == 0 (wres_blocks): hardware XCD = blockIdx.x % 8 = bg % 8, so the
    // blocks of every channel group that walk the same tiles (same bg) sit on one XCD and share its L2 halos
    const int nb = gridDim.x / groups;  // blocks per channel group
    const int grp = blockIdx.x / nb, bg = blockIdx.x - grp * nb;
    const int n0 = grp * 64;
    const int xcd = bg & 7, nx = (nb + 7 - xcd) >> 3, jx = bg >> 3;  // blocks of this XCD, index among them
    const int q = ntiles >> 3, rr8 = ntiles & 7;
    const int tbeg = xcd * q + min(xcd, rr8), tcnt = q + (xcd < rr8 ? 1 : 0);
    const int mytiles = jx < tcnt ? (tcnt - 1 - jx) / nx + 1 : 0;
    if (tid < 9) tapoff[tid] = make_int2(g.dh[tid], g.dw[tid]);

    // ---- the 64-channel weight slice, fp32 W2[co][t][ci] -> fp16 Bs[(c*9 + t)*64 + co][k] (ci = 32c + k)
    for (int f = tid; f < 64 * 9 * 16; f += 512) {
        const int co = f / 144, rem = f - co * 144, t = rem >> 4, ci = 4 * (rem & 15);
        const float4 w = ld4(a.w2 + (long long)(n0 + co) * a.ldw + t * 64 + ci);
        const half4_t h = {(_Float16)w.x, (_Float16)w.y, (_Float16)w.z, (_Float16)w.w};
        *reinterpret_cast<half4_t*>(&Bs[(((ci >> 5) * 9 + t) * 64 + co) * HALO_PH + (ci & 31)]) = h;
    }

    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, (short)0, (int)std::min<long long>((long long)g.B * img * XES, 0x7FFFFFF0LL), 0x00020000);
    const int lane = tid & 63, wave = tid >> 6;
    const int orow = wave & 3, wn = wave >> 2;
    const int lr = lane & 31, lh = lane >> 5;

    auto tile_of = [&](int k, int& b, int& i0, int& j0) {
        int l = tbeg + jx + k * nx;
        const int rt = l % nrt; l /= nrt;
        const int ct = l % nct;
        b = l / nct;
        i0 = rt * HALO_R;
        j0 = ct * HALO_TW;
    };
    // halo chunks are prefetched TWO steps ahead (two register sets, alternating): one step of MFMA work
    // (~2.3k cycles per SIMD) does not cover an HBM-bound 50 KB-per-CU chunk load
    using HRT = std::conditional_t<XH, half4_t, float4>;  // fp16 X: raw halves until the LDS store
    auto hload = [&](HRT (&h)[WRES_HV], int step) {
        int b, i0, j0;
        tile_of(step >> 1, b, i0, j0);
        const int c = step & 1;
        const int base = b * (int)img;  // element offset of image b (host checks the batch < 2 GB)
#pragma unroll
        for (int v = 0; v < WRES_HV; ++v) {
            const int e = tid + 512 * v;
            const int px = e >> 3, c4 = e & 7;
            const int hr = px / HALO_HW, hc = px - hr * HALO_HW;
            const int ih = i0 - 1 + hr, iw = j0 - 1 + hc;
            const bool ok = e < HALO_E && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
            const int off = ok ? (base + (ih * g.Wi + iw) * g.ldx + 32 * c + 4 * c4) * XES : (int)0x80000000;
            if constexpr (XH) {
                h[v] = __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
            } else {
                h[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            }
        }
    };
    auto hstore = [&](const HRT (&h)[WRES_HV], int buf) {
#pragma unroll
        for (int v = 0; v < WRES_HV; ++v) {
            const int e = tid + 512 * v;
            if (e < HALO_E) {
                half4_t hh;
                if constexpr (XH) hh = h[v];
                else hh = half4_t{(_Float16)h[v].x, (_Float16)h[v].y, (_Float16)h[v].z, (_Float16)h[v].w};
                *reinterpret_cast<half4_t*>(&Hs[buf * HBUF + (e >> 3) * HALO_PH + 4 * (e & 7)]) = hh;
            }
        }
    };

    // the product is formed transposed (C^T = W X^T, as conv1x1_stream_kernel): lane (lr, lh) of A tile `at`
    // holds pixel j0 + 32 at + lr and, per register quad qd, the 4 consecutive channels n0 + 32 wn + 8 qd + 4 lh
    // .. + 3 — the epilogue loads / stores float4 straight from the accumulators
    floatx16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const float slope = (a.e.act == HYRES_ACT_PRELU) ? a.e.slope[0] : 0.f;
    const bool pre_res = a.e.kind == HYRES_EPI_BIAS && a.e.res != nullptr;
    float4 rres[2][4];  // the tile's residual operand, prefetched one step before the epilogue
    const int steps = mytiles * 2;  // two 32-channel chunks per tile
    auto tile_pix = [&](int k, int at, int& i, long long& pix) {
        int b, i0, j0;
        tile_of(k, b, i0, j0);
        i = i0 + orow;
        pix = ((long long)b * g.Ho + i) * g.Wo + j0 + 32 * at + lr;
    };
    auto body = [&](int s, HRT (&hl)[WRES_HV], const HRT (&hs)[WRES_HV]) {
        const int k = s >> 1, c = s & 1;
        // the epilogue's residual is loaded BEFORE the halo two steps ahead: vmcnt retires loads in issue
        // order, so waiting for it then does not wait for that halo too (the bias comes from LDS for the same
        // reason)
        if (c == 1 && pre_res) {
#pragma unroll
            for (int at = 0; at < 2; ++at) {
                int i;
                long long pix;
                tile_pix(k, at, i, pix);
#pragma unroll
                for (int qd = 0; qd < 4; ++qd)
                    rres[at][qd] = i < g.Ho ? ldv4<YH>(a.e.res, pix * a.e.ldres + n0 + 32 * wn + 8 * qd + 4 * lh)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        if (s + 2 < steps) hload(hl, s + 2);
        const _Float16* H = Hs + (s & 1) * HBUF;
        const _Float16* Bc = Bs + c * 9 * 64 * HALO_PH;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int2 o = tapoff[t];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const half8 bf = *reinterpret_cast<const half8*>(&Bc[(t * 64 + wn * 32 + lr) * HALO_PH + 16 * ks + 8 * lh]);
#pragma unroll
                for (int at = 0; at < 2; ++at) {
                    const int px = (orow + 1 + o.x) * HALO_HW + at * 32 + lr + 1 + o.y;
                    const half8 af = *reinterpret_cast<const half8*>(&H[px * HALO_PH + 16 * ks + 8 * lh]);
                    acc[at] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf, af, acc[at], 0, 0, 0);
                }
            }
        }
        if (c == 1) {
#pragma unroll
            for (int at = 0; at < 2; ++at) {
                int i;
                long long pix;
                tile_pix(k, at, i, pix);
                if (i < g.Ho) {
#pragma unroll
                    for (int qd = 0; qd < 4; ++qd) {
                        const int n = n0 + 32 * wn + 8 * qd + 4 * lh;
                        const float4 v = make_float4(acc[at][4 * qd], acc[at][4 * qd + 1], acc[at][4 * qd + 2],
                                                     acc[at][4 * qd + 3]);
                        epi_store4<YH>(a.e, a.y, g.ldy, pix, n, v, slope, pre_res, rres[at][qd]);
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[at][r] = 0.f;
            }
        }
        if (s + 1 < steps) hstore(hs, (s + 1) & 1);
        __syncthreads();
    };
    HRT hA[WRES_HV], hB[WRES_HV];
    if (steps > 0) {
        hload(hA, 0);
        hstore(hA, 0);
    }
    if (steps > 1) hload(hB, 1);
    __syncthreads();
    for (int s = 0; s < steps; s += 2) {
        body(s, hA, hB);
        if (s + 1 < steps) body(s + 1, hB, hA);
    }
}

// ------------------------------------------------------------------------------------------------
// Weight-resident persistent fp32 3x3 conv, Ci = 64 (the fp32 headline path's dominant family: the 64-channel
// 3x3 convs of the ResidualUnits / RBBs / MultiScaleRefine at 64^2..256^2 and their input-gradients, the
// `conv_fwd_kernel<2, 1, 2, 2, 0, false, false>` population). That implicit-GEMM kernel is MFMA-bound at
// ~0.6-0.7 of the fp32 peak isolated: each 32-deep K chunk costs two barriers, a register->LDS store of
// 24 KB and a re-gather of the shifted A rows from L2, against 32 MFMAs per wave. Here one 512-thread block
// per CU holds the fp32 weights of a 32-channel output slice in LDS (9 taps x 32 co x 64 ci, 36-float rows:
// 83 KB) for the whole launch and walks 4-row x 64-pixel tiles; per tile and 32-channel chunk only the
// 6 x 66-pixel fp32 halo moves (7 float4 per thread, loaded during the previous chunk's MFMAs), so a wave
// issues 144 MFMAs (9 taps x 16 k-steps) per barrier pair. Fragments as in conv_fwd_body (k-permuted rows:
// one ds_read_b128 feeds 4 MFMA steps, 36-float pitch conflict-free); the product is formed transposed
// (C^T = W X^T) so the epilogue stores float4 from the accumulators. 8 waves = 4 output rows x 2 pixel
// halves, one 32 x 32 accumulator each. Exact fp32 (v_mfma_f32_32x32x2f32), the same sums per output as
// the implicit-GEMM kernel up to the K order.
constexpr int WF_PK = 36;  // floats per staged row (32 + 4 pad)
constexpr int WF_LDS_W = 2 * 9 * 32 * WF_PK;
constexpr int WF_LDS_H = HALO_NPX * WF_PK;

// Epilogue (BIAS kind: bias, residual, pre-activation store, ReLU / PReLU / ReLU-mask, accumulate): every operand
// it reads (bias, residual, mask, old y) is requested at the START of the tile's second chunk through buffer
// resources — an absent operand gets an empty resource, so its loads return 0 with no branch — and consumed only
// after that chunk's 144 MFMAs. The generic epi_store4 issued each load behind its own branch and waited on it
// (~8 serialised HBM round trips per tile; +14 % on a 3x3 with a residual).
__global__ __launch_bounds__(512, 1) void conv3x3_wres_f32_kernel(const ConvArgs a, int ntiles, int groups) {
    __shared__ __attribute__((aligned(16))) float lds[WF_LDS_W + WF_LDS_H];
    __shared__ int2 tapoff[9];
    // the whole VGPR file of its SIMDs (2 waves x 256; the code needs 182). Round 5 saw one run-to-run difference in
    // tests/test_bf6_gpu.py::test_bf6_refine_branch_determinism in the subset that runs this kernel (native fp32 GEMM on
    // MultiScaleRefine's scale 1) beside bf16x6 convs on another branch stream; of the kernels in that configuration it
    // is the one 512-thread persistent kernel whose allocation left a hole (144 VGPRs) other waves could share — a mix
    // only tests make (the fp32 GEMM mode is global). Free: its 140 KB of LDS already limits the CU to one block
    asm volatile("" ::: "v255");
    float* const Ws = lds;
    float* const Hs = lds + WF_LDS_W;
    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    const int nrt = (g.Ho + HALO_R - 1) / HALO_R, nct = g.Wo / HALO_TW;
    const int nb = gridDim.x / groups;  // group-major, nb % 8 == 0: see conv3x3_wres_f16_kernel
    const int grp = blockIdx.x / nb, bg = blockIdx.x - grp * nb;
    const int n0 = grp * 32;
    const int xcd = bg & 7, nx = (nb + 7 - xcd) >> 3, jx = bg >> 3;
    const int q = ntiles >> 3, rr8 = ntiles & 7;
    const int tbeg = xcd * q + min(xcd, rr8), tcnt = q + (xcd < rr8 ? 1 : 0);
    const int mytiles = jx < tcnt ? (tcnt - 1 - jx) / nx + 1 : 0;
    if (tid < 9) tapoff[tid] = make_int2(g.dh[tid], g.dw[tid]);
    // weights W2[co][t][ci] -> Ws[((c*9 + t)*32 + co)*36 + k], ci = 32c + k
    for (int f = tid; f < 32 * 9 * 16; f += 512) {
        const int co = f / 144, rem = f - co * 144, t = rem >> 4, ci = 4 * (rem & 15);
        *reinterpret_cast<float4*>(&Ws[(((ci >> 5) * 9 + t) * 32 + co) * WF_PK + (ci & 31)]) =
            ld4(a.w2 + (long long)(n0 + co) * a.ldw + t * 64 + ci);
    }
    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, (short)0, (int)std::min<long long>((long long)g.B * img * 4, 0x7FFFFFF0LL), 0x00020000);
    const int lane = tid & 63, wave = tid >> 6;
    const int orow = wave & 3, ph = wave >> 2;  // output row in the tile, 32-pixel half
    const int lr = lane & 31, lh = lane >> 5;

    auto tile_of = [&](int k, int& b, int& i0, int& j0) {
        int l = tbeg + jx + k * nx;
        const int rt = l % nrt; l /= nrt;
        const int ct = l % nct;
        b = l / nct;
        i0 = rt * HALO_R;
        j0 = ct * HALO_TW;
    };
    float4 hreg[WRES_HV];
    auto hload = [&](int step) {
        int b, i0, j0;
        tile_of(step >> 1, b, i0, j0);
        const int c = step & 1;
        const int base = b * (int)img;
#pragma unroll
        for (int v = 0; v < WRES_HV; ++v) {
            const int e = tid + 512 * v;
            const int px = e >> 3, c4 = e & 7;
            const int hr = px / HALO_HW, hc = px - hr * HALO_HW;
            const int ih = i0 - 1 + hr, iw = j0 - 1 + hc;
            const bool ok = e < HALO_E && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
            const int off = ok ? (base + (ih * g.Wi + iw) * g.ldx + 32 * c + 4 * c4) * 4 : (int)0x80000000;
            hreg[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        }
    };
    auto hstore = [&]() {
#pragma unroll
        for (int v = 0; v < WRES_HV; ++v) {
            const int e = tid + 512 * v;
            if (e < HALO_E) *reinterpret_cast<float4*>(&Hs[(e >> 3) * WF_PK + 4 * (e & 7)]) = hreg[v];
        }
    };
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const hyres_epilogue& e = a.e;
    const float slope = (e.act == HYRES_ACT_PRELU) ? e.slope[0] : 0.f;
    const long long npix = (long long)g.B * g.Ho * g.Wo;
    const __amdgpu_buffer_rsrc_t r_bias = opnd_rsrc(e.bias, (long long)g.Co * 4);
    const __amdgpu_buffer_rsrc_t r_res = opnd_rsrc(e.res, npix * e.ldres * 4);
    const __amdgpu_buffer_rsrc_t r_mask = opnd_rsrc(e.act == HYRES_ACT_RELU_MASK ? e.aux0 : nullptr, npix * e.ld0 * 4);
    const __amdgpu_buffer_rsrc_t r_old = opnd_rsrc(e.accumulate ? a.y : nullptr, npix * g.ldy * 4);
    float4 ebias[4], eres[4], emask[4], eold[4];
    const int steps = mytiles * 2;
    if (steps > 0) {
        hload(0);
        hstore();
    }
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
        const int k = s >> 1, c = s & 1;
        int b, i0, j0;
        tile_of(k, b, i0, j0);
        const int i = i0 + orow;
        const long long pix = ((long long)b * g.Ho + i) * g.Wo + j0 + 32 * ph + lr;
        if (c == 1) {  // the epilogue's operands, issued before the next halo (vmcnt retires in issue order)
            const bool okr = i < g.Ho;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int n = n0 + 8 * qd + 4 * lh;
                const int ob = n * 4;
                const int orr = okr ? (int)((pix * e.ldres + n) * 4) : (int)0x80000000;
                const int om = okr ? (int)((pix * e.ld0 + n) * 4) : (int)0x80000000;
                const int oy = okr ? (int)((pix * g.ldy + n) * 4) : (int)0x80000000;
                ebias[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_bias, ob, 0, 0));
                eres[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_res, orr, 0, 0));
                emask[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_mask, om, 0, 0));
                eold[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_old, oy, 0, 0));
            }
        }
        if (s + 1 < steps) hload(s + 1);
        const float* Wc = Ws + c * 9 * 32 * WF_PK;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int2 o = tapoff[t];
            const float* arow = &Hs[((orow + 1 + o.x) * HALO_HW + 32 * ph + lr + 1 + o.y) * WF_PK + lh * 16];
            const float* brow = &Wc[(t * 32 + lr) * WF_PK + lh * 16];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4 av = *reinterpret_cast<const float4*>(arow + 4 * u);
                const float4 bv = *reinterpret_cast<const float4*>(brow + 4 * u);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.x, av.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.y, av.y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.z, av.z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv.w, av.w, acc, 0, 0, 0);
            }
        }
        if (c == 1) {
            if (i < g.Ho) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    const int n = n0 + 8 * qd + 4 * lh;
                    float o[4] = {acc[4 * qd] + ebias[qd].x + eres[qd].x, acc[4 * qd + 1] + ebias[qd].y + eres[qd].y,
                                  acc[4 * qd + 2] + ebias[qd].z + eres[qd].z, acc[4 * qd + 3] + ebias[qd].w + eres[qd].w};
                    if (e.out2) st4(e.out2 + pix * e.ldo2 + n, make_float4(o[0], o[1], o[2], o[3]));
                    if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) o[k] = fmaxf(o[k], 0.f);
                    } else if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) o[k] = o[k] >= 0.f ? o[k] : slope * o[k];
                    } else if (e.act == HYRES_ACT_RELU_MASK) {
                        o[0] = emask[qd].x > 0.f ? o[0] : 0.f;
                        o[1] = emask[qd].y > 0.f ? o[1] : 0.f;
                        o[2] = emask[qd].z > 0.f ? o[2] : 0.f;
                        o[3] = emask[qd].w > 0.f ? o[3] : 0.f;
                    }
                    st4(a.y + pix * g.ldy + n,
                        make_float4(o[0] + eold[qd].x, o[1] + eold[qd].y, o[2] + eold[qd].z, o[3] + eold[qd].w));
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        }
        __syncthreads();  // every wave is done with this chunk's halo
        if (s + 1 < steps) hstore();
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// fp32-accurate weight-resident 3x3 conv on the bf16 MFMA ("bf16x6", hyres_conv_tuning key 7 = 1, the default).
// conv3x3_wres_f32_kernel above runs at ~0.7 of the fp32 MFMA peak, and that peak (157 TF/s) is 1/16 of the bf16
// MFMA's. Here every fp32 operand is split into three bf16 pieces x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1): 24 significant bits, |x - x0 - x1 - x2| <= 2^-25 |x|) and each product is formed from the
// six cross products with i + j <= 2 (the dropped ones are below 2^-26 |x y|) with fp32 accumulation on
// v_mfma_f32_32x32x16_bf16 (products of bf16 values are exact in fp32): per product the error is at most about
// 2^-25 relative, below the half-ulp rounding (2^-24) of the fp32 MFMA's own fmaf chain; 6 bf16 MFMAs per 16-deep K
// step against 8 fp32 ones per 2 x 8, i.e. 2.67x fewer MFMA cycles. The weights of the block's 32-channel output
// slice are split once into LDS (3 planes x 4 chunks of 16 input channels x 9 taps x 32 rows of 32 B: 108 KB), the
// halo of each 16-channel chunk is split when staged (3 planes x 396 px x 32 B: 37 KB; 9 taps reuse it). Both
// images swizzle the 16-B half of a 32-B row by bit 3 of the row: every ds_read_b128 lane group then hits 16
// distinct 16-B slots (conflict-free). Same tiles, waves, tile order and epilogue as conv3x3_wres_f32_kernel.
constexpr int BF6_WPL = 4 * 9 * 32 * 16;  // bf16 per weight plane
constexpr int BF6_HPL = HALO_NPX * 16;    // bf16 per halo plane
constexpr int BF6_HE = HALO_NPX * 4;      // float4 per 16-channel halo chunk
constexpr int BF6_HV = (BF6_HE + 511) / 512;
// 16-B segment (0 / 1) of element k (0..15) of row r in a swizzled [row][16] bf16 image, as an element offset
__device__ __forceinline__ int bf6_off(int r, int k) { return r * 16 + ((((k >> 3) ^ (r >> 3)) & 1) << 3) + (k & 7); }

// V (hyres_conv_tuning key 12, default 1): bit 0 — each tap's six fragments are read one tap ahead into a second
// register set (hand-issued ds_read_b128: the compiler sank its own reads next to their MFMAs, waiting on each) —
// 133 -> 125 us at 128^2, 481 -> 453 us at 256^2 (profiles/r5i_wres_variants_micro.txt); bit 1 — waves 4..7 at static
// priority 1: no effect (kept for the A/B). Every variant forms the same MFMAs in the same order (bit-identical)
// D (round 5): the halo radius = the taps' largest offset, 1 (3x3) or 2 (MultiScaleRefine's dilation-2 3x3s,
// enhancement.py:44-51): (4 + 2D) x (64 + 2D) halo pixels; at D = 2 the three halo planes are 52 KB, 159 KB of LDS in all
template <bool GUARD, int V, int D = 1>
__global__ __launch_bounds__(512, 1) void conv3x3_wres_bf6_kernel(const ConvArgs a, int ntiles, int groups) {
    constexpr int HW = HALO_TW + 2 * D, NPX = (HALO_R + 2 * D) * HW;  // halo row length, pixels
    constexpr int HPL = NPX * 16, HE = NPX * 4, HV = (HE + 511) / 512;  // bf16 per halo plane, float4 per chunk
    __shared__ __attribute__((aligned(16))) __bf16 lds[3 * BF6_WPL + 3 * HPL];
    __shared__ int2 tapoff[9];
    __bf16* const Ws = lds;
    __bf16* const Hs = lds + 3 * BF6_WPL;
    // GUARD: the block takes the whole VGPR file of its SIMDs (2 waves x 256; the code needs 220). With the compiler's
    // 224, waves of OTHER kernels co-resident on those SIMDs (a bilinear on a side stream) computed wrong values while
    // this kernel's own output stayed exact (round 4, tests/test_bf6_gpu.py::test_bf6_kernels_beside_a_bilinear: 0.25
    // off, gone with this line). The error signature and the probes that isolate it: DESIGN §4 "Cross-kernel
    // interference" (scripts/diag_bf6_mechanism.py, scripts/coresidency_probe.hip). No cost to this kernel (its LDS
    // already limits the CU to one block). GUARD = false exists only for that diagnosis (hyres_conv_tuning key 9 = 0).
    if constexpr (GUARD) asm volatile("" ::: "v255");
    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    const int nrt = (g.Ho + HALO_R - 1) / HALO_R, nct = g.Wo / HALO_TW;
    const int nb = gridDim.x / groups;  // group-major, nb % 8 == 0: see conv3x3_wres_f16_kernel
    const int grp = blockIdx.x / nb, bg = blockIdx.x - grp * nb;
    const int n0 = grp * 32;
    const int xcd = bg & 7, nx = (nb + 7 - xcd) >> 3, jx = bg >> 3;
    const int q = ntiles >> 3, rr8 = ntiles & 7;
    const int tbeg = xcd * q + min(xcd, rr8), tcnt = q + (xcd < rr8 ? 1 : 0);
    const int mytiles = jx < tcnt ? (tcnt - 1 - jx) / nx + 1 : 0;
    if (tid < 9) tapoff[tid] = make_int2(g.dh[tid], g.dw[tid]);
    // weights W2[co][t][ci] (fp32) -> three bf16 planes, row (chunk c = ci / 16, tap t, co), element ci % 16
    for (int f = tid; f < 32 * 9 * 16; f += 512) {
        const int co = f / 144, rem = f - co * 144, t = rem >> 4, ci = 4 * (rem & 15);
        bf16x4_t h, m, l;
        bf6_split4(ld4(a.w2 + (long long)(n0 + co) * a.ldw + t * 64 + ci), h, m, l);
        const int row = ((ci >> 4) * 9 + t) * 32 + co;
        const int o = bf6_off(row, ci & 15);
        *reinterpret_cast<bf16x4_t*>(&Ws[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&Ws[BF6_WPL + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&Ws[2 * BF6_WPL + o]) = l;
    }
    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, (short)0, (int)std::min<long long>((long long)g.B * img * 4, 0x7FFFFFF0LL), 0x00020000);
    const int lane = tid & 63, wave = tid >> 6;
    const int orow = wave & 3, ph = wave >> 2;  // output row in the tile, 32-pixel half
    const int lr = lane & 31, lh = lane >> 5;

    auto tile_of = [&](int k, int& b, int& i0, int& j0) {
        int l = tbeg + jx + k * nx;
        const int rt = l % nrt; l /= nrt;
        const int ct = l % nct;
        b = l / nct;
        i0 = rt * HALO_R;
        j0 = ct * HALO_TW;
    };
    // halo chunks are prefetched TWO steps ahead (two register sets, alternating, as conv3x3_wres_f16_kernel): one
    // 16-channel step is 54 MFMAs per wave (~1.7k cycles), too short to cover an HBM load issued one step ahead
    auto hload = [&](float4 (&hreg)[HV], int step) {  // step = 4 * tile + chunk (16 channels)
        int b, i0, j0;
        tile_of(step >> 2, b, i0, j0);
        const int c = step & 3;
        const int base = b * (int)img;
#pragma unroll
        for (int v = 0; v < HV; ++v) {
            const int e = tid + 512 * v;
            const int px = e >> 2, c4 = e & 3;
            const int hr = px / HW, hc = px - hr * HW;
            const int ih = i0 - D + hr, iw = j0 - D + hc;
            const bool ok = e < HE && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
            const int off = ok ? (base + (ih * g.Wi + iw) * g.ldx + 16 * c + 4 * c4) * 4 : (int)0x80000000;
            hreg[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        }
    };
    // the next step's halo is split into its bf16 pieces in registers DURING this step's MFMAs (hsplit, independent
    // VALU work the scheduler interleaves with them); between the two barriers only the LDS stores remain (hput)
    bf16x4_t sp[HV][3];
    auto hsplit = [&](const float4 (&hreg)[HV]) {
#pragma unroll
        for (int v = 0; v < HV; ++v) bf6_split4(hreg[v], sp[v][0], sp[v][1], sp[v][2]);
    };
    auto hput = [&]() {
#pragma unroll
        for (int v = 0; v < HV; ++v) {
            const int e = tid + 512 * v;
            if (e < HE) {
                const int o = bf6_off(e >> 2, 4 * (e & 3));
                *reinterpret_cast<bf16x4_t*>(&Hs[o]) = sp[v][0];
                *reinterpret_cast<bf16x4_t*>(&Hs[HPL + o]) = sp[v][1];
                *reinterpret_cast<bf16x4_t*>(&Hs[2 * HPL + o]) = sp[v][2];
            }
        }
    };
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const hyres_epilogue& e = a.e;
    const float slope = (e.act == HYRES_ACT_PRELU || e.act == HYRES_ACT_PRELU_MASK) ? e.slope[0] : 0.f;
    const long long npix = (long long)g.B * g.Ho * g.Wo;
    const __amdgpu_buffer_rsrc_t r_bias = opnd_rsrc(e.bias, (long long)g.Co * 4);
    const __amdgpu_buffer_rsrc_t r_res = opnd_rsrc(e.res, npix * e.ldres * 4);
    const __amdgpu_buffer_rsrc_t r_mask = opnd_rsrc(
        (e.act == HYRES_ACT_RELU_MASK || e.act == HYRES_ACT_PRELU_MASK) ? e.aux0 : nullptr, npix * e.ld0 * 4);
    const __amdgpu_buffer_rsrc_t r_old = opnd_rsrc(e.accumulate ? a.y : nullptr, npix * g.ldy * 4);
    float4 ebias[4], eres[4], emask[4], eold[4];
    float pslope = 0.f;  // HYRES_ACT_PRELU_MASK: this thread's share of sum_{pre <= 0} pre * gradient
    const int steps = mytiles * 4;
    float4 hA[HV], hB[HV];
    if (steps > 0) {
        hload(hA, 0);
        hsplit(hA);
        hput();
    }
    if (steps > 1) hload(hB, 1);
    __syncthreads();
    // step s: the set that held step s's halo (stored) receives step s + 2; the other holds step s + 1
    auto body = [&](int s, float4 (&hl)[HV], const float4 (&hs)[HV]) {
        const int k = s >> 2, c = s & 3;
        int b, i0, j0;
        tile_of(k, b, i0, j0);
        const int i = i0 + orow;
        const long long pix = ((long long)b * g.Ho + i) * g.Wo + j0 + 32 * ph + lr;
        if (c == 3) {  // the epilogue's operands, issued before the next halo (vmcnt retires in issue order)
            const bool okr = i < g.Ho;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int n = n0 + 8 * qd + 4 * lh;
                const int ob = n * 4;
                const int orr = okr ? (int)((pix * e.ldres + n) * 4) : (int)0x80000000;
                const int om = okr ? (int)((pix * e.ld0 + n) * 4) : (int)0x80000000;
                const int oy = okr ? (int)((pix * g.ldy + n) * 4) : (int)0x80000000;
                ebias[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_bias, ob, 0, 0));
                eres[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_res, orr, 0, 0));
                emask[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_mask, om, 0, 0));
                eold[qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_old, oy, 0, 0));
            }
        }
        if (s + 2 < steps) hload(hl, s + 2);
        if constexpr ((V & 1) != 0) {
            // explicit software pipeline: tap t + 1's six fragments are read (hand-issued ds_read_b128, so the
            // compiler cannot sink them to their uses) while tap t's MFMAs run; each MFMA pair waits only for its
            // own two reads (the LDS return counter retires in order; any other LGKM op only makes a wait longer)
            typedef __attribute__((address_space(3))) __bf16 lds_bf16;
            const unsigned wbase = (unsigned)(size_t)(lds_bf16*)Ws, hbase = (unsigned)(size_t)(lds_bf16*)Hs;
            auto rd = [&](unsigned addr) -> bf16x8_t {
                bf16x8_t r;
                asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr) : "memory");
                return r;
            };
            auto frag = [&](int t, bf16x8_t (&wv)[3], bf16x8_t (&xv)[3]) {
                const int wrow = (c * 9 + t) * 32 + lr;
                const int hrow = (orow + D + g.dh[t]) * HW + 32 * ph + lr + D + g.dw[t];
                const unsigned wo = wbase + 2u * (wrow * 16 + (((lh ^ (wrow >> 3)) & 1) << 3));
                const unsigned ho = hbase + 2u * (hrow * 16 + (((lh ^ (hrow >> 3)) & 1) << 3));
                wv[2] = rd(wo + 4u * BF6_WPL);
                xv[0] = rd(ho);
                wv[1] = rd(wo + 2u * BF6_WPL);
                xv[1] = rd(ho + 2u * HPL);
                wv[0] = rd(wo);
                xv[2] = rd(ho + 4u * HPL);
            };
            bf16x8_t fw[2][3], fx[2][3];
            hsplit(hs);  // unconditional (unused after the last step): no branch inside the tap loop
            frag(0, fw[0], fx[0]);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                bf16x8_t(&w)[3] = fw[t & 1];
                bf16x8_t(&x)[3] = fx[t & 1];
                if (t + 1 < 9) {
                    frag(t + 1, fw[(t + 1) & 1], fx[(t + 1) & 1]);
                    asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(w[2]), "+v"(x[0]));
                } else {
                    asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(w[2]), "+v"(x[0]));
                }
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acc, 0, 0, 0);
                if (t + 1 < 9) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(w[1]), "+v"(x[1]));
                else asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(w[1]), "+v"(x[1]));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acc, 0, 0, 0);
                if (t + 1 < 9) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(w[0]), "+v"(x[2]));
                else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(x[2]));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[0], acc, 0, 0, 0);
            }
        } else {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int2 o = tapoff[t];
            const int wrow = (c * 9 + t) * 32 + lr;                                    // A: weights, row = co
            const int hrow = (orow + D + o.x) * HW + 32 * ph + lr + D + o.y;          // B: halo, row = pixel
            const int wo = wrow * 16 + (((lh ^ (wrow >> 3)) & 1) << 3);
            const int ho = hrow * 16 + (((lh ^ (hrow >> 3)) & 1) << 3);
            const bf16x8_t w0 = *reinterpret_cast<const bf16x8_t*>(&Ws[wo]);
            const bf16x8_t w1 = *reinterpret_cast<const bf16x8_t*>(&Ws[BF6_WPL + wo]);
            const bf16x8_t w2 = *reinterpret_cast<const bf16x8_t*>(&Ws[2 * BF6_WPL + wo]);
            const bf16x8_t x0 = *reinterpret_cast<const bf16x8_t*>(&Hs[ho]);
            const bf16x8_t x1 = *reinterpret_cast<const bf16x8_t*>(&Hs[HPL + ho]);
            const bf16x8_t x2 = *reinterpret_cast<const bf16x8_t*>(&Hs[2 * HPL + ho]);
            // the small cross products first, the leading one last
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, x0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x2, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x0, acc, 0, 0, 0);
            if (t == 1 && s + 1 < steps) hsplit(hs);  // step s + 1's halo (loaded a step ago) -> bf16 pieces
        }
        }
        if (c == 3) {
            if (i < g.Ho) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    const int n = n0 + 8 * qd + 4 * lh;
                    float o[4] = {acc[4 * qd] + ebias[qd].x + eres[qd].x, acc[4 * qd + 1] + ebias[qd].y + eres[qd].y,
                                  acc[4 * qd + 2] + ebias[qd].z + eres[qd].z, acc[4 * qd + 3] + ebias[qd].w + eres[qd].w};
                    if (e.out2) st4(e.out2 + pix * e.ldo2 + n, make_float4(o[0], o[1], o[2], o[3]));
                    if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) o[kk] = fmaxf(o[kk], 0.f);
                    } else if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) o[kk] = o[kk] >= 0.f ? o[kk] : slope * o[kk];
                    } else if (e.act == HYRES_ACT_RELU_MASK) {
                        o[0] = emask[qd].x > 0.f ? o[0] : 0.f;
                        o[1] = emask[qd].y > 0.f ? o[1] : 0.f;
                        o[2] = emask[qd].z > 0.f ? o[2] : 0.f;
                        o[3] = emask[qd].w > 0.f ? o[3] : 0.f;
                    } else if (e.act == HYRES_ACT_PRELU_MASK) {  // as prelu_bwd4_kernel, per element
                        const float pv[4] = {emask[qd].x, emask[qd].y, emask[qd].z, emask[qd].w};
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) {
                            if (!(pv[kk] > 0.f)) pslope += pv[kk] * o[kk];
                            o[kk] = pv[kk] > 0.f ? o[kk] : slope * o[kk];
                        }
                    }
                    st4(a.y + pix * g.ldy + n,
                        make_float4(o[0] + eold[qd].x, o[1] + eold[qd].y, o[2] + eold[qd].z, o[3] + eold[qd].w));
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        }
        __syncthreads();  // every wave is done with this chunk's halo
        if (s + 1 < steps) hput();
        __syncthreads();
    };
    if constexpr ((V & 2) != 0) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    for (int s = 0; s < steps; s += 2) {
        body(s, hA, hB);
        if (s + 1 < steps) body(s + 1, hB, hA);
    }
    if (e.act == HYRES_ACT_PRELU_MASK) {  // block partial of the slope gradient (every body ended with a barrier)
        float* red = reinterpret_cast<float*>(lds);
        red[tid] = pslope;
        __syncthreads();
        for (int k = 256; k > 0; k >>= 1) {
            if (tid < k) red[tid] += red[tid + k];
            __syncthreads();
        }
        if (tid == 0) const_cast<float*>(e.aux2)[blockIdx.x] = red[0];
    }
}

// HYRES_ACT_PRELU_MASK's second kernel: the block partials summed in a fixed order, added to the slope gradient
__global__ __launch_bounds__(256) void prelu_slope_sum_kernel(const float* part, int n, float* dst) {
    __shared__ float red[256];
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) dst[0] += red[0];
}

// ------------------------------------------------------------------------------------------------
// Streaming 1x1 conv (K = Ci <= 128, Co = 32*NT): the K-short pointwise layers of the ResidualUnits /
// RBBs at 64^2..256^2 sit at the fp32 ridge (64-128 FLOP per output element against 8-12 bytes), and the
// tiled kernel above runs them as lock-stepped blocks (load, then MFMA, then epilogue), so their MFMA and
// HBM phases add instead of overlapping. Here each WAVE streams its own 32-pixel tiles with no block
// barrier after the one-time weight staging:
//   * W [Co][K] sits in LDS for the whole (persistent) block, pitch K+4 (conflict-free ds_read_b128);
//   * the wave's A operand goes HBM -> registers directly in the MFMA layout: lane (r, h) holds pixel
//     p0+r, channels 8j+4h..8j+4h+3 (j < K/8), so a float4 feeds 4 MFMA k-steps; each float4 is reloaded
//     for the wave's next tile right after its last MFMA (rolling prefetch);
//   * the product is formed transposed (C^T = W X^T), so each lane's accumulator holds 4 consecutive
//     channels of one pixel per register quad: the results are stored as float4 straight from the
//     accumulator layout — no LDS round trip.
// Exact fp32 (v_mfma_f32_32x32x2f32), epilogue bias + ReLU / PReLU (+ pre-activation copy). Layers whose
// epilogue streams a second operand (residual, ReLU mask, old y) stay on the tiled kernel: prefetching
// that operand per wave tile doubles the registers (2 waves/SIMD) and measured slower than the tiles
// (128^2 64->128 +res 95 vs 92 us, 64^2 27 vs 24 us; profiles/r2_micro_1x1_stream.txt).
// R16 (autocast, f16_operands): both operands are rounded to fp16 as they are loaded, and the products of
// those fp16 values are formed exactly by the fp32 MFMA with fp32 accumulation — the same arithmetic as the
// f16 MFMA (whose products of fp16 inputs are exact in fp32) up to the summation order. These layers are
// HBM-bound (<= 128 FLOP per output element), so the f16 rate buys nothing and the streaming structure does.
__device__ __forceinline__ float4 round_f16(float4 v) {
    return make_float4((float)(_Float16)v.x, (float)(_Float16)v.y, (float)(_Float16)v.z, (float)(_Float16)v.w);
}

template <int NT, int KC, bool R16 = false>
__global__ __launch_bounds__(256, 2) void conv1x1_stream_kernel(const ConvArgs a) {
    constexpr int K = 8 * KC, KP = K + 4, CO = 32 * NT;
    __shared__ __attribute__((aligned(16))) float Ws[CO * KP];
    const hyres_conv_geom& g = a.g;
    const hyres_epilogue& e = a.e;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    for (int i = tid; i < CO * (K / 4); i += 256) {
        const int co = i / (K / 4), k4 = i - co * (K / 4);
        float4 w = ld4(a.w2 + (long long)co * a.ldw + 4 * k4);
        if constexpr (R16) w = round_f16(w);
        *reinterpret_cast<float4*>(&Ws[co * KP + 4 * k4]) = w;
    }
    __shared__ __attribute__((aligned(16))) float bs[CO];
    for (int i = tid; i < CO; i += 256) bs[i] = e.bias ? e.bias[i] : 0.f;
    const float slope = (e.act == HYRES_ACT_PRELU) ? e.slope[0] : 0.f;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
    const int ntile = (a.M + 31) / 32;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    auto load_a = [&](int tile, int j) -> float4 {
        const int p = tile * 32 + lr;
        const int off = (tile < ntile && p < a.M) ? (p * g.ldx + 8 * j + 4 * lh) * 4 : (int)0x80000000;
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    };
    float4 av[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) av[j] = load_a(gw, j);
    // GEMM as C^T = W X^T (MFMA A operand = weights, B operand = pixels): lane (r, h) ends up holding
    // pixel p0+r, channels 32t + 8q + 4h .. +3 in acc[t][4q .. 4q+3] -> one float4 per (t, q)
    for (int tile = gw; tile < ntile; tile += nw) {
        const int p = tile * 32 + lr;
        const bool pok = p < a.M;
        floatx16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            float4 bv[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) bv[t] = *reinterpret_cast<const float4*>(&Ws[(32 * t + lr) * KP + 8 * j + 4 * lh]);
            float4 x = av[j];
            if constexpr (R16) x = round_f16(x);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[t].x, x.x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[t].y, x.y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[t].z, x.z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[t].w, x.w, acc[t], 0, 0, 0);
            }
            av[j] = load_a(tile + nw, j);  // rolling prefetch of the wave's next tile
        }
        if (a.prio) __builtin_amdgcn_s_setprio(0);
        if (!pok) continue;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = 32 * t + 8 * q + 4 * lh;
                const float4 b4 = *reinterpret_cast<const float4*>(&bs[n]);
                float o[4] = {acc[t][4 * q] + b4.x, acc[t][4 * q + 1] + b4.y, acc[t][4 * q + 2] + b4.z,
                              acc[t][4 * q + 3] + b4.w};
                if (e.out2) st4(e.out2 + (long long)p * e.ldo2 + n, make_float4(o[0], o[1], o[2], o[3]));
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (e.act == HYRES_ACT_RELU) o[c] = fmaxf(o[c], 0.f);
                    else if (e.act == HYRES_ACT_PRELU) o[c] = o[c] >= 0.f ? o[c] : slope * o[c];
                }
                st4(a.y + (long long)p * g.ldy + n, make_float4(o[0], o[1], o[2], o[3]));
            }
    }
}

// ------------------------------------------------------------------------------------------------
// Streaming 1x1 conv with fp16 activations in HBM (AMP training / autocast, io_f16 = 3: X and Y / residual / mask /
// old y all fp16), K = Ci in {64, 96, 128}, Co = 32 * NT in {64, 96, 128}, on the f16 MFMA. These layers (the
// ResidualUnits' 1x1 convs and their input-gradients with the ReLU mask and the accumulated residual gradient) are
// HBM-latency-bound on the tiled kernel (64-row blocks of 2-4 K chunks, each load then barrier then MFMA: ~0.3 of
// HBM). Here, as conv1x1_stream_kernel, each WAVE streams its own 32-pixel tiles with no barrier after the one-time
// weight staging (W -> fp16 in LDS, pitch K + 8 halves): the wave's X fragments come HBM -> registers in the MFMA
// layout (lane (r, h): pixel p0 + r, channels 16j + 8h .. + 7, one 16-byte load per k-step) with a rolling prefetch
// of the next tile, and the product is formed transposed (C^T = W X^T) so each lane's accumulator holds 4 consecutive
// channels of one pixel. Layers with a streamed epilogue operand (residual, ReLU mask, old y) stay on the tiles
// (measured: stream_h_nt). Arithmetic: fp16 operands, fp32 accumulation, fp32 epilogue, one rounding at the fp16
// store — the tiled f16 kernel's, in the same K order.
typedef _Float16 half8s_t __attribute__((ext_vector_type(8)));

template <int NT, int KC>
__global__ __launch_bounds__(256, 2) void conv1x1_stream_h_kernel(const ConvArgs a) {
    constexpr int K = 16 * KC, KP = K + 8, CO = 32 * NT;
    __shared__ __attribute__((aligned(16))) _Float16 Ws[CO * KP];
    __shared__ __attribute__((aligned(16))) float bs[CO];
    const hyres_conv_geom& g = a.g;
    const hyres_epilogue& e = a.e;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    for (int i = tid; i < CO * (K / 4); i += 256) {
        const int co = i / (K / 4), k4 = i - co * (K / 4);
        const float4 w = ld4(a.w2 + (long long)co * a.ldw + 4 * k4);
        *reinterpret_cast<half4_t*>(&Ws[co * KP + 4 * k4]) = half4_t{(_Float16)w.x, (_Float16)w.y, (_Float16)w.z,
                                                                     (_Float16)w.w};
    }
    for (int i = tid; i < CO; i += 256) bs[i] = e.bias ? e.bias[i] : 0.f;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
    _Float16* const y = reinterpret_cast<_Float16*>(a.y);
    const int ntile = (a.M + 31) / 32;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    auto load_x = [&](int tile, int j) -> half8s_t {
        const int p = tile * 32 + lr;
        const int off = (tile < ntile && p < a.M) ? (p * g.ldx + 16 * j + 8 * lh) * 2 : (int)0x80000000;
        return __builtin_bit_cast(half8s_t, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    };
    half8s_t xv[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) xv[j] = load_x(gw, j);
    for (int tile = gw; tile < ntile; tile += nw) {
        const int p = tile * 32 + lr;
        const bool pok = p < a.M;
        floatx16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            const half8s_t x = xv[j];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const half8s_t w = *reinterpret_cast<const half8s_t*>(&Ws[(32 * t + lr) * KP + 16 * j + 8 * lh]);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w, x, acc[t], 0, 0, 0);
            }
            xv[j] = load_x(tile + nw, j);  // rolling prefetch of the wave's next tile
        }
        if (!pok) continue;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = 32 * t + 8 * q + 4 * lh;
                const float4 b4 = *reinterpret_cast<const float4*>(&bs[n]);
                float o[4] = {acc[t][4 * q] + b4.x, acc[t][4 * q + 1] + b4.y, acc[t][4 * q + 2] + b4.z,
                              acc[t][4 * q + 3] + b4.w};
                if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
                }
                const half4_t h = {(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
                *reinterpret_cast<half4_t*>(y + (long long)p * g.ldy + n) = h;
            }
    }
}

// ------------------------------------------------------------------------------------------------
// Streaming 1x1 conv with fp16 activations AND streamed epilogue operands (round 6, AMP training: the ResidualUnit /
// RBB tails relu(W x + b + residual) and the input-gradients with the ReLU mask and the accumulated gradient; io_f16 =
// 3, every operand fp16), K = Ci in {64, 128}, Co = 32 * NT in {64, 128}, F: residual (1) | ReLU mask (2) |
// accumulate (4). conv1x1_stream_h_kernel's X stream and f16 products (C^T = W X^T: the tiled kernel's products, bit-
// identical), with conv1x1_stream_b6_kernel's two fixes for the streamed operands: co tile t + 1's operands are in
// flight while co tile t multiplies (two register sets), and every operand / store moves as pixel rows — the
// accumulator goes through a per-wave LDS scratch (MFMA layout in, rows out: lane l -> pixel p0 + (l >> 3) + 8q,
// channels 32t + 4 (l & 7) .. + 3), so an instruction covers 8 pixel rows x 64 contiguous bytes instead of the lane
// layout's 32 rows x 8 B (profiles/r5h_access_probe.txt: the narrow pieces cap a read+write stream near 3 TB/s). The
// round-5 version without the row-shaped epilogue measured 2-10 % slower than the tiles (profiles/r5g_stream_hf_ab.txt).
// Arithmetic: fp16 operands, fp32 accumulation and epilogue ((acc + b) + residual, mask, + old y), one fp16 rounding
// at the store — the tiled f16 kernel's (tests/test_stream_h_gpu.py: bit for bit).
// F & 8 (round 6, AMP training with SpatialAttention folded into MultiScaleRefine's fusion 1x1): HYRES_EPI_SA_BWD, the
// fusion's input-gradient 64 -> 192 (NT = 6, KC = 4) with SpatialAttention's mean / max backward added per pixel —
// acc + d mean / C + (channel == argmax ? d max : 0) (+ old y), epi_store4's SA_BWD arithmetic; the per-pixel operands
// (aux0 [P][ld0] fp32 pairs, aux2 int argmax) roll a tile ahead like the others.
template <int NT, int KC, int F>
__global__ __launch_bounds__(256, 2) void conv1x1_stream_hf_kernel(const ConvArgs a) {
    constexpr int K = 16 * KC, KP = K + 8, CO = 32 * NT, EP = 36;
    constexpr bool RES = (F & 1) != 0, MASK = (F & 2) != 0, ACC = (F & 4) != 0, SAB = (F & 8) != 0;
    static_assert(!SAB || (!RES && !MASK), "SA_BWD: no residual / mask");
    // RS (F & 16, round 6, AMP training with SpatialAttention folded): HYRES_EPI_ROWSCALE, the fusion 1x1 forward
    // 192 -> 64 (NT = 2, KC = 12) — o = acc * aux1[p] + bias, the pre-activation copy to out2 (fp16), then ReLU / PReLU
    constexpr bool RS = (F & 16) != 0;
    static_assert(!RS || (!RES && !MASK && !ACC && !SAB), "ROWSCALE: no other operand");
    // PM (F & 32, with SAB): conv1x1_stream_b6_kernel's PReLU mask on channels [0, 64), pre fp16; the gradient is
    // rounded to fp16 first (the unfused chain's stored value)
    constexpr bool PM = (F & 32) != 0;
    static_assert(!PM || (SAB && !ACC), "PReLU mask: the SA_BWD form without accumulate");
    static_assert(NT % 2 == 0, "operands alternate between two register sets per co tile");
    __shared__ __attribute__((aligned(16))) _Float16 Ws[CO * KP];
    __shared__ __attribute__((aligned(16))) float bs[CO];
    __shared__ __attribute__((aligned(16))) float Es[4 * 32 * EP];
    const hyres_conv_geom& g = a.g;
    const hyres_epilogue& e = a.e;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    for (int i = tid; i < CO * (K / 4); i += 256) {
        const int co = i / (K / 4), k4 = i - co * (K / 4);
        const float4 w = ld4(a.w2 + (long long)co * a.ldw + 4 * k4);
        *reinterpret_cast<half4_t*>(&Ws[co * KP + 4 * k4]) = half4_t{(_Float16)w.x, (_Float16)w.y, (_Float16)w.z,
                                                                     (_Float16)w.w};
    }
    for (int i = tid; i < CO; i += 256) bs[i] = e.bias ? e.bias[i] : 0.f;
    __syncthreads();
    const long long npix = a.M;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_res = opnd_rsrc(RES ? e.res : nullptr, npix * e.ldres * 2);
    const __amdgpu_buffer_rsrc_t r_mask = opnd_rsrc(MASK ? e.aux0 : nullptr, npix * e.ld0 * 2);
    const __amdgpu_buffer_rsrc_t r_old = opnd_rsrc(ACC ? a.y : nullptr, npix * g.ldy * 2);
    const __amdgpu_buffer_rsrc_t r_gm = opnd_rsrc(SAB ? e.aux0 : nullptr, npix * e.ld0 * 4);
    const __amdgpu_buffer_rsrc_t r_am = opnd_rsrc(SAB ? e.aux2 : nullptr, npix * 4);
    const __amdgpu_buffer_rsrc_t r_rs = opnd_rsrc(RS ? e.aux1 : nullptr, npix * e.ld1 * 4);
    const float slope = (RS && e.act == HYRES_ACT_PRELU) ? e.slope[0] : 0.f;
    _Float16* const o2 = reinterpret_cast<_Float16*>(e.out2);
    constexpr int OOR = (int)0x80000000;
    _Float16* const y = reinterpret_cast<_Float16*>(a.y);
    const int ntile = (a.M + 31) / 32;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    auto load_x = [&](int tile, int j) -> half8s_t {
        const int p = tile * 32 + lr;
        const int off = (tile < ntile && p < a.M) ? (p * g.ldx + 16 * j + 8 * lh) * 2 : OOR;
        return __builtin_bit_cast(half8s_t, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    };
    const int cr = lane >> 3, cc = 4 * (lane & 7);
    auto ooff = [&](int tile, int ld, int t, int q) -> int {
        const int p = tile * 32 + cr + 8 * q;
        return (tile < ntile && p < a.M) ? (p * ld + 32 * t + cc) * 2 : OOR;
    };
    half4_t eres[RES ? 2 : 1][4], emask[MASK ? 2 : 1][4], eold[ACC ? 2 : 1][4], epre[PM ? 2 : 1][4];
    const __amdgpu_buffer_rsrc_t r_pm = opnd_rsrc(PM ? e.aux1 : nullptr, npix * e.ld1 * 2);
    const float pslope_a = PM ? e.slope[0] : 0.f;
    float pslope = 0.f;
    auto load_epi = [&](int tile, int t, int set) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (RES) eres[set][q] = bload4h(r_res, ooff(tile, e.ldres, t, q));
            if constexpr (MASK) emask[set][q] = bload4h(r_mask, ooff(tile, e.ld0, t, q));
            if constexpr (ACC) eold[set][q] = bload4h(r_old, ooff(tile, g.ldy, t, q));
            if constexpr (PM) epre[set][q] = bload4h(r_pm, t < 2 ? ooff(tile, e.ld1, t, q) : OOR);
        }
    };
    // SA_BWD's / ROWSCALE's per-pixel operands: one set per tile, two sets (the next tile's are issued with its X)
    float2 sgm[SAB ? 2 : 1][4];
    int sam[SAB ? 2 : 1][4];
    float srs[RS ? 2 : 1][4];
    auto load_rs = [&](int tile, int set) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int p = tile * 32 + cr + 8 * q;
            const bool ok = tile < ntile && p < a.M;
            srs[set][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r_rs, ok ? p * e.ld1 * 4 : OOR, 0, 0));
        }
    };
    auto load_sab = [&](int tile, int set) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int p = tile * 32 + cr + 8 * q;
            const bool ok = tile < ntile && p < a.M;
            sgm[set][q] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r_gm, ok ? p * e.ld0 * 4 : OOR,
                                                                                          0, 0));
            sam[set][q] = __builtin_amdgcn_raw_buffer_load_b32(r_am, ok ? p * 4 : OOR, 0, 0);
        }
    };
    half8s_t xv[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) xv[j] = load_x(gw, j);
    load_epi(gw, 0, 0);
    if constexpr (SAB) load_sab(gw, 0);
    if constexpr (RS) load_rs(gw, 0);
    float* const es = Es + wave * 32 * EP;
    int tset = 0;
    for (int tile = gw; tile < ntile; tile += nw, tset ^= 1) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int cur = t & 1;
            if (t + 1 < NT) load_epi(tile, t + 1, cur ^ 1);
            else load_epi(tile + nw, 0, cur ^ 1);
            if constexpr (SAB) {
                if (t == NT - 1) {  // constant set indices (a dynamic one puts the arrays in scratch)
                    if (tset) load_sab(tile + nw, 0);
                    else load_sab(tile + nw, 1);
                }
            }
            if constexpr (RS) {
                if (t == NT - 1) {
                    if (tset) load_rs(tile + nw, 0);
                    else load_rs(tile + nw, 1);
                }
            }
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const half8s_t w = *reinterpret_cast<const half8s_t*>(&Ws[(32 * t + lr) * KP + 16 * j + 8 * lh]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w, xv[j], acc, 0, 0, 0);
                if (t == NT - 1) xv[j] = load_x(tile + nw, j);  // the next tile's X after its last use
            }
            // accumulator -> the wave's scratch in the MFMA layout -> back as pixel rows (LDS instructions of one wave
            // run in order; the fences keep the compiler from moving the previous co tile's reads past these writes)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(&es[lr * EP + 8 * q + 4 * lh]) =
                    make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = 32 * t + cc;
                const float4 b4 = *reinterpret_cast<const float4*>(&bs[n]);
                const float4 av = *reinterpret_cast<const float4*>(&es[(cr + 8 * q) * EP + cc]);
                const int p = tile * 32 + cr + 8 * q;
                float o[4] = {av.x + b4.x, av.y + b4.y, av.z + b4.z, av.w + b4.w};
                if constexpr (SAB) {  // epi_store4's SA_BWD: (acc + d mean / C) + (channel == argmax ? d max : 0)
                    const float2 gm = tset ? sgm[1][q] : sgm[0][q];
                    const int mi = tset ? sam[1][q] : sam[0][q];
                    o[0] = av.x + gm.x + (n == mi ? gm.y : 0.f);
                    o[1] = av.y + gm.x + (n + 1 == mi ? gm.y : 0.f);
                    o[2] = av.z + gm.x + (n + 2 == mi ? gm.y : 0.f);
                    o[3] = av.w + gm.x + (n + 3 == mi ? gm.y : 0.f);
                }
                if constexpr (PM) {
                    if (t < 2 && p < a.M) {
                        const float4 pv4 = h2f4(epre[cur][q]);
                        const float pv[4] = {pv4.x, pv4.y, pv4.z, pv4.w};
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            o[c] = (float)(_Float16)o[c];
                            if (!(pv[c] > 0.f)) pslope += pv[c] * o[c];
                            o[c] = pv[c] > 0.f ? o[c] : pslope_a * o[c];
                        }
                    }
                }
                if constexpr (RS) {  // epi_store4's ROWSCALE: (acc * scale) + bias, out2, then the activation
                    const float sc = tset ? srs[1][q] : srs[0][q];
                    o[0] = av.x * sc + b4.x;
                    o[1] = av.y * sc + b4.y;
                    o[2] = av.z * sc + b4.z;
                    o[3] = av.w * sc + b4.w;
                    if (p < a.M)
                        *reinterpret_cast<half4_t*>(o2 + (long long)p * e.ldo2 + n) =
                            half4_t{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
                    if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                        for (int c = 0; c < 4; ++c) o[c] = o[c] >= 0.f ? o[c] : slope * o[c];
                    }
                }
                if constexpr (RES) {
                    const float4 r = h2f4(eres[cur][q]);
                    o[0] += r.x; o[1] += r.y; o[2] += r.z; o[3] += r.w;
                }
                if constexpr (MASK) {
                    const float4 m = h2f4(emask[cur][q]);
                    o[0] = m.x > 0.f ? o[0] : 0.f;
                    o[1] = m.y > 0.f ? o[1] : 0.f;
                    o[2] = m.z > 0.f ? o[2] : 0.f;
                    o[3] = m.w > 0.f ? o[3] : 0.f;
                } else if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
                }
                if constexpr (ACC) {
                    const float4 v = h2f4(eold[cur][q]);
                    o[0] += v.x; o[1] += v.y; o[2] += v.z; o[3] += v.w;
                }
                if (p < a.M)
                    *reinterpret_cast<half4_t*>(y + (long long)p * g.ldy + n) =
                        half4_t{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if constexpr (PM) {  // wave sums (xor shuffles), then the four waves' in a fixed order
        __shared__ float pred[4];
        for (int off = 32; off > 0; off >>= 1) pslope += __shfl_xor(pslope, off);
        if (lane == 0) pred[wave] = pslope;
        __syncthreads();
        if (tid == 0) e.out2[blockIdx.x] = (pred[0] + pred[1]) + (pred[2] + pred[3]);
    }
}

// ------------------------------------------------------------------------------------------------
// Streaming 1x1 conv on the bf16 MFMA with fp32 accuracy (bf16x6, round 5): the fp32 ResidualUnit / RBB 1x1 layers and
// their input-gradients, K = Ci in {64, 128}, Co = 32 * NT in {64, 128}, with the streamed epilogue operands the tiled
// kernel fuses: residual (F & 1), ReLU mask (F & 2), accumulate into y (F & 4). These layers are HBM-bound (at bs 16,
// 128^2: 64->128 + residual moves 335 MB for 17 GFLOP) and ran on the 64-row implicit-GEMM tiles at ~3.3 TB/s: every
// block loads, waits at a barrier, multiplies, then streams its epilogue, so HBM idles while the MFMAs run and the
// other way round. Here, as conv1x1_stream_kernel, each WAVE streams its own 32-pixel tiles with no barrier after the
// one-time weight staging, and EVERY streamed operand rolls a tile ahead in registers:
//   * W [Co][K] is split once per block into three bf16 planes in LDS (pitch K + 8: conflict-free ds_read_b128);
//   * the wave's X tile goes HBM -> registers in the MFMA B layout (lane (r, h): pixel p0 + r, channels 16s + 8h .. +7
//     for k-step s: two float4), is split into its three bf16 pieces in registers (bf6_split4), and each float4 is
//     reloaded for the wave's NEXT tile right after its split;
//   * the epilogue operands (residual, mask, old y: one float4 per (co tile t, quad q)) of co tile t + 1 are issued
//     when co tile t starts (two register sets), so each is in flight during a whole co tile's MFMAs;
//   * the 32-output co tiles are done one at a time (one accumulator; the X pieces re-split per co tile from the
//     raw fp32 registers — a few VALU ops against six MFMAs per k-step): what keeps every operand in flight within
//     the VGPR file without spills;
//   * C^T = W X^T: lane (r, h) holds pixel p0 + r, channels 32t + 8q + 4h .. +3 in acc[t][4q..4q+3] — float4 stores.
// Products: bf6_mfma (six bf16 cross products per 16-deep k-step, fp32 accumulation), the same arithmetic as every
// other bf16x6 kernel. Its waves fill the VGPR file exactly (4 x 128 or 2 x 256; see conv3x3_wres_bf6_kernel: a
// kernel that converts with v_cvt_pk_bf16_f32 and runs bf16 MFMAs must not leave room for other kernels' waves).
// VGPR allocation per wave: 256 (2 waves per SIMD, two epilogue operand sets). Measured (profiles/r5e_stream_b6.txt):
// 128 VGPRs / 4 waves per SIMD with one operand set was slower (256^2 64->64: 153 vs 143 us), and so was prefetching
// X two tiles and the operands a whole tile ahead (128^2 128->64: 50.4 vs 46.7 us, 64^2 64->128 +res 23.9 vs 20.1)
template <int NT, int KS, int F>
constexpr int stream_b6_vgprs() {
    return 256;
}
// the forms whose LDS (weight planes + epilogue scratch > 80 KB) admits one block per CU: one wave per SIMD
template <int NT, int KS>
constexpr bool stream_b6_one_block() {
    return NT == 6 || KS == 12 || (NT == 4 && KS == 8);
}
template <int NT, int KS, int F, bool CE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(stream_b6_one_block<NT, KS>() ? 1 : 512 / stream_b6_vgprs<NT, KS, F>())))
void conv1x1_stream_b6_kernel(const ConvArgs a) {
    constexpr int K = 16 * KS, KP = K + 8, CO = 32 * NT;
    constexpr bool RES = (F & 1) != 0, MASK = (F & 2) != 0, ACC = (F & 4) != 0;
    // SAB (F & 8, round 6): the HYRES_EPI_SA_BWD epilogue of MultiScaleRefine's fusion-1x1 input-gradient (64 -> 192 at
    // 256^2): o = (acc + aux0[p][0]) + (n == aux2[p] ? aux0[p][1] : 0), epi_store's order; no bias, no activation.
    // The per-pixel operands are loaded once per 32-pixel tile, the next tile's while this one multiplies
    constexpr bool SAB = (F & 8) != 0;
    static_assert(!SAB || (CE && !RES && !MASK), "SA_BWD: the coalesced epilogue, no residual / mask");
    // RS (F & 16, round 6): HYRES_EPI_ROWSCALE — MultiScaleRefine's fusion 1x1 in training with SpatialAttention folded
    // (192 -> 64 at 256^2, refine_ops.sa_fold_fusion): o = acc * aux1[p] + bias, then out2 (the pre-activation) and the
    // PReLU; the per-pixel scale is loaded once per tile like SAB's operands
    constexpr bool RS = (F & 16) != 0;
    static_assert(!RS || (CE && !RES && !MASK && !ACC && !SAB), "ROWSCALE: the coalesced epilogue, no other operand");
    // PM (F & 32, round 6, with SAB): HYRES_ACT_PRELU_MASK on output channels [0, 64) — MultiScaleRefine's scale-1
    // block writes PReLU(.) into multi[..., 0:64], so d multi's first 64 channels are that PReLU output's whole
    // gradient: o = pre > 0 ? o : slope * o (pre = aux1 [P][ld1]), sum_{pre <= 0} pre * o into this block's partial
    // (out2[block]); the slope gradient (res, ADDED) by prelu_slope_sum_kernel after the launch
    constexpr bool PM = (F & 32) != 0;
    static_assert(!PM || (SAB && !ACC && NT >= 2), "PReLU mask: the SA_BWD form without accumulate");
    constexpr int WPL = CO * KP;  // bf16 per weight plane
    __shared__ __attribute__((aligned(16))) __bf16 Ws[3 * WPL];
    __shared__ __attribute__((aligned(16))) float bs[CO];
    // CE: per-wave epilogue scratch, one 32 x 32 co tile (pitch 36 floats: the MFMA-layout float4 writes of 16 lanes
    // land on 16 distinct 4-bank groups)
    constexpr int EP = 36;
    __shared__ __attribute__((aligned(16))) float Es[CE ? 4 * 32 * EP : 4];
    // exactly 2 or 4 waves' worth of VGPRs: no room for another kernel's wave on these SIMDs. NT = 6 (the 64 -> 192
    // SA_BWD form, 102 KB of LDS) and KS = 12 (the 192 -> 64 ROWSCALE form, 95 KB) admit one block per CU, i.e. one
    // wave per SIMD — they take all 512 registers
    if constexpr (stream_b6_one_block<NT, KS>()) asm volatile("" ::: "v255", "a255");
    else if constexpr (stream_b6_vgprs<NT, KS, F>() == 128) asm volatile("" ::: "v127");
    else asm volatile("" ::: "v255");
    const hyres_conv_geom& g = a.g;
    const hyres_epilogue& e = a.e;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    for (int i = tid; i < CO * (K / 4); i += 256) {
        const int co = i / (K / 4), k4 = i - co * (K / 4);
        bf16x4_t h, m, l;
        bf6_split4(ld4(a.w2 + (long long)co * a.ldw + 4 * k4), h, m, l);
        const int o = co * KP + 4 * k4;
        *reinterpret_cast<bf16x4_t*>(&Ws[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&Ws[WPL + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&Ws[2 * WPL + o]) = l;
    }
    for (int i = tid; i < CO; i += 256) bs[i] = e.bias ? e.bias[i] : 0.f;
    const float slope = (e.act == HYRES_ACT_PRELU) ? e.slope[0] : 0.f;
    __syncthreads();

    const long long npix = a.M;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_res = opnd_rsrc(RES ? e.res : nullptr, npix * e.ldres * 4);
    const __amdgpu_buffer_rsrc_t r_mask = opnd_rsrc(MASK ? e.aux0 : nullptr, npix * e.ld0 * 4);
    const __amdgpu_buffer_rsrc_t r_old = opnd_rsrc(ACC ? a.y : nullptr, npix * g.ldy * 4);
    constexpr int OOR = (int)0x80000000;
    const int ntile = (a.M + 31) / 32;
    const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    auto xoff = [&](int tile, int s, int u) -> int {
        const int p = tile * 32 + lr;
        return (tile < ntile && p < a.M) ? (p * g.ldx + 16 * s + 8 * lh + 4 * u) * 4 : OOR;
    };
    // epilogue operand q of co tile t. MFMA layout: lane (r, h) -> pixel p0 + r, channels 32t + 8q + 4h (one wave
    // instruction touches 32 pixel rows x 32 B). CE (coalesced): lane l -> pixel p0 + (l >> 3) + 8q, channels
    // 32t + 4 (l & 7) (one instruction = 8 pixel rows x 128 B contiguous; profiles/r5h_access_probe.txt: the 32-B
    // shape caps a read+write stream at ~3.0-3.5 TB/s, full rows reach 5.3-5.9)
    const int cr = lane >> 3, cc = 4 * (lane & 7);
    auto ooff = [&](int tile, int ld, int t, int q) -> int {
        if constexpr (CE) {
            const int p = tile * 32 + cr + 8 * q;
            return (tile < ntile && p < a.M) ? (p * ld + 32 * t + cc) * 4 : OOR;
        } else {
            const int p = tile * 32 + lr;
            return (tile < ntile && p < a.M) ? (p * ld + 32 * t + 8 * q + 4 * lh) * 4 : OOR;
        }
    };
    static_assert(NT % 2 == 0, "the epilogue operands alternate between two register sets per co tile");
    // epilogue operands: with two register sets (256-VGPR variants) co tile t's are in set t & 1 while co tile t + 1's
    // (or the next tile's co tile 0) are in flight in the other, issued when co tile t starts; with one set (128-VGPR
    // variants, 4 waves per SIMD) the next co tile's are issued right after this one's epilogue
    constexpr int SETS = stream_b6_vgprs<NT, KS, F>() == 128 ? 1 : 2;
    float4 xv[KS][2];
    float4 eres[RES ? SETS : 1][4], emask[MASK ? SETS : 1][4], eold[ACC ? SETS : 1][4];
    float4 epre[PM ? SETS : 1][4];
    const __amdgpu_buffer_rsrc_t r_pm = opnd_rsrc(PM ? e.aux1 : nullptr, npix * e.ld1 * 4);
    const float pslope_a = PM ? e.slope[0] : 0.f;
    float pslope = 0.f;
    // SAB: this tile's (d mean / C, d max) and argmax per epilogue row q, and the next tile's in flight
    float2 sg[SAB ? 4 : 1], sgn[SAB ? 4 : 1];
    int si[SAB ? 4 : 1], sin_[SAB ? 4 : 1];
    const __amdgpu_buffer_rsrc_t r_sg = opnd_rsrc(SAB ? e.aux0 : nullptr, npix * e.ld0 * 4);
    const __amdgpu_buffer_rsrc_t r_si = opnd_rsrc(SAB ? e.aux2 : nullptr, npix * 4);
    auto load_sab = [&](int tile, float2 (&g2)[SAB ? 4 : 1], int (&i1)[SAB ? 4 : 1]) {
        if constexpr (SAB) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = tile * 32 + cr + 8 * q;
                const bool ok = tile < ntile && p < a.M;
                g2[q] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r_sg, ok ? p * e.ld0 * 4 : OOR, 0, 0));
                i1[q] = __builtin_bit_cast(int, __builtin_amdgcn_raw_buffer_load_b32(r_si, ok ? p * 4 : OOR, 0, 0));
            }
        }
    };
    float rsc[RS ? 4 : 1], rscn[RS ? 4 : 1];
    const __amdgpu_buffer_rsrc_t r_rs = opnd_rsrc(RS ? e.aux1 : nullptr, npix * e.ld1 * 4);
    auto load_rs = [&](int tile, float (&r1)[RS ? 4 : 1]) {
        if constexpr (RS) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int p = tile * 32 + cr + 8 * q;
                const bool ok = tile < ntile && p < a.M;
                r1[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r_rs, ok ? p * e.ld1 * 4 : OOR, 0, 0));
            }
        }
    };
    auto load_epi = [&](int tile, int t, int set) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (RES) eres[set][q] = bload4(r_res, ooff(tile, e.ldres, t, q));
            if constexpr (MASK) emask[set][q] = bload4(r_mask, ooff(tile, e.ld0, t, q));
            if constexpr (ACC) eold[set][q] = bload4(r_old, ooff(tile, g.ldy, t, q));
            if constexpr (PM) epre[set][q] = bload4(r_pm, t < 2 ? ooff(tile, e.ld1, t, q) : OOR);
        }
    };
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) xv[s][u] = bload4(xr, xoff(gw, s, u));
    load_epi(gw, 0, 0);
    load_sab(gw, sg, si);
    load_rs(gw, rsc);
    for (int tile = gw; tile < ntile; tile += nw) {
        load_sab(tile + nw, sgn, sin_);
        load_rs(tile + nw, rscn);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int cur = SETS == 2 ? (t & 1) : 0;
            if constexpr (SETS == 2) {
                if (t + 1 < NT) load_epi(tile, t + 1, cur ^ 1);
                else load_epi(tile + nw, 0, cur ^ 1);
            }
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                // the X pieces are re-split per co tile (a few VALU ops) rather than held for all k-steps
                // (the empty asm makes each co tile's split its own computation: common-subexpression elimination
                // would otherwise keep every k-step's pieces live across all co tiles and spill)
                typedef float f32x4v_t __attribute__((ext_vector_type(4)));
                f32x4v_t v0 = __builtin_bit_cast(f32x4v_t, xv[s][0]), v1 = __builtin_bit_cast(f32x4v_t, xv[s][1]);
                asm volatile("" : "+v"(v0), "+v"(v1));
                const float4 x0 = __builtin_bit_cast(float4, v0), x1 = __builtin_bit_cast(float4, v1);
                bf16x4_t h0, m0, l0, h1, m1, l1;
                bf6_split4(x0, h0, m0, l0);
                bf6_split4(x1, h1, m1, l1);
                const bf16x8_t xb[3] = {__builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7),
                                        __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7),
                                        __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7)};
                if (t == NT - 1) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) xv[s][u] = bload4(xr, xoff(tile + nw, s, u));  // the next tile's X
                }
                const int o = (32 * t + lr) * KP + 16 * s + 8 * lh;
                const bf16x8_t wb[3] = {*reinterpret_cast<const bf16x8_t*>(&Ws[o]),
                                        *reinterpret_cast<const bf16x8_t*>(&Ws[WPL + o]),
                                        *reinterpret_cast<const bf16x8_t*>(&Ws[2 * WPL + o])};
                acc = bf6_mfma(wb, xb, acc);
            }
            float* const es = Es + wave * 32 * EP;
            if constexpr (CE) {
                // the accumulator goes to the wave's scratch in the MFMA layout and comes back as pixel rows
                // (LDS instructions of one wave execute in order: the fences only keep the compiler from moving the
                // previous co tile's reads past these writes or these writes past the reads below)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4*>(&es[lr * EP + 8 * q + 4 * lh]) =
                        make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = CE ? 32 * t + cc : 32 * t + 8 * q + 4 * lh;
                const float4 b4 = *reinterpret_cast<const float4*>(&bs[n]);
                float4 av;
                if constexpr (CE) av = *reinterpret_cast<const float4*>(&es[(cr + 8 * q) * EP + cc]);
                else av = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                const int p = CE ? tile * 32 + cr + 8 * q : tile * 32 + lr;
                const bool pok = p < a.M;
                float o[4] = {av.x + b4.x, av.y + b4.y, av.z + b4.z, av.w + b4.w};
                if constexpr (SAB) {
                    const float av4[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = av4[c] + sg[q].x + (n + c == si[q] ? sg[q].y : 0.f);
                }
                if constexpr (PM) {
                    if (t < 2 && pok) {  // as prelu_bwd4_kernel on the stored gradient
                        const float pv[4] = {epre[cur][q].x, epre[cur][q].y, epre[cur][q].z, epre[cur][q].w};
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            if (!(pv[c] > 0.f)) pslope += pv[c] * o[c];
                            o[c] = pv[c] > 0.f ? o[c] : pslope_a * o[c];
                        }
                    }
                }
                if constexpr (RS) {  // epi_store4's ROWSCALE: (acc * scale) + bias
                    o[0] = av.x * rsc[q] + b4.x;
                    o[1] = av.y * rsc[q] + b4.y;
                    o[2] = av.z * rsc[q] + b4.z;
                    o[3] = av.w * rsc[q] + b4.w;
                }
                if constexpr (RES) {
                    o[0] += eres[cur][q].x; o[1] += eres[cur][q].y; o[2] += eres[cur][q].z; o[3] += eres[cur][q].w;
                }
                if constexpr (!PM) {  // (PM: out2 holds the slope partials)
                    if (pok && e.out2) st4(e.out2 + (long long)p * e.ldo2 + n, make_float4(o[0], o[1], o[2], o[3]));
                }
                if constexpr (MASK) {
                    o[0] = emask[cur][q].x > 0.f ? o[0] : 0.f;
                    o[1] = emask[cur][q].y > 0.f ? o[1] : 0.f;
                    o[2] = emask[cur][q].z > 0.f ? o[2] : 0.f;
                    o[3] = emask[cur][q].w > 0.f ? o[3] : 0.f;
                } else if (e.act == HYRES_ACT_RELU) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c], 0.f);
                } else if (e.act == HYRES_ACT_PRELU) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[c] = o[c] >= 0.f ? o[c] : slope * o[c];
                }
                if constexpr (ACC) {
                    o[0] += eold[cur][q].x; o[1] += eold[cur][q].y; o[2] += eold[cur][q].z; o[3] += eold[cur][q].w;
                }
                if (pok) st4(a.y + (long long)p * g.ldy + n, make_float4(o[0], o[1], o[2], o[3]));
            }
            if constexpr (SETS == 1) {
                if (t + 1 < NT) load_epi(tile, t + 1, 0);
                else load_epi(tile + nw, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the next co tile's LDS reads and splits out of this one
        }
        if constexpr (SAB) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                sg[q] = sgn[q];
                si[q] = sin_[q];
            }
        }
        if constexpr (RS) {
#pragma unroll
            for (int q = 0; q < 4; ++q) rsc[q] = rscn[q];
        }
    }
    if constexpr (PM) {  // wave sums (xor shuffles), then the four waves' in a fixed order
        __shared__ float pred[4];
        for (int off = 32; off > 0; off >>= 1) pslope += __shfl_xor(pslope, off);
        if (lane == 0) pred[wave] = pslope;
        __syncthreads();
        if (tid == 0) e.out2[blockIdx.x] = (pred[0] + pred[1]) + (pred[2] + pred[3]);
    }
}

// split-K reduction + epilogue: one thread per (phase, m, n)
template <bool H>
__global__ void conv_splitk_reduce_kernel(const ConvArgs a) {
    const hyres_conv_geom& g = a.g;
    const long long per_phase = (long long)a.M * g.Co;
    const long long total = per_phase * g.nphase;
    const int HqWq = g.Hq * g.Wq;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int phase = (int)(idx / per_phase);
        const long long r = idx - phase * per_phase;
        const int m = (int)(r / g.Co);
        const int n = (int)(r - (long long)m * g.Co);
        float v = 0.f;
        for (int s = 0; s < a.nsplit; ++s) v += a.slab[((long long)(s * g.nphase + phase) * a.M + m) * g.Co + n];
        const int b = m / HqWq;
        const int rr = m - b * HqWq;
        const int i = rr / g.Wq, j = rr - (rr / g.Wq) * g.Wq;
        const long long pix = (long long)(b * g.Ho + i * g.osh + g.oph[phase]) * g.Wo + j * g.osw + g.opw[phase];
        epi_store<H, true>(a.e, a.y, g.ldy, pix, n, v, epi_channel(a.e, n));
    }
}

// float4 variant (vec4 launches): 4 channels per thread, split loads unrolled, float4 epilogue
template <bool H>
__global__ __launch_bounds__(256) void conv_splitk_reduce4_kernel(const ConvArgs a) {
    const hyres_conv_geom& g = a.g;
    const int C4 = g.Co >> 2;
    const long long per_phase = (long long)a.M * C4;
    const long long total = per_phase * g.nphase;
    const long long sstride = (long long)g.nphase * a.M * g.Co;
    const int HqWq = g.Hq * g.Wq;
    const float slope = (a.e.act == HYRES_ACT_PRELU) ? a.e.slope[0] : 0.f;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int phase = (int)(idx / per_phase);
        const long long r = idx - phase * per_phase;
        const int m = (int)(r / C4);
        const int n = 4 * (int)(r - (long long)m * C4);
        const float* sp = a.slab + ((long long)phase * a.M + m) * g.Co + n;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
        for (int s = 0; s < a.nsplit; ++s) {
            const float4 u = ld4(sp + s * sstride);
            v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        const int b = m / HqWq;
        const int rr = m - b * HqWq;
        const int i = rr / g.Wq, j = rr - (rr / g.Wq) * g.Wq;
        const long long pix = (long long)(b * g.Ho + i * g.osh + g.oph[phase]) * g.Wo + j * g.osw + g.opw[phase];
        epi_store4<H, true>(a.e, a.y, g.ldy, pix, n, v, slope);
    }
}

// ------------------------------------------------------------------------------------------------
// Narrow output (Co <= 4: the 3-channel image-side layers — g_s's last deconv 128->3, MultiScaleRefine's
// conv 64->3 and the input-gradient of its conv 3->64). A 32-wide MFMA column tile would be >90% padding,
// so these run on the VALU. Each 16-lane group owns one output pixel: lane l reads channels
// [64s + 4l, +4) of every tap (a wave reads 4 adjacent pixels = contiguous NHWC rows, coalesced), keeps
// CO partial sums, and the group folds them with 4 xor-shuffles. The phase's weights are staged once per
// block in LDS as [tap][co][Ci] (a lane's float4 reads are consecutive across the group: conflict-free).
// HBM traffic = the input once (tap re-reads hit L1/L2) + CO outputs.
// ------------------------------------------------------------------------------------------------
constexpr int NARROW_PIX = 256;      // output pixels per block
constexpr int NARROW_WLDS = 8192;    // floats of staged weights (ntap * CO * Ci)

template <int CO, int S, bool XH = false>
__global__ __launch_bounds__(256) void conv_narrow_kernel(const ConvArgs a) {
    __shared__ __attribute__((aligned(16))) float Ws[NARROW_WLDS];
    __shared__ int2 tapoff[HYRES_MAX_TAPS];
    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x;
    const int phase = blockIdx.y;
    const int ntap = g.ntap[phase], tap0 = g.tap0[phase];
    constexpr int CI = 64 * S;
    for (int idx = tid; idx < ntap * CO * (CI / 4); idx += 256) {
        const int c4 = idx % (CI / 4);
        const int r = idx / (CI / 4);
        const int co = r % CO, t = r / CO;
        *reinterpret_cast<float4*>(&Ws[4 * idx]) = ld4(a.w2 + (long long)co * a.ldw + (tap0 + t) * CI + 4 * c4);
    }
    for (int i = tid; i < ntap; i += 256) tapoff[i] = make_int2(g.dh[tap0 + i], g.dw[tap0 + i]);
    __syncthreads();

    const int HqWq = g.Hq * g.Wq;
    // XCD-aware pixel-tile order (as conv_fwd_kernel): neighbouring rows' tiles, which share the 3x3
    // halo, run on one XCD's L2
    int bx = blockIdx.x;
    if (a.xcd) {
        const int nb = gridDim.x, q = nb >> 3, r = nb & 7, x = bx & 7;
        bx = x * q + min(x, r) + (bx >> 3);
    }
    const int b0 = (bx * NARROW_PIX) / HqWq;
    constexpr int XES = XH ? 2 : 4;  // X element bytes (XH: fp16 activations, autocast inference)
    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const long long xrem = ((long long)g.B - b0) * img * XES;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(a.x) + (long long)b0 * img * XES), (short)0,
        (int)(xrem < 0x7FFFFFF0LL ? xrem : 0x7FFFFFF0LL), 0x00020000);
    const int l16 = tid & 15, slot = tid >> 4;  // 16 pixel slots per block pass
    for (int it = 0; it < NARROW_PIX / 16; ++it) {
        const int m = bx * NARROW_PIX + it * 16 + slot;
        const bool ok = m < a.M;
        const int mm = ok ? m : 0;
        const int b = mm / HqWq;
        const int r = mm - b * HqWq;
        const int i = r / g.Wq, j = r - (r / g.Wq) * g.Wq;
        const int base = (int)((b - b0) * img);
        float acc[CO];
#pragma unroll
        for (int c = 0; c < CO; ++c) acc[c] = 0.f;
        // taps in groups of TG: all TG input rows are requested before the first FMA (a loop of one load
        // then its FMAs serialised ~9 memory latencies per output pixel: 254 us -> see DESIGN §4)
        constexpr int TG = 9;
        for (int t0 = 0; t0 < ntap; t0 += TG) {
            std::conditional_t<XH, half4_t, float4> xv[TG][S];  // fp16 X: converted at the FMAs
#pragma unroll
            for (int u = 0; u < TG; ++u) {
                const int t = t0 + u;
                const int2 o = tapoff[t < ntap ? t : 0];
                const int ih = i * g.ish + o.x, iw = j * g.isw + o.y;
                const bool in = ok && t < ntap && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
                const int off = in ? (base + (ih * g.Wi + iw) * g.ldx + 4 * l16) * XES : (int)0x80000000;
#pragma unroll
                for (int s2 = 0; s2 < S; ++s2) {
                    if constexpr (XH) {
                        xv[u][s2] = __builtin_bit_cast(
                            half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, in ? off + 128 * s2 : off, 0, 0));
                    } else {
                        xv[u][s2] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                  xr, in ? off + 256 * s2 : off, 0, 0));
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < TG; ++u) {
                const int t = t0 + u;
                if (t >= ntap) break;
#pragma unroll
                for (int s2 = 0; s2 < S; ++s2) {
                    float4 xf;
                    if constexpr (XH) xf = make_float4((float)xv[u][s2].x, (float)xv[u][s2].y, (float)xv[u][s2].z,
                                                       (float)xv[u][s2].w);
                    else xf = xv[u][s2];
#pragma unroll
                    for (int co = 0; co < CO; ++co) {
                        const float4 w =
                            *reinterpret_cast<const float4*>(&Ws[(t * CO + co) * CI + 64 * s2 + 4 * l16]);
                        acc[co] = fmaf(xf.x, w.x, acc[co]);
                        acc[co] = fmaf(xf.y, w.y, acc[co]);
                        acc[co] = fmaf(xf.z, w.z, acc[co]);
                        acc[co] = fmaf(xf.w, w.w, acc[co]);
                    }
                }
            }
        }
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            float v = acc[co];
            v += __shfl_xor(v, 8);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 1);
            acc[co] = v;
        }
        float v = acc[0];
#pragma unroll
        for (int co = 1; co < CO; ++co) v = l16 == co ? acc[co] : v;
        if (ok && l16 < CO) {
            const long long pix = (long long)(b * g.Ho + i * g.osh + g.oph[phase]) * g.Wo + j * g.osw + g.opw[phase];
            epi_store(a.e, a.y, g.ldy, pix, l16, v, epi_channel(a.e, l16));
        }
    }
}

// Co <= 4 with register blocking along W (round 5). conv_narrow_kernel is VALU-bound, not memory-bound: on
// MultiScaleRefine's 3x3 64 -> 3 at bs16 256^2 (215 us) the PMC passes read 270 MB (1.0x the input) while each 4-pixel
// wave pass issues ~307 VALU instructions of which 108 are the FMAs — the rest is per-pixel index decode, 9 tap
// addresses and bounds, and the fold (profiles/r5u_narrow_pmc.txt); its per-pixel weight re-reads add 27
// ds_read_b128. Here a lane group (Ci / 4 lanes, 4 channels each) computes a STRIP of 4 consecutive base pixels of
// one row: the phase's taps form a kh x kw grid of consecutive (dh, dw) offsets (every 3x3 conv and every phase of
// the 5x5 stride-2 transposed conv: checked on the host), so the strip needs kh x (kw + 3) input pixels, loaded once
// (<= 18 float4 per lane) and each reused by up to 3 taps; the weights of the phase live in VGPRs (9 taps x Co float4,
// zero for absent taps) for the whole launch; index decode and addressing once per strip; the 4 x Co partial sums
// folded with xor-shuffles and stored by lanes (r, co). Needs Wq % 4 == 0 (strips never cross a row).
// Same products per output as conv_narrow_kernel, different summation order (fp32 FMAs).
constexpr int NSTRIP = 4;
template <int CO, int S, bool XH = false>
__global__ __launch_bounds__(256) void conv_narrow_strip_kernel(const ConvArgs a) {
    constexpr int CI = 64 * S, LP = 16 * S, GROUPS = 256 / LP, XES = XH ? 2 : 4;
    constexpr int STRIPS = NARROW_PIX / NSTRIP, PASSES = STRIPS / GROUPS;
    const hyres_conv_geom& g = a.g;
    const int tid = threadIdx.x, lq = tid % LP, grp = tid / LP;
    const int phase = blockIdx.y;
    const int ntap = g.ntap[phase], tap0 = g.tap0[phase];
    // the phase's taps as a kh x kw grid listed row-major with steps of +-1 in dh and dw (host-checked: the conv's
    // taps ascend, the transposed conv's phases descend); (r, c) below count from the grid's smallest (dh, dw)
    const int da = g.dh[tap0], wa = g.dw[tap0], dz = g.dh[tap0 + ntap - 1], wz = g.dw[tap0 + ntap - 1];
    const int kh = (da > dz ? da - dz : dz - da) + 1, kw = (wa > wz ? wa - wz : wz - wa) + 1;
    const int dh0 = min(da, dz), dw0 = min(wa, wz);
    const bool rh = da > dz, rw = wa > wz;  // descending rows / columns
    float4 w[3][3][CO];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int t = (rh ? kh - 1 - r : r) * kw + (rw ? kw - 1 - c : c);
#pragma unroll
            for (int co = 0; co < CO; ++co)
                w[r][c][co] = (r < kh && c < kw) ? ld4(a.w2 + (long long)co * a.ldw + (tap0 + t) * CI + 4 * lq)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    const int HqWq = g.Hq * g.Wq;
    int bx = blockIdx.x;
    if (a.xcd) {  // XCD-aware pixel-tile order, as conv_narrow_kernel
        const int nb = gridDim.x, q = nb >> 3, r = nb & 7, x = bx & 7;
        bx = x * q + min(x, r) + (bx >> 3);
    }
    const int b0 = (bx * NARROW_PIX) / HqWq;
    const long long img = (long long)g.Hi * g.Wi * g.ldx;
    const long long xrem = ((long long)g.B - b0) * img * XES;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(a.x) + (long long)b0 * img * XES), (short)0,
        (int)(xrem < 0x7FFFFFF0LL ? xrem : 0x7FFFFFF0LL), 0x00020000);
    for (int it = 0; it < PASSES; ++it) {
        const int m = bx * NARROW_PIX + (it * GROUPS + grp) * NSTRIP;  // first pixel of the strip
        const bool ok = m < a.M;
        const int mm = ok ? m : 0;
        const int b = mm / HqWq, rr = mm - b * HqWq;
        const int i = rr / g.Wq, j = rr - (rr / g.Wq) * g.Wq;
        const int base = (int)((b - b0) * img);
        const int ih0 = i * g.ish + dh0, iw0 = j * g.isw + dw0;
        std::conditional_t<XH, half4_t, float4> xv[3][NSTRIP + 2];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < NSTRIP + 2; ++c) {
                const int ih = ih0 + r, iw = iw0 + c;
                const bool in = ok && r < kh && c < kw + NSTRIP - 1 && (unsigned)ih < (unsigned)g.Hi &&
                                (unsigned)iw < (unsigned)g.Wi;
                const int off = in ? (base + (ih * g.Wi + iw) * g.ldx + 4 * lq) * XES : (int)0x80000000;
                if constexpr (XH) xv[r][c] = __builtin_bit_cast(half4_t, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
                else xv[r][c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            }
        float acc[NSTRIP][CO];
#pragma unroll
        for (int p = 0; p < NSTRIP; ++p)
#pragma unroll
            for (int co = 0; co < CO; ++co) acc[p][co] = 0.f;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < NSTRIP + 2; ++c) {
                float4 xf;
                if constexpr (XH) xf = make_float4((float)xv[r][c].x, (float)xv[r][c].y, (float)xv[r][c].z, (float)xv[r][c].w);
                else xf = xv[r][c];
#pragma unroll
                for (int p = 0; p < NSTRIP; ++p) {
                    const int t = c - p;  // this input column is tap column t of strip pixel p
                    if (t < 0 || t > 2) continue;
#pragma unroll
                    for (int co = 0; co < CO; ++co) {
                        acc[p][co] = fmaf(xf.x, w[r][t][co].x, acc[p][co]);
                        acc[p][co] = fmaf(xf.y, w[r][t][co].y, acc[p][co]);
                        acc[p][co] = fmaf(xf.z, w[r][t][co].z, acc[p][co]);
                        acc[p][co] = fmaf(xf.w, w[r][t][co].w, acc[p][co]);
                    }
                }
            }
#pragma unroll
        for (int p = 0; p < NSTRIP; ++p)
#pragma unroll
            for (int co = 0; co < CO; ++co) {
                float v = acc[p][co];
#pragma unroll
                for (int off = LP / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
                acc[p][co] = v;
            }
        // lane q < NSTRIP * CO stores pixel q / CO, channel q % CO
        float v = 0.f;
#pragma unroll
        for (int p = 0; p < NSTRIP; ++p)
#pragma unroll
            for (int co = 0; co < CO; ++co) v = lq == p * CO + co ? acc[p][co] : v;
        const int sp = lq / CO, sc = lq - sp * CO;
        if (ok && lq < NSTRIP * CO && m + sp < a.M) {
            const long long pix = (long long)(b * g.Ho + i * g.osh + g.oph[phase]) * g.Wo + (j + sp) * g.osw + g.opw[phase];
            epi_store(a.e, a.y, g.ldy, pix, sc, v, epi_channel(a.e, sc));
        }
    }
}

// the strip kernel's host-side conditions: every phase's taps a row-major grid of consecutive offsets, <= 3 x 3,
// unit input stride along W, strips inside rows
static bool narrow_strip_ok(const hyres_conv_geom* g) {
    if (g_tune[13] == 0 || g->Wq % NSTRIP != 0 || g->isw != 1) return false;
    for (int p = 0; p < g->nphase; ++p) {
        const int n = g->ntap[p], t0 = g->tap0[p];
        if (n < 1) return false;
        const int da = g->dh[t0], wa = g->dw[t0], dz = g->dh[t0 + n - 1], wz = g->dw[t0 + n - 1];
        const int kh = std::abs(da - dz) + 1, kw = std::abs(wa - wz) + 1;
        const int sh = dz >= da ? 1 : -1, sw = wz >= wa ? 1 : -1;
        if (kh > 3 || kw > 3 || kh * kw != n) return false;
        for (int t = 0; t < n; ++t)
            if (g->dh[t0 + t] != da + sh * (t / kw) || g->dw[t0 + t] != wa + sw * (t % kw)) return false;
    }
    return true;
}

static bool narrow_ok(const hyres_conv_geom* g) {
    if (g->Co > 4 || (g->Ci != 64 && g->Ci != 128)) return false;
    int maxtap = 0;
    for (int p = 0; p < g->nphase; ++p) maxtap = std::max(maxtap, g->ntap[p]);
    return maxtap * g->Co * g->Ci <= NARROW_WLDS;
}

template <int CO>
static void launch_narrow(const ConvArgs& a, dim3 grid, hipStream_t st) {
    if (narrow_strip_ok(&a.g)) {  // hyres_conv_tuning key 13 (default 1)
        const bool h = (a.e.io_f16 & HYRES_IO_X16) != 0;
        if (a.g.Ci == 64) {
            if (h) hipLaunchKernelGGL((conv_narrow_strip_kernel<CO, 1, true>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_narrow_strip_kernel<CO, 1>), grid, dim3(256), 0, st, a);
        } else {
            if (h) hipLaunchKernelGGL((conv_narrow_strip_kernel<CO, 2, true>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_narrow_strip_kernel<CO, 2>), grid, dim3(256), 0, st, a);
        }
        return;
    }
    if (a.e.io_f16 & HYRES_IO_X16) {
        if (a.g.Ci == 64) hipLaunchKernelGGL((conv_narrow_kernel<CO, 1, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv_narrow_kernel<CO, 2, true>), grid, dim3(256), 0, st, a);
        return;
    }
    if (a.g.Ci == 64) hipLaunchKernelGGL((conv_narrow_kernel<CO, 1>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_narrow_kernel<CO, 2>), grid, dim3(256), 0, st, a);
}


// ------------------------------------------------------------------------------------------------
// weight re-layout
// ------------------------------------------------------------------------------------------------
struct PrepArgs {
    const float* w;
    float* w2;
    const float* mask;
    int mode, rows, cols, ntaps, KH, KW, Ci, Co;
    int kh[HYRES_MAX_TAPS], kw[HYRES_MAX_TAPS];
};

__device__ __forceinline__ float prep_value(const PrepArgs& a, long long idx) {
    const int c = (int)(idx % a.cols);
    const long long rt = idx / a.cols;
    const int t = (int)(rt % a.ntaps);
    const int r = (int)(rt / a.ntaps);
    const int kh = a.kh[t], kw = a.kw[t];
    long long src;
    switch (a.mode) {
        case HYRES_WPREP_CONV: src = (((long long)r * a.Ci + c) * a.KH + kh) * a.KW + kw; break;
        case HYRES_WPREP_CONV_DGRAD: src = (((long long)c * a.Ci + r) * a.KH + kh) * a.KW + kw; break;
        case HYRES_WPREP_DECONV: src = (((long long)c * a.Co + r) * a.KH + kh) * a.KW + kw; break;
        default: src = (((long long)r * a.Co + c) * a.KH + kh) * a.KW + kw; break;
    }
    float v = a.w[src];
    if (a.mask) v *= a.mask[src];
    return v;
}

struct PrepDesc {
    PrepArgs a;
    long long begin, count;
};

// grid (chunks, n descriptors): blockIdx.y picks the descriptor (block-uniform: its fields are scalar
// loads), blocks stride over its outputs with 32-bit index math
__global__ __launch_bounds__(256) void weight_prep_batch_kernel(const PrepDesc* d, int n, long long total) {
    const PrepArgs& a = d[blockIdx.y].a;
    const int count = (int)d[blockIdx.y].count;
    const int tc = a.ntaps * a.cols;
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < count; idx += gridDim.x * 256) {
        const int r = idx / tc;
        const int rem = idx - r * tc;
        const int t = rem / a.cols;
        const int c = rem - t * a.cols;
        const int kh = a.kh[t], kw = a.kw[t];
        int src;
        switch (a.mode) {
            case HYRES_WPREP_CONV: src = ((r * a.Ci + c) * a.KH + kh) * a.KW + kw; break;
            case HYRES_WPREP_CONV_DGRAD: src = ((c * a.Ci + r) * a.KH + kh) * a.KW + kw; break;
            case HYRES_WPREP_DECONV: src = ((c * a.Co + r) * a.KH + kh) * a.KW + kw; break;
            default: src = ((r * a.Co + c) * a.KH + kh) * a.KW + kw; break;
        }
        a.w2[idx] = a.w[src];
    }
}

__global__ void weight_prep_kernel(const PrepArgs a) {
    const long long total = (long long)a.rows * a.ntaps * a.cols;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(idx % a.cols);
        const long long rt = idx / a.cols;
        const int t = (int)(rt % a.ntaps);
        const int r = (int)(rt / a.ntaps);
        const int kh = a.kh[t], kw = a.kw[t];
        long long src;
        switch (a.mode) {
            case HYRES_WPREP_CONV:  // W[Co][Ci][KH][KW]; r = co, c = ci
                src = (((long long)r * a.Ci + c) * a.KH + kh) * a.KW + kw; break;
            case HYRES_WPREP_CONV_DGRAD:  // r = ci, c = co
                src = (((long long)c * a.Ci + r) * a.KH + kh) * a.KW + kw; break;
            case HYRES_WPREP_DECONV:  // W[Ci][Co][K][K]; r = co, c = ci
                src = (((long long)c * a.Co + r) * a.KH + kh) * a.KW + kw; break;
            default:  // DECONV_DGRAD: r = ci, c = co
                src = (((long long)r * a.Co + c) * a.KH + kh) * a.KW + kw; break;
        }
        float v = a.w[src];
        if (a.mask) v *= a.mask[src];
        a.w2[idx] = v;
    }
}



// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
template <int TM, int TN, int WM_, int WN_>
static int launch_fwd(const ConvArgs& a, int mode, hipStream_t st) {
    constexpr int BM = 32 * TM * WM_, BN = 32 * TN * WN_;
    dim3 grid(ceil_div(a.M, BM), ceil_div(a.g.Co, BN), a.g.nphase * a.nsplit);
    if (a.xcd) grid = dim3(grid.x * grid.y, 1, grid.z);
    if (a.e.io_f16 & 3) {
        const int io = a.e.io_f16 & 3;
#define HY_H(MODE_, SPLIT_)                                                                                       \
    {                                                                                                            \
        if (io == 1) hipLaunchKernelGGL((conv_fwd_h_kernel<TM, TN, WM_, WN_, MODE_, SPLIT_, 1>), grid, dim3(256), 0, st, a); \
        else if (io == 2) hipLaunchKernelGGL((conv_fwd_h_kernel<TM, TN, WM_, WN_, MODE_, SPLIT_, 2>), grid, dim3(256), 0, st, a); \
        else hipLaunchKernelGGL((conv_fwd_h_kernel<TM, TN, WM_, WN_, MODE_, SPLIT_, 3>), grid, dim3(256), 0, st, a); \
    }
        if (mode == 2) {
            if (a.nsplit > 1) hipLaunchKernelGGL((conv_fwd_h_kernel<TM, TN, WM_, WN_, 2, true, 2>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_h_kernel<TM, TN, WM_, WN_, 2, false, 2>), grid, dim3(256), 0, st, a);
        } else if (a.nsplit > 1) {
            if (mode == 0) HY_H(0, true) else HY_H(1, true)
        } else {
            if (mode == 0) HY_H(0, false) else HY_H(1, false)
        }
#undef HY_H
        return HY_LAUNCH_CHECK("conv_fwd_h_kernel");
    }
    if (a.e.f16_operands && mode != 2) {
        if (a.nsplit > 1) {
            if (mode == 0) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 0, true, true>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 1, true, true>), grid, dim3(256), 0, st, a);
        } else {
            if (mode == 0) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 0, false, true>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 1, false, true>), grid, dim3(256), 0, st, a);
        }
        return HY_LAUNCH_CHECK("conv_fwd_kernel(f16)");
    }
    if (g_tune[7] == 1 && mode != 2) {  // fp32 GEMM on the bf16 MFMA (bf16x6)
        if constexpr (TM == 1 && TN == 1 && WM_ == 2 && WN_ == 2) {
            // double-buffered staging (key 20 = 1, or -1: on for the <= 16384-pixel grids). Isolated it wins at 32^2
            // (3x3 96 -> 96 39.6 -> 37.3 us, 1x1 192 -> 96 13.9 -> 13.1 us) and loses on the larger-K 64^2 / 5x5 layers
            // (+2..5 %: the 49 KB of LDS cost the 4th block per CU, profiles/r6m_b6db.txt); in the graphed step the
            // small-grid rule measured 0.2-0.3 ms SLOWER (profiles/r6n_b6db_step_ab.txt: those layers run beside the
            // branch streams' kernels), so the default is off
            if (g_tune[20] == 1 || (g_tune[20] < 0 && a.M <= 16384)) {
                if (a.nsplit > 1) {
                    if (mode == 0) hipLaunchKernelGGL((conv_fwd_b6db_kernel<1, 1, 2, 2, 0, true>), grid, dim3(256), 0, st, a);
                    else hipLaunchKernelGGL((conv_fwd_b6db_kernel<1, 1, 2, 2, 1, true>), grid, dim3(256), 0, st, a);
                } else {
                    if (mode == 0) hipLaunchKernelGGL((conv_fwd_b6db_kernel<1, 1, 2, 2, 0, false>), grid, dim3(256), 0, st, a);
                    else hipLaunchKernelGGL((conv_fwd_b6db_kernel<1, 1, 2, 2, 1, false>), grid, dim3(256), 0, st, a);
                }
                return HY_LAUNCH_CHECK("conv_fwd_b6db_kernel");
            }
        }
        if (a.nsplit > 1) {
            if (mode == 0) hipLaunchKernelGGL((conv_fwd_b6_kernel<TM, TN, WM_, WN_, 0, true>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_b6_kernel<TM, TN, WM_, WN_, 1, true>), grid, dim3(256), 0, st, a);
        } else {
            if (mode == 0) hipLaunchKernelGGL((conv_fwd_b6_kernel<TM, TN, WM_, WN_, 0, false>), grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_b6_kernel<TM, TN, WM_, WN_, 1, false>), grid, dim3(256), 0, st, a);
        }
        return HY_LAUNCH_CHECK("conv_fwd_b6_kernel");
    }
    // split-K launches are a separate instantiation (partials to the slab, no epilogue)
    if (a.nsplit > 1) {
        if (mode == 0) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 0, true>), grid, dim3(256), 0, st, a);
        else if (mode == 1) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 1, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 2, true>), grid, dim3(256), 0, st, a);
    } else {
        if (mode == 0) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 0, false>), grid, dim3(256), 0, st, a);
        else if (mode == 1) hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 1, false>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WM_, WN_, 2, false>), grid, dim3(256), 0, st, a);
    }
    return HY_LAUNCH_CHECK("conv_fwd_kernel");
}

// persistent grid: as many blocks as fit on the chip at once (occupancy query, cached per instantiation),
// capped by blocks_per_cu (<= 0: no cap) and by the 32-pixel tiles available (4 per block)
template <int NT, int KC>
static int launch_stream_one(const ConvArgs& a, int blocks_per_cu, hipStream_t st) {
    static int occ = -1;
    if (occ < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv1x1_stream_kernel<NT, KC>, 256, 0) != hipSuccess || n < 1)
            n = 1;
        occ = n;
    }
    const int per_cu = blocks_per_cu > 0 ? std::min(occ, blocks_per_cu) : occ;
    const int blocks = std::max(1, std::min(ceil_div(ceil_div(a.M, 32), 4), 256 * per_cu));
    if (a.e.f16_operands) hipLaunchKernelGGL((conv1x1_stream_kernel<NT, KC, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv1x1_stream_kernel<NT, KC>), dim3(blocks), dim3(256), 0, st, a);
    return HY_LAUNCH_CHECK("conv1x1_stream_kernel");
}

static int launch_stream(const ConvArgs& a, int nt, int kc, int blocks_per_cu, hipStream_t st) {
#define HY_STREAM(NT, KC) \
    if (nt == NT && kc == KC) return launch_stream_one<NT, KC>(a, blocks_per_cu, st);
    HY_STREAM(2, 8) HY_STREAM(2, 12) HY_STREAM(2, 16)
    HY_STREAM(3, 8) HY_STREAM(3, 12) HY_STREAM(3, 16)
    HY_STREAM(4, 8) HY_STREAM(4, 12) HY_STREAM(4, 16)
    HY_STREAM(6, 8)
#undef HY_STREAM
    return set_error(HYRES_E_ARG, "conv1x1_stream: no instantiation for NT=%d KC=%d", nt, kc);
}

static void fill_taps(hyres_conv_geom* g, int p, int* tapcount, int K, int pad, int ph, int pw) {
    // sub-pixel phase (ph, pw) of a stride-2 transposed structure: taps kh with (ph+pad-kh) even
    g->tap0[p] = *tapcount;
    int n = 0;
    for (int kh = 0; kh < K; ++kh) {
        if (((ph + pad - kh) & 1) != 0) continue;
        for (int kw = 0; kw < K; ++kw) {
            if (((pw + pad - kw) & 1) != 0) continue;
            int t = *tapcount + n;
            g->dh[t] = (ph + pad - kh) / 2;
            g->dw[t] = (pw + pad - kw) / 2;
            g->kh[t] = kh;
            g->kw[t] = kw;
            ++n;
        }
    }
    g->ntap[p] = n;
    g->oph[p] = ph;
    g->opw[p] = pw;
    *tapcount += n;
}

static void dense_taps(hyres_conv_geom* g, int KH, int KW, int sgn, int dil, int pad) {
    // one phase, taps in (kh, kw) raster order; offset = sgn * (k*dil - pad)
    g->ntap[0] = KH * KW;
    g->tap0[0] = 0;
    g->ntaps = KH * KW;
    for (int kh = 0; kh < KH; ++kh)
        for (int kw = 0; kw < KW; ++kw) {
            int t = kh * KW + kw;
            g->dh[t] = sgn * (kh * dil - pad);
            g->dw[t] = sgn * (kw * dil - pad);
            g->kh[t] = kh;
            g->kw[t] = kw;
        }
}

// keys: HYRES_TUNE_TILE, _SPLIT_BLOCKS, _SPLIT_MINCHUNKS, _WGRAD_BLOCKS, _WGRAD_MINCHUNKS, _WGRAD_NT,
// _WGRAD_MAXSPLIT
// key 7: fp32 GEMMs bf16x6 (0: native fp32 MFMA); key 8: fp16 streaming 1x1; key 9: the bf16x6 weight-resident 3x3's
// whole-VGPR-file guard (0 = diagnostic unguarded build, DESIGN §4 "Cross-kernel interference"); key 10: the bf16x6
// streaming 1x1 kernel (0 = those layers on the tiled implicit GEMM, for A/B)
int g_tune[HYRES_TUNE_KEYS] = {-1, -1, -1, -1, -1, -1, -1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 1, 1, 1, 0, 1, 0, 1};

}  // namespace hyres

using namespace hyres;

extern "C" {

int hyres_geom_conv2d(hyres_conv_geom* g, int B, int H, int W, int Ci, int ldx, int Co, int ldy, int KH,
                      int KW, int stride, int pad, int dil) {
    HY_REQUIRE(g && KH * KW <= HYRES_MAX_TAPS && stride >= 1 && dil >= 1, HYRES_E_ARG, "bad conv args");
    *g = hyres_conv_geom{};
    g->B = B; g->Hi = H; g->Wi = W; g->Ci = Ci; g->ldx = ldx;
    g->Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
    g->Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
    g->Co = Co; g->ldy = ldy;
    g->nphase = 1; g->Hq = g->Ho; g->Wq = g->Wo;
    g->osh = g->osw = 1; g->ish = g->isw = stride;
    dense_taps(g, KH, KW, 1, dil, pad);
    return ok();
}

int hyres_geom_conv2d_dgrad(hyres_conv_geom* g, int B, int H, int W, int Ci, int ld_dx, int Co, int ld_dy,
                            int KH, int KW, int stride, int pad, int dil) {
    HY_REQUIRE(g && KH * KW <= HYRES_MAX_TAPS, HYRES_E_ARG, "bad conv dgrad args");
    *g = hyres_conv_geom{};
    const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
    const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
    g->B = B; g->Hi = Ho; g->Wi = Wo; g->Ci = Co; g->ldx = ld_dy;
    g->Ho = H; g->Wo = W; g->Co = Ci; g->ldy = ld_dx;
    if (stride == 1) {
        g->nphase = 1; g->Hq = H; g->Wq = W; g->osh = g->osw = 1; g->ish = g->isw = 1;
        dense_taps(g, KH, KW, -1, dil, pad);  // dX[h] += dY[h + pad - k*dil] W[k]
        return ok();
    }
    HY_REQUIRE(stride == 2 && dil == 1 && KH == KW && (H % 2) == 0 && (W % 2) == 0 && Ho * 2 == H &&
                   Wo * 2 == W, HYRES_E_SHAPE, "conv dgrad: only stride 2, dil 1, square K, even H/W");
    g->nphase = 4; g->Hq = H / 2; g->Wq = W / 2; g->osh = g->osw = 2; g->ish = g->isw = 1;
    int cnt = 0;
    for (int p = 0; p < 4; ++p) fill_taps(g, p, &cnt, KH, pad, p >> 1, p & 1);
    g->ntaps = cnt;
    return ok();
}

int hyres_geom_deconv2d(hyres_conv_geom* g, int B, int H, int W, int Ci, int ldx, int Co, int ldy, int K,
                        int pad) {
    HY_REQUIRE(g && K * K <= HYRES_MAX_TAPS, HYRES_E_ARG, "bad deconv args");
    HY_REQUIRE(2 * pad == K - 1, HYRES_E_SHAPE, "deconv: expects padding = K//2, output_padding = 1");
    *g = hyres_conv_geom{};
    g->B = B; g->Hi = H; g->Wi = W; g->Ci = Ci; g->ldx = ldx;
    g->Ho = 2 * H; g->Wo = 2 * W; g->Co = Co; g->ldy = ldy;
    g->nphase = 4; g->Hq = H; g->Wq = W; g->osh = g->osw = 2; g->ish = g->isw = 1;
    int cnt = 0;
    for (int p = 0; p < 4; ++p) fill_taps(g, p, &cnt, K, pad, p >> 1, p & 1);
    g->ntaps = cnt;
    return ok();
}

int hyres_geom_deconv2d_dgrad(hyres_conv_geom* g, int B, int H, int W, int Ci, int ld_dx, int Co, int ld_dy,
                              int K, int pad) {
    HY_REQUIRE(g && K * K <= HYRES_MAX_TAPS, HYRES_E_ARG, "bad deconv dgrad args");
    *g = hyres_conv_geom{};
    g->B = B; g->Hi = 2 * H; g->Wi = 2 * W; g->Ci = Co; g->ldx = ld_dy;
    g->Ho = H; g->Wo = W; g->Co = Ci; g->ldy = ld_dx;
    g->nphase = 1; g->Hq = H; g->Wq = W; g->osh = g->osw = 1; g->ish = g->isw = 2;
    dense_taps(g, K, K, 1, 1, pad);  // dX[i] += dY[2i - pad + k] W[k]
    return ok();
}

int hyres_geom_filter_taps(hyres_conv_geom* g, const unsigned char* keep, int KW) {
    HY_REQUIRE(g && keep && KW > 0, HYRES_E_ARG, "filter_taps: bad args");
    hyres_conv_geom o = *g;
    int cnt = 0;
    for (int p = 0; p < g->nphase; ++p) {
        o.tap0[p] = cnt;
        int n = 0;
        for (int t = g->tap0[p]; t < g->tap0[p] + g->ntap[p]; ++t) {
            if (!keep[g->kh[t] * KW + g->kw[t]]) continue;
            o.dh[cnt] = g->dh[t]; o.dw[cnt] = g->dw[t]; o.kh[cnt] = g->kh[t]; o.kw[cnt] = g->kw[t];
            ++cnt;
            ++n;
        }
        o.ntap[p] = n;
    }
    o.ntaps = cnt;
    *g = o;
    return ok();
}

int hyres_conv_weight_prep(const hyres_conv_geom* g, const float* w, float* w2, int mode, int Ci, int Co,
                           int KH, int KW, int pad, const float* mask, hyres_stream_t s) {
    HY_REQUIRE(g && w && w2, HYRES_E_ARG, "weight_prep: NULL");
    (void)pad;
    PrepArgs a{};
    a.w = w; a.w2 = w2; a.mask = mask; a.mode = mode; a.KH = KH; a.KW = KW; a.Ci = Ci; a.Co = Co;
    a.ntaps = g->ntaps;
    for (int t = 0; t < g->ntaps; ++t) {
        HY_REQUIRE(g->kh[t] < KH && g->kw[t] < KW, HYRES_E_SHAPE, "weight_prep: tap %d outside %dx%d", t, KH, KW);
        a.kh[t] = g->kh[t];
        a.kw[t] = g->kw[t];
    }
    switch (mode) {
        case HYRES_WPREP_CONV: a.rows = Co; a.cols = Ci; break;
        case HYRES_WPREP_CONV_DGRAD: a.rows = Ci; a.cols = Co; break;
        case HYRES_WPREP_DECONV: a.rows = Co; a.cols = Ci; break;
        case HYRES_WPREP_DECONV_DGRAD: a.rows = Ci; a.cols = Co; break;
        default: return set_error(HYRES_E_ARG, "weight_prep: bad mode %d", mode);
    }
    HY_REQUIRE(a.cols == g->Ci && a.rows >= g->Co, HYRES_E_SHAPE,
               "weight_prep: geometry channels (%d->%d) != weight (%d->%d)", g->Ci, g->Co, a.cols, a.rows);
    long long total = (long long)a.rows * a.ntaps * a.cols;
    int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(weight_prep_kernel, dim3(blocks), dim3(256), 0, as_stream(s), a);
    return HY_LAUNCH_CHECK("weight_prep_kernel");
}

long long hyres_prep_desc_bytes(void) { return (long long)sizeof(PrepDesc); }

int hyres_prep_desc_fill(void* desc, const hyres_conv_geom* g, const float* w, float* w2, int mode, int Ci, int Co,
                         int KH, int KW, long long begin, long long* count) {
    HY_REQUIRE(desc && g && w && w2 && count, HYRES_E_ARG, "prep_desc_fill: NULL");
    PrepDesc d{};
    PrepArgs& a = d.a;
    a.w = w; a.w2 = w2; a.mask = nullptr; a.mode = mode; a.KH = KH; a.KW = KW; a.Ci = Ci; a.Co = Co;
    a.ntaps = g->ntaps;
    for (int t = 0; t < g->ntaps; ++t) {
        HY_REQUIRE(g->kh[t] < KH && g->kw[t] < KW, HYRES_E_SHAPE, "prep_desc: tap %d outside %dx%d", t, KH, KW);
        a.kh[t] = g->kh[t];
        a.kw[t] = g->kw[t];
    }
    switch (mode) {
        case HYRES_WPREP_CONV: case HYRES_WPREP_DECONV: a.rows = Co; a.cols = Ci; break;
        case HYRES_WPREP_CONV_DGRAD: case HYRES_WPREP_DECONV_DGRAD: a.rows = Ci; a.cols = Co; break;
        default: return set_error(HYRES_E_ARG, "prep_desc: bad mode %d", mode);
    }
    d.begin = begin;
    d.count = (long long)a.rows * a.ntaps * a.cols;
    HY_REQUIRE(d.count < (1LL << 31), HYRES_E_SHAPE, "prep_desc: weight too large");
    *count = d.count;
    memcpy(desc, &d, sizeof(d));
    return ok();
}

int hyres_conv_weight_prep_batch(const void* descs, int n, long long total, hyres_stream_t s) {
    HY_REQUIRE(descs && n > 0 && n <= 65535 && total > 0, HYRES_E_ARG, "prep_batch: bad size");
    hipLaunchKernelGGL(weight_prep_batch_kernel, dim3(64, n), dim3(256), 0, as_stream(s), (const PrepDesc*)descs, n,
                       total);
    return HY_LAUNCH_CHECK("weight_prep_batch_kernel");
}


// conv3x3_halo_f16_kernel applies (see above)
static bool halo16_ok(const hyres_conv_geom* g, const hyres_epilogue* e) {
    if (!e->f16_operands || g->nphase != 1 || g->ntaps != 9 || g->Ci % 32 != 0 || g->Co % 64 != 0) return false;
    if (g->ish != 1 || g->isw != 1 || g->Hi != g->Ho || g->Wi != g->Wo || g->Hq != g->Ho || g->Wq != g->Wo) return false;
    if (g->Wo % HALO_TW != 0 || e->square_input) return false;
    for (int t = 0; t < 9; ++t)
        if (g->dh[t] < -1 || g->dh[t] > 1 || g->dw[t] < -1 || g->dw[t] > 1) return false;
    return true;
}

// conv3x3_wres_f16_kernel: the halo16 geometry with Ci == 64, enough 256-pixel tiles per block to amortise
// the one-time weight conversion (>= 2 per block)
static int g_cus = 0;
static int num_cus() {
    if (!g_cus) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                     hipSuccess || n < 1)
            n = 256;
        g_cus = n;
    }
    return g_cus;
}

// blocks per output-channel group: one per CU (persistent), a multiple of 8 so that the group-major block order
// keeps block bg of every group on XCD bg % 8
static int wres_blocks(int groups) {
    return std::max(8, (num_cus() / groups) & ~7);
}

static bool wres16_ok(const hyres_conv_geom* g) {
    if (g->Ci != 64) return false;
    const long long tiles = (long long)g->B * ((g->Ho + HALO_R - 1) / HALO_R) * (g->Wo / HALO_TW);
    const int groups = g->Co / 64;
    return tiles >= 2LL * wres_blocks(groups) && (long long)g->B * g->Hi * g->Wi * g->ldx * 4 < 0x7FFFFFF0LL;
}

static int launch_wres16(const ConvArgs& a, hipStream_t st) {
    const hyres_conv_geom& g = a.g;
    const int ntiles = g.B * ((g.Ho + HALO_R - 1) / HALO_R) * (g.Wo / HALO_TW);
    const int groups = g.Co / 64;
    const int per = wres_blocks(groups);
    const dim3 grid(per * groups);
    switch (a.e.io_f16 & 3) {
        case 0: hipLaunchKernelGGL(conv3x3_wres_f16_kernel<0>, grid, dim3(512), 0, st, a, ntiles, groups); break;
        case 1: hipLaunchKernelGGL(conv3x3_wres_f16_kernel<1>, grid, dim3(512), 0, st, a, ntiles, groups); break;
        case 2: hipLaunchKernelGGL(conv3x3_wres_f16_kernel<2>, grid, dim3(512), 0, st, a, ntiles, groups); break;
        default: hipLaunchKernelGGL(conv3x3_wres_f16_kernel<3>, grid, dim3(512), 0, st, a, ntiles, groups); break;
    }
    return HY_LAUNCH_CHECK("conv3x3_wres_f16_kernel");
}

// the 3x3's largest tap offset (the weight-resident halo radius)
static int wres_halo(const hyres_conv_geom* g) {
    int d = 0;
    for (int t = 0; t < 9; ++t) d = std::max(d, std::max(std::abs(g->dh[t]), std::abs(g->dw[t])));
    return d;
}

// conv3x3_wres_f32_kernel: fp32 operands, the halo16 geometry with Ci == 64 and Co % 32 == 0, >= 2 tiles per
// block
static bool wres32_ok(const hyres_conv_geom* g, const hyres_epilogue* e) {
    if (g_tune[14] == 0) return false;  // A/B: the implicit GEMM instead
    if (e->f16_operands || e->io_f16 || e->square_input || e->kind != HYRES_EPI_BIAS || g->nphase != 1 ||
        g->ntaps != 9 || g->Ci != 64 || g->Co % 32 != 0)
        return false;
    // the epilogue operands are addressed with 32-bit byte offsets
    const long long npix = (long long)g->B * g->Ho * g->Wo;
    const int ld = std::max(g->ldy, std::max(e->res ? e->ldres : 0, e->aux0 ? e->ld0 : 0));
    if (npix * ld * 4 >= 0x7FFFFFF0LL) return false;
    if (g->ish != 1 || g->isw != 1 || g->Hi != g->Ho || g->Wi != g->Wo || g->Hq != g->Ho || g->Wq != g->Wo ||
        g->Wo % HALO_TW != 0)
        return false;
    // halo radius 1, or 2 for the bf16x6 kernel (dilation-2 3x3s: its D = 2 build)
    if (wres_halo(g) > (g_tune[7] == 1 && g_tune[9] != 0 ? 2 : 1)) return false;
    const long long tiles = (long long)g->B * ((g->Ho + HALO_R - 1) / HALO_R) * (g->Wo / HALO_TW);
    const int groups = g->Co / 32;
    return tiles >= 2LL * wres_blocks(groups) && (long long)g->B * g->Hi * g->Wi * g->ldx * 4 < 0x7FFFFFF0LL;
}

// fp32 GEMM mode of the weight-resident 3x3 (hyres_conv_tuning key 7): 0 = native fp32 MFMA, 1 = bf16x6
static bool wres_bf6() { return g_tune[7] == 1; }

static int launch_wres32(const ConvArgs& a, hipStream_t st) {
    const hyres_conv_geom& g = a.g;
    const int ntiles = g.B * ((g.Ho + HALO_R - 1) / HALO_R) * (g.Wo / HALO_TW);
    const int groups = g.Co / 32;
    const int per = wres_blocks(groups);
    if (wres_bf6()) {
        const dim3 grid(per * groups);
        if (wres_halo(&g) == 2)  // dilation 2 (wres32_ok admits it only with the guard on): the pipelined build
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<true, 1, 2>), grid, dim3(512), 0, st, a, ntiles, groups);
        else if (g_tune[9] == 0)  // diagnostic only: the allocation that let other kernels' waves share its SIMDs
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<false, 0>), grid, dim3(512), 0, st, a, ntiles, groups);
        else if (g_tune[12] == 1)
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<true, 1>), grid, dim3(512), 0, st, a, ntiles, groups);
        else if (g_tune[12] == 2)
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<true, 2>), grid, dim3(512), 0, st, a, ntiles, groups);
        else if (g_tune[12] == 3)
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<true, 3>), grid, dim3(512), 0, st, a, ntiles, groups);
        else
            hipLaunchKernelGGL((conv3x3_wres_bf6_kernel<true, 0>), grid, dim3(512), 0, st, a, ntiles, groups);
        const int rc = HY_LAUNCH_CHECK("conv3x3_wres_bf6_kernel");
        if (rc || a.e.act != HYRES_ACT_PRELU_MASK) return rc;
        hipLaunchKernelGGL(prelu_slope_sum_kernel, dim3(1), dim3(256), 0, st, a.e.aux2, (int)grid.x,
                           const_cast<float*>(a.e.aux1));
        return HY_LAUNCH_CHECK("prelu_slope_sum_kernel");
    }
    hipLaunchKernelGGL(conv3x3_wres_f32_kernel, dim3(per * groups), dim3(512), 0, st, a, ntiles, groups);
    return HY_LAUNCH_CHECK("conv3x3_wres_f32_kernel");
}

static int launch_halo16(const ConvArgs& a, hipStream_t st) {
    const hyres_conv_geom& g = a.g;
    const int blocks = g.B * ((g.Ho + HALO_R - 1) / HALO_R) * (g.Wo / HALO_TW) * (g.Co / 64);
    switch (a.e.io_f16 & 3) {
        case 0: hipLaunchKernelGGL(conv3x3_halo_f16_kernel<0>, dim3(blocks), dim3(256), 0, st, a); break;
        case 1: hipLaunchKernelGGL(conv3x3_halo_f16_kernel<1>, dim3(blocks), dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL(conv3x3_halo_f16_kernel<2>, dim3(blocks), dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL(conv3x3_halo_f16_kernel<3>, dim3(blocks), dim3(256), 0, st, a); break;
    }
    return HY_LAUNCH_CHECK("conv3x3_halo_f16_kernel");
}

// Kernel choice of hyres_conv_forward, shared with hyres_conv_kernel_name / hyres_conv_plan (the profiler's
// label). tile: 0 = <2,2,2,2> (128x128), 1 = <2,1,2,2> (128x64), 2 = <1,1,4,1> (128x32), 3 = <1,2,2,2>
// (64x128), 4 = <1,1,2,2> (64x64).
//   * short-K 1x1 layers (<= 4 K chunks): half-height tiles — the short main loop cannot hide the operand
//     and epilogue latencies, so twice as many blocks go in flight;
//   * small grids (<= 65536 output pixels: the 64^2 and 32^2 regions at bs 16): 64-row tiles, 64 wide up to
//     192 channels (fp32) / below 192 (f16), else 64x128 (fp32) / 128x128 (f16); measured per geometry
//     over every tile and split-K target (scripts/tile_sweep.py, profiles/r2_tile_sweep_*.txt);
//   * the scalar-load path (Ci % 32 != 0: the 3-channel image side) 64-row tiles (3->64 at 256^2: 198 -> 140 us);
//   * otherwise 128-row tiles as wide as Co allows.
// Split-K engages only when the chosen tile leaves fewer than 512 blocks and K has >= 8 chunks.
struct ConvChoice {
    bool narrow;
    int tile, mode;
};
// conv1x1_stream_kernel eligibility: single-tap stride-1 fp32 1x1 with K = Ci in {64, 96, 128}, Co in
// {64, 96, 128} (or 192 with K = 64), BIAS epilogue with no streamed operand (residual / ReLU mask /
// old y), grids >= 65536 output pixels. Returns NT (Co / 32) or 0.
static int stream_nt(const hyres_conv_geom* g, const hyres_epilogue* e) {
    constexpr long long min_px = 65536;
    if ((e->io_f16 & 3) || e->square_input || e->kind != HYRES_EPI_BIAS) return 0;
    if (g->nphase != 1 || g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0) return 0;
    if (g->Hi != g->Hq || g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq) return 0;
    if ((long long)g->B * g->Hq * g->Wq < min_px) return 0;
    if (g->Ci != 64 && g->Ci != 96 && g->Ci != 128) return 0;
    if (e->res || e->act == HYRES_ACT_RELU_MASK || e->accumulate) return 0;
    if (g->Co == 64 || g->Co == 96 || g->Co == 128) return g->Co / 32;
    if (g->Co == 192 && g->Ci == 64) return 6;
    return 0;
}

// conv1x1_stream_h_kernel eligibility: fp16 X and Y (io_f16 = 3), single-tap stride-1 1x1 with Ci and Co in
// {64, 96, 128}, BIAS epilogue with ReLU / none and no streamed operand, grids >= 16384 output pixels, 16-byte X rows.
// Returns NT (Co / 32) or 0.
static int stream_h_nt(const hyres_conv_geom* g, const hyres_epilogue* e) {
    if (g_tune[8] == 0 || (e->io_f16 & 3) != 3 || e->square_input || e->kind != HYRES_EPI_BIAS || e->out2) return 0;
    // a streamed epilogue operand (residual, ReLU mask, old y) measured slower than the tiles (128^2 64->128 +res
    // 45.2 vs 43.5 us, 64^2 16.5 vs 13.9 us; without one 24.8 vs 30.7 and 60.3 vs 80.8 us: profiles/r4e_h1x1.txt),
    // as for the fp32 streaming kernel: those layers stay tiled
    if (e->res || e->act == HYRES_ACT_RELU_MASK || e->accumulate) return 0;
    if (e->act != HYRES_ACT_NONE && e->act != HYRES_ACT_RELU) return 0;
    if (g->nphase != 1 || g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0) return 0;
    if (g->Hi != g->Hq || g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq) return 0;
    if ((long long)g->B * g->Hq * g->Wq < 16384) return 0;
    if (g->Ci != 64 && g->Ci != 96 && g->Ci != 128) return 0;
    if (g->Co != 64 && g->Co != 96 && g->Co != 128) return 0;
    if (g->ldx % 8 || g->ldy % 4) return 0;
    return g->Co / 32;
}

// conv1x1_stream_hf_kernel eligibility (hyres_conv_tuning key 17 = 1, default): fp16 X and Y / operands (io_f16 = 3),
// f16 operands, single-tap stride-1 1x1, (Ci, Co) in {64, 128}^2, >= 16384 output pixels, BIAS epilogue with none /
// ReLU / ReLU mask and at least one streamed operand (residual, mask, old y; without one: conv1x1_stream_h_kernel),
// no out2, 16-byte X rows / 8-byte Y rows. Returns NT | KC << 4 | F << 8, or 0.
static int stream_hf_cfg(const hyres_conv_geom* g, const hyres_epilogue* e) {
    if (g_tune[17] == 0 || (e->io_f16 & 3) != 3 || !e->f16_operands || e->square_input) return 0;
    if (e->kind == HYRES_EPI_ROWSCALE) {  // round 6: the fusion 1x1 forward under AMP with SpatialAttention folded
        if (g_tune[21] == 0 || g->Ci != 192 || g->Co != 64 || e->res || e->accumulate || !e->out2 || e->ldo2 % 4 ||
            (e->act != HYRES_ACT_NONE && e->act != HYRES_ACT_RELU && e->act != HYRES_ACT_PRELU) || g->nphase != 1 ||
            g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0 || g->Hi != g->Hq ||
            g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq || (long long)g->B * g->Hq * g->Wq < 16384 ||
            g->ldx % 8 || g->ldy % 4)
            return 0;
        return 2 | (12 << 4) | (16 << 8);
    }
    if (e->kind == HYRES_EPI_SA_BWD) {  // round 6: the fusion 1x1's input-gradient under AMP, 64 -> 192
        const bool pm = e->act == HYRES_ACT_PRELU_MASK && !e->accumulate;  // + the scale-1 PReLU backward
        if (g_tune[21] == 0 || g->Ci != 64 || g->Co != 192 || (e->act != HYRES_ACT_NONE && !pm) || (e->res && !pm) ||
            (e->out2 && !pm) || (pm && (!e->aux1 || e->ld1 < 64 || e->ld1 % 4 || !e->res)) || g->nphase != 1 ||
            g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0 || g->Hi != g->Hq ||
            g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq || (long long)g->B * g->Hq * g->Wq < 16384 ||
            g->ldx % 8 || g->ldy % 4 || e->ld0 % 2)
            return 0;
        return 6 | (4 << 4) | ((pm ? 40 : (8 | (e->accumulate ? 4 : 0))) << 8);
    }
    if (e->out2) return 0;
    if (e->kind != HYRES_EPI_BIAS) return 0;
    if (e->act != HYRES_ACT_NONE && e->act != HYRES_ACT_RELU && e->act != HYRES_ACT_RELU_MASK) return 0;
    if (g->nphase != 1 || g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0) return 0;
    if (g->Hi != g->Hq || g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq) return 0;
    if ((long long)g->B * g->Hq * g->Wq < 16384) return 0;
    if ((g->Ci != 64 && g->Ci != 128) || (g->Co != 64 && g->Co != 128)) return 0;
    if (g->ldx % 8 || g->ldy % 4 || (e->res && e->ldres % 4) || (e->act == HYRES_ACT_RELU_MASK && e->ld0 % 4)) return 0;
    const int F = (e->res ? 1 : 0) | (e->act == HYRES_ACT_RELU_MASK ? 2 : 0) | (e->accumulate ? 4 : 0);
    if (!F) return 0;
    return (g->Co / 32) | ((g->Ci / 16) << 4) | (F << 8);
}

// conv1x1_stream_b6_kernel eligibility (bf16x6 fp32 GEMMs, hyres_conv_tuning key 10 = 1): fp32 X / Y, single-tap
// stride-1 1x1 with (Ci, Co) in {(64, 64), (64, 128), (128, 64)}, BIAS epilogue with none / ReLU / PReLU / ReLU mask,
// any of residual / mask / accumulate, grids >= 65536 output pixels. Returns the packed choice NT | KS << 4 | F << 8,
// or 0.
static int stream_b6_cfg(const hyres_conv_geom* g, const hyres_epilogue* e) {
    if (g_tune[7] != 1 || g_tune[10] == 0) return 0;
    if (e->io_f16 || e->f16_operands || e->square_input) return 0;
    if (e->kind == HYRES_EPI_SA_BWD) {  // round 6: the fusion 1x1's input-gradient, 64 -> 192 (coalesced epilogue only)
        const bool pm = e->act == HYRES_ACT_PRELU_MASK && !e->accumulate;
        if (g_tune[11] == 0 || g_tune[21] == 0 || g->Ci != 64 || g->Co != 192 || (e->act != HYRES_ACT_NONE && !pm) ||
            (e->res && !pm) || (e->out2 && !pm) || (pm && (!e->aux1 || e->ld1 < 64 || e->ld1 % 4 || !e->res)) ||
            g->nphase != 1 || g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0 ||
            g->Hi != g->Hq || g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq || (long long)g->B * g->Hq * g->Wq < 65536)
            return 0;
        return 6 | (4 << 4) | ((pm ? 40 : (8 | (e->accumulate ? 4 : 0))) << 8);
    }
    if (g->nphase != 1 || g->ntaps != 1 || g->ish != 1 || g->isw != 1 || g->dh[0] != 0 || g->dw[0] != 0) return 0;
    if (g->Hi != g->Hq || g->Wi != g->Wq || g->Ho != g->Hq || g->Wo != g->Wq) return 0;
    if ((long long)g->B * g->Hq * g->Wq < 65536) return 0;
    if (e->kind == HYRES_EPI_ROWSCALE) {  // round 6: the fusion 1x1 forward with SpatialAttention folded, 192 -> 64
        if (g_tune[11] == 0 || g_tune[21] == 0 || g->Ci != 192 || g->Co != 64 || e->res || e->accumulate ||
            (e->act != HYRES_ACT_NONE && e->act != HYRES_ACT_RELU && e->act != HYRES_ACT_PRELU))
            return 0;
        return 2 | (12 << 4) | (16 << 8);
    }
    if (e->kind != HYRES_EPI_BIAS) return 0;
    const bool shape = (g->Ci == 64 && (g->Co == 64 || g->Co == 128)) || (g->Ci == 128 && g->Co == 64) ||
                       (g->Ci == 128 && g->Co == 128);
    if (!shape) return 0;
    const int F = (e->res ? 1 : 0) | (e->act == HYRES_ACT_RELU_MASK ? 2 : 0) | (e->accumulate ? 4 : 0);
    // 128 -> 128 (round 6, the GDN-side 1x1s at 128^2): 122 KB of LDS, one wave per SIMD — built for the operand-free
    // and ReLU-mask forms only
    if (g->Ci == 128 && g->Co == 128 && F != 0 && F != 2) return 0;
    return (g->Co / 32) | ((g->Ci / 16) << 4) | (F << 8);
}

extern "C++" {
template <int NT, int KC>
static int launch_stream_h_one(const ConvArgs& a, hipStream_t st) {
    static int occ = -1;
    if (occ < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv1x1_stream_h_kernel<NT, KC>, 256, 0) != hipSuccess ||
            n < 1)
            n = 1;
        occ = n;
    }
    const int blocks = std::max(1, std::min(ceil_div(ceil_div(a.M, 32), 4), 256 * occ));
    hipLaunchKernelGGL((conv1x1_stream_h_kernel<NT, KC>), dim3(blocks), dim3(256), 0, st, a);
    return HY_LAUNCH_CHECK("conv1x1_stream_h_kernel");
}
}  // extern "C++"

extern "C++" {
template <int NT, int KS, int F, bool CE>
static int launch_stream_b6_ce(const ConvArgs& a, hipStream_t st) {
    static int occ = -1;
    if (occ < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv1x1_stream_b6_kernel<NT, KS, F, CE>, 256, 0) !=
                hipSuccess ||
            n < 1)
            n = 1;
        occ = n;
    }
    const int blocks = std::max(1, std::min(ceil_div(ceil_div(a.M, 32), 4), num_cus() * occ));
    hipLaunchKernelGGL((conv1x1_stream_b6_kernel<NT, KS, F, CE>), dim3(blocks), dim3(256), 0, st, a);
    if constexpr ((F & 32) != 0) {  // the PReLU mask's slope partials, summed in a fixed order and added
        const int rc = HY_LAUNCH_CHECK("conv1x1_stream_b6_kernel");
        if (rc) return rc;
        hipLaunchKernelGGL(prelu_slope_sum_kernel, dim3(1), dim3(256), 0, st, (const float*)a.e.out2, blocks,
                           const_cast<float*>(a.e.res));
        return HY_LAUNCH_CHECK("prelu_slope_sum_kernel");
    }
    return HY_LAUNCH_CHECK("conv1x1_stream_b6_kernel");
}
template <int NT, int KS, int F>
static int launch_stream_b6_one(const ConvArgs& a, hipStream_t st) {
    return g_tune[11] == 0 ? launch_stream_b6_ce<NT, KS, F, false>(a, st) : launch_stream_b6_ce<NT, KS, F, true>(a, st);
}
template <int NT, int KS>
static int launch_stream_b6_f(const ConvArgs& a, int f, hipStream_t st) {
    switch (f) {
        case 0: return launch_stream_b6_one<NT, KS, 0>(a, st);
        case 1: return launch_stream_b6_one<NT, KS, 1>(a, st);
        case 2: return launch_stream_b6_one<NT, KS, 2>(a, st);
        case 3: return launch_stream_b6_one<NT, KS, 3>(a, st);
        case 4: return launch_stream_b6_one<NT, KS, 4>(a, st);
        case 5: return launch_stream_b6_one<NT, KS, 5>(a, st);
        case 6: return launch_stream_b6_one<NT, KS, 6>(a, st);
        default: return launch_stream_b6_one<NT, KS, 7>(a, st);
    }
}
}  // extern "C++"

static int launch_stream_b6(const ConvArgs& a, int cfg, hipStream_t st) {
    const int nt = cfg & 15, ks = (cfg >> 4) & 15, f = cfg >> 8;
    if (nt == 6 && ks == 4 && f == 8) return launch_stream_b6_ce<6, 4, 8, true>(a, st);
    if (nt == 6 && ks == 4 && f == 12) return launch_stream_b6_ce<6, 4, 12, true>(a, st);
    if (nt == 6 && ks == 4 && f == 40) return launch_stream_b6_ce<6, 4, 40, true>(a, st);
    if (nt == 2 && ks == 12 && f == 16) return launch_stream_b6_ce<2, 12, 16, true>(a, st);
    if (nt == 2 && ks == 4) return launch_stream_b6_f<2, 4>(a, f, st);
    if (nt == 4 && ks == 4) return launch_stream_b6_f<4, 4>(a, f, st);
    if (nt == 2 && ks == 8) return launch_stream_b6_f<2, 8>(a, f, st);
    if (nt == 4 && ks == 8 && f == 0) return launch_stream_b6_one<4, 8, 0>(a, st);
    if (nt == 4 && ks == 8 && f == 2) return launch_stream_b6_one<4, 8, 2>(a, st);
    return set_error(HYRES_E_ARG, "conv1x1_stream_b6: no instantiation for NT=%d KS=%d", nt, ks);
}

extern "C++" {
template <int NT, int KC, int F>
static int launch_stream_hf_one(const ConvArgs& a, hipStream_t st) {
    static int occ = -1;
    if (occ < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv1x1_stream_hf_kernel<NT, KC, F>, 256, 0) != hipSuccess ||
            n < 1)
            n = 1;
        occ = n;
    }
    const int blocks = std::max(1, std::min(ceil_div(ceil_div(a.M, 32), 4), num_cus() * occ));
    hipLaunchKernelGGL((conv1x1_stream_hf_kernel<NT, KC, F>), dim3(blocks), dim3(256), 0, st, a);
    if constexpr ((F & 32) != 0) {  // the PReLU mask's slope partials, summed in a fixed order and added
        const int rc = HY_LAUNCH_CHECK("conv1x1_stream_hf_kernel");
        if (rc) return rc;
        hipLaunchKernelGGL(prelu_slope_sum_kernel, dim3(1), dim3(256), 0, st, (const float*)a.e.out2, blocks,
                           const_cast<float*>(a.e.res));
        return HY_LAUNCH_CHECK("prelu_slope_sum_kernel");
    }
    return HY_LAUNCH_CHECK("conv1x1_stream_hf_kernel");
}
template <int NT, int KC>
static int launch_stream_hf_f(const ConvArgs& a, int f, hipStream_t st) {
    switch (f) {
        case 1: return launch_stream_hf_one<NT, KC, 1>(a, st);
        case 2: return launch_stream_hf_one<NT, KC, 2>(a, st);
        case 3: return launch_stream_hf_one<NT, KC, 3>(a, st);
        case 4: return launch_stream_hf_one<NT, KC, 4>(a, st);
        case 5: return launch_stream_hf_one<NT, KC, 5>(a, st);
        case 6: return launch_stream_hf_one<NT, KC, 6>(a, st);
        default: return launch_stream_hf_one<NT, KC, 7>(a, st);
    }
}
}  // extern "C++"

static int launch_stream_hf(const ConvArgs& a, int cfg, hipStream_t st) {
    const int nt = cfg & 15, kc = (cfg >> 4) & 15, f = cfg >> 8;
    if (nt == 6 && kc == 4 && f == 8) return launch_stream_hf_one<6, 4, 8>(a, st);
    if (nt == 6 && kc == 4 && f == 12) return launch_stream_hf_one<6, 4, 12>(a, st);
    if (nt == 6 && kc == 4 && f == 40) return launch_stream_hf_one<6, 4, 40>(a, st);
    if (nt == 2 && kc == 12 && f == 16) return launch_stream_hf_one<2, 12, 16>(a, st);
    if (nt == 2 && kc == 4) return launch_stream_hf_f<2, 4>(a, f, st);
    if (nt == 2 && kc == 8) return launch_stream_hf_f<2, 8>(a, f, st);
    if (nt == 4 && kc == 4) return launch_stream_hf_f<4, 4>(a, f, st);
    if (nt == 4 && kc == 8) return launch_stream_hf_f<4, 8>(a, f, st);
    return set_error(HYRES_E_ARG, "conv1x1_stream_hf: no instantiation for NT=%d KC=%d", nt, kc);
}

static int launch_stream_h(const ConvArgs& a, int nt, int kc, hipStream_t st) {
#define HY_STREAM_H(NT, KC) \
    if (nt == NT && kc == KC) return launch_stream_h_one<NT, KC>(a, st);
    HY_STREAM_H(2, 4) HY_STREAM_H(2, 6) HY_STREAM_H(2, 8)
    HY_STREAM_H(3, 4) HY_STREAM_H(3, 6) HY_STREAM_H(3, 8)
    HY_STREAM_H(4, 4) HY_STREAM_H(4, 6) HY_STREAM_H(4, 8)
#undef HY_STREAM_H
    return set_error(HYRES_E_ARG, "conv1x1_stream_h: no instantiation for NT=%d KC=%d", nt, kc);
}

static const int TILE_BM[5] = {128, 128, 128, 64, 64};
static const int TILE_BN[5] = {128, 64, 32, 128, 64};

// Tile / split-K overrides set through hyres_conv_tuning (tuning sweeps; -1 = the heuristics below)
// keys: HYRES_TUNE_TILE, _SPLIT_BLOCKS, _SPLIT_MINCHUNKS, _WGRAD_BLOCKS, _WGRAD_MINCHUNKS, _WGRAD_NT

static ConvChoice choose_conv(const hyres_conv_geom* g, const hyres_epilogue* e, bool aligned) {
    ConvChoice c{};
    c.mode = (g->Ci % KT == 0) ? (e->square_input ? 1 : 0) : 2;
    c.narrow = narrow_ok(g) && !e->square_input && e->kind == HYRES_EPI_BIAS && aligned;
    constexpr long long small_px = 65536;
    const bool f16 = e->f16_operands && c.mode != 2;
    const bool short_k = c.mode != 2 && g->nphase == 1 && g->ntaps == 1 && g->Ci <= 4 * KT;
    const long long mtot = (long long)g->B * g->Hq * g->Wq * g->nphase;
    // fp32 small grids (round 6, profiles/r6g_tile32.txt, 32^2 bs16 bf16x6): the 1x1 96 -> 192 (+res) 14.9 -> 13.1 us on
    // 64x64 tiles, 640 -> 512 102 -> 81 us on 128x128
    // (hyres_conv_tuning key 18 = 0: the round-5 rule, A/B)
    const bool r6 = g_tune[18] != 0;
    if (short_k && g->Co > 64 && !(r6 && !f16 && mtot <= small_px && g->Co <= 192)) c.tile = 3;
    else if (short_k && g->Co > 32) c.tile = 4;
    else if (c.mode != 2 && g->Co > 32 && mtot <= small_px) {
        // K depth of the deepest phase: the K-heavy single-phase layers take the bigger tiles (fragment reuse) —
        // 128^2 -> 64^2 5x5 s2 128 -> 128 434 -> 347 us on 128x128, 32^2 3x3 384 -> 192 195 -> 183 us and 64^2 -> 32^2
        // 5x5 s2 128 -> 192 183 -> 172 us on 128x64 (profiles/r6p_tile5.txt)
        int maxtap = 0;
        for (int ph = 0; ph < g->nphase; ++ph) maxtap = std::max(maxtap, g->ntap[ph]);
        const bool kheavy = g->nphase == 1 && (long long)maxtap * g->Ci >= 1024;
        if (f16) c.tile = g->Co >= 192 ? 0 : 4;
        else if (r6 && (g->Co >= 512 || (kheavy && mtot >= small_px && g->Co >= 128))) c.tile = 0;
        else if (r6 && kheavy && g->Co == 192) c.tile = 1;
        else c.tile = g->Co > 192 ? 3 : 4;
    }
    else if (c.mode == 2 && g->Co > 32) c.tile = g->Co > 64 ? 3 : 4;  // scalar-load path: 64-row tiles
    else if (g->Co > 64) c.tile = 0;
    else if (g->Co > 32) c.tile = 1;
    else c.tile = 2;
    if (g_tune[0] >= 0 && g_tune[0] <= 4) c.tile = g_tune[0];
    return c;
}

struct ConvPlan {
    int nsplit, cps;
};

static ConvPlan conv_plan(const hyres_conv_geom* g, int tile) {
    ConvPlan p{};
    const long long M = (long long)g->B * g->Hq * g->Wq;
    long long blocks = (long long)ceil_div(M, TILE_BM[tile]) * ceil_div(g->Co, TILE_BN[tile]) * g->nphase;
    int maxtap = 0;
    for (int ph = 0; ph < g->nphase; ++ph) maxtap = std::max(maxtap, g->ntap[ph]);
    const int nk = (g->Ci % KT == 0) ? maxtap * (g->Ci / KT) : ceil_div((long long)maxtap * g->Ci, KT);
    p.nsplit = 1;
    p.cps = nk;
    const int sb = g_tune[1] >= 0 ? g_tune[1] : 512;
    const int sc = g_tune[2] > 0 ? g_tune[2] : 4;
    if (blocks < sb && nk >= 2 * sc) {
        // split K so that ~sb blocks are in flight, at least sc chunks per split
        int want = (int)std::min<long long>(ceil_div(sb, blocks), 64);
        int ns = std::max(1, std::min(want, nk / sc));
        p.cps = ceil_div(nk, ns);
        p.nsplit = ceil_div(nk, p.cps);
    }
    return p;
}

static long long plan_ws_bytes(const hyres_conv_geom* g, const ConvPlan& p) {
    if (p.nsplit <= 1) return 0;
    return (long long)p.nsplit * g->nphase * ((long long)g->B * g->Hq * g->Wq) * g->Co * 4;
}

int hyres_conv_tuning(int key, int value, int* old) {
    HY_REQUIRE(key >= 0 && key < HYRES_TUNE_KEYS, HYRES_E_ARG, "conv_tuning: key %d", key);
    if (old) *old = g_tune[key];
    g_tune[key] = value;
    return ok();
}

long long hyres_conv_workspace_bytes(const hyres_conv_geom* g) {
    // the larger of the fp32 and fp16-operand plans (the tile, hence the split, depends on the dtype)
    if (!g || narrow_ok(g)) return 0;
    long long need = 0;
    for (int f16 = 0; f16 < 2; ++f16) {
        hyres_epilogue e{};
        e.kind = HYRES_EPI_BIAS;
        e.f16_operands = f16;
        need = std::max(need, plan_ws_bytes(g, conv_plan(g, choose_conv(g, &e, true).tile)));
    }
    return need;
}

int hyres_conv_plan(const hyres_conv_geom* g, const hyres_epilogue* e, int* tile, int* nsplit) {
    HY_REQUIRE(g && e, HYRES_E_ARG, "conv_plan: NULL argument");
    const ConvChoice ch = choose_conv(g, e, true);
    const ConvPlan p = ch.narrow ? ConvPlan{1, 0} : conv_plan(g, ch.tile);
    if (tile) *tile = ch.narrow ? -1 : ch.tile;
    if (nsplit) *nsplit = p.nsplit;
    return ok();
}

int hyres_conv_forward(const hyres_conv_geom* g, const float* x, const float* w2, int ldw, float* y,
                       const hyres_epilogue* e, void* ws, long long ws_bytes, hyres_stream_t s) {
    HY_REQUIRE(g && x && w2 && y && e, HYRES_E_ARG, "conv_forward: NULL argument");
    HY_REQUIRE(g->nphase >= 1 && g->nphase <= 4 && g->Ci > 0 && g->Co > 0, HYRES_E_SHAPE, "conv: bad geom");
    HY_REQUIRE(ldw >= g->ntaps * g->Ci, HYRES_E_SHAPE, "conv: ldw %d < ntaps*Ci %d", ldw, g->ntaps * g->Ci);
    ConvArgs a;
    a.g = *g; a.x = x; a.w2 = w2; a.ldw = ldw; a.y = y; a.e = *e;
    a.M = g->B * g->Hq * g->Wq;
    a.xcd = 1;
    a.prio = 1;
    a.b6sw = g_tune[19] != 0;
    const ConvChoice ch = choose_conv(g, e, aligned16(x) && aligned16(w2) && g->ldx % 4 == 0 && ldw % 4 == 0);
    ConvPlan plan = conv_plan(g, ch.tile);
    a.nsplit = 1;
    a.cps = 0;
    a.slab = nullptr;
    {
        auto al = [](const void* p, int ld) { return p == nullptr || (aligned16(p) && ld % 4 == 0); };
        // HYRES_EPI_SA_BWD reads aux0 ([P][2]) and aux2 (argmax), HYRES_EPI_ROWSCALE aux1 (the scale), one scalar per
        // pixel: no alignment needed
        const bool sa = e->kind == HYRES_EPI_SA_BWD, rs = e->kind == HYRES_EPI_ROWSCALE;
        a.vec4 = g->Co % 4 == 0 && al(y, g->ldy) && al(e->bias, 4) && al(e->res, e->ldres) && al(e->out2, e->ldo2) &&
                 (sa || al(e->aux0, e->ld0)) && (rs || al(e->aux1, e->ld1)) && (sa || al(e->aux2, e->ld2));
    }
    {
        const long long npo = (long long)g->B * g->Ho * g->Wo;
        const int ld = std::max(g->ldy, std::max(e->res ? e->ldres : 0, e->aux0 ? e->ld0 : 0));
        a.rsrc_ok = npo * ld * 4 < 0x7FFFFFF0LL;
    }
    const long long need = plan_ws_bytes(g, plan);
    if (!ch.narrow && plan.nsplit > 1 && ws && ws_bytes >= need) {  // without workspace: single pass (correct, slower)
        a.nsplit = plan.nsplit;
        a.cps = plan.cps;
        a.slab = (float*)ws;
        if (!aligned16(ws)) a.vec4 = 0;
    }
    {
        const long long wb = (long long)g->Co * ldw * 4;
        const long long img_bytes = (long long)g->Hi * g->Wi * g->ldx * 4;
        HY_REQUIRE(wb < 0x7FFFFFF0LL && 3 * img_bytes < 0x7FFFFFF0LL && (long long)g->Ho * g->Wo * g->ldy < 0x7FFFFFFFLL,
                   HYRES_E_SHAPE, "conv: per-image tensor too large for 32-bit offsets");
        a.w_bytes = (int)wb;
    }
    int mode;
    if (g->Ci % KT == 0) {
        HY_REQUIRE(aligned16(x) && aligned16(w2) && g->ldx % 4 == 0 && ldw % 4 == 0, HYRES_E_ALIGN,
                   "conv: vector path needs 16B-aligned x/w2 and ldx,ldw %% 4 == 0");
        mode = e->square_input ? 1 : 0;
    } else {
        HY_REQUIRE(g->nphase == 1 && !e->square_input, HYRES_E_SHAPE,
                   "conv: Ci %% 32 != 0 supported only single-phase, no square");
        mode = 2;
    }
    if (e->kind == HYRES_EPI_GDN || e->kind == HYRES_EPI_IGDN)
        HY_REQUIRE(e->aux0 && e->out2, HYRES_E_ARG, "conv: GDN epilogue needs aux0/out2");
    if (e->kind == HYRES_EPI_GDN_BWD || e->kind == HYRES_EPI_IGDN_BWD)
        HY_REQUIRE(e->aux0 && e->aux1 && e->aux2, HYRES_E_ARG, "conv: GDN bwd epilogue needs aux0..2");
    if (e->act == HYRES_ACT_PRELU) HY_REQUIRE(e->slope, HYRES_E_ARG, "conv: PReLU needs slope");
    HY_REQUIRE(e->io_f16 >= 0 && e->io_f16 <= 4, HYRES_E_ARG, "conv: io_f16 %d (fp16 X/Y bits, or AUX16 alone)",
               e->io_f16);
    if (e->io_f16 & 3) {
        HY_REQUIRE(e->io_f16 >= 1 && e->io_f16 <= 3 && (!(e->kind == HYRES_EPI_GDN_BWD || e->kind == HYRES_EPI_IGDN_BWD)
                                                         || (e->io_f16 & 2)),
                   HYRES_E_ARG, "conv: a fp16 GDN-backward epilogue needs fp16 Y (its operands share Y's dtype)");
        HY_REQUIRE(!(e->io_f16 & 1) || mode != 2, HYRES_E_ARG, "conv: fp16 X needs Ci %% 32 == 0");
        HY_REQUIRE(!ch.narrow || !(e->io_f16 & 2), HYRES_E_ARG, "conv: the Co <= 4 kernel writes fp32 only");
    }
    if (e->act == HYRES_ACT_RELU_MASK)
        HY_REQUIRE(e->aux0 && e->kind == HYRES_EPI_BIAS, HYRES_E_ARG, "conv: ReLU mask needs aux0, BIAS epilogue");
    if (e->act == HYRES_ACT_PRELU_MASK && e->kind == HYRES_EPI_SA_BWD) {  // round 6: the scale-1 PReLU on SA_BWD
        HY_REQUIRE(e->aux1 && e->ld1 >= 64 && e->slope && e->res && e->out2 && e->ldo2 >= HYRES_PRELU_PARTIALS &&
                       !e->accumulate,
                   HYRES_E_ARG, "conv: SA_BWD + PReLU mask needs aux1 (pre-activation of channels 0..63, ld1 >= 64), "
                   "slope, res (slope gradient), out2 (>= %d partials), no accumulate", HYRES_PRELU_PARTIALS);
    } else if (e->act == HYRES_ACT_PRELU_MASK) {
        HY_REQUIRE(e->aux0 && e->aux1 && e->aux2 && e->slope && e->kind == HYRES_EPI_BIAS && !e->accumulate &&
                       !e->out2 && e->io_f16 == 0 && !e->f16_operands && e->ld2 >= HYRES_PRELU_PARTIALS,
                   HYRES_E_ARG, "conv: PReLU mask needs aux0 (pre-activation), aux1 (slope gradient), aux2 (>= %d "
                   "partials), slope; BIAS, no accumulate / out2, fp32", HYRES_PRELU_PARTIALS);
        HY_REQUIRE(mode == 0 && a.vec4 && wres32_ok(g, e) && wres_bf6() &&
                       wres_blocks(g->Co / 32) * (g->Co / 32) <= HYRES_PRELU_PARTIALS,
                   HYRES_E_ARG, "conv: the PReLU-mask epilogue runs on conv3x3_wres_bf6_kernel only");
    }
    if (e->kind == HYRES_EPI_ROWSCALE)
        HY_REQUIRE(e->aux1 && !e->square_input && !e->accumulate, HYRES_E_ARG,
                   "conv: ROWSCALE needs aux1 (per-pixel scale), no square_input / accumulate");
    if (e->kind == HYRES_EPI_SA_BWD)
        HY_REQUIRE(e->aux0 && e->aux2 && e->ld0 >= 2 && !e->square_input &&
                       ((e->act == HYRES_ACT_NONE && !e->res && !e->out2) || e->act == HYRES_ACT_PRELU_MASK) &&
                       (!(e->io_f16 & 2) || stream_hf_cfg(g, e)),
                   HYRES_E_ARG, "conv: SA_BWD needs aux0 ([P][ld0 >= 2]) and aux2 (argmax), no act / res / out2, fp32 Y "
                   "(fp16 Y: conv1x1_stream_hf_kernel's 64 -> 192 only)");
    hipStream_t st = as_stream(s);
    if (ch.narrow) {
        a.nsplit = 1;
        dim3 grid(ceil_div(a.M, NARROW_PIX), g->nphase);
        switch (g->Co) {
            case 1: launch_narrow<1>(a, grid, st); break;
            case 2: launch_narrow<2>(a, grid, st); break;
            case 3: launch_narrow<3>(a, grid, st); break;
            default: launch_narrow<4>(a, grid, st); break;
        }
        return HY_LAUNCH_CHECK("conv_narrow_kernel");
    }
    if (mode == 0 && a.vec4 && wres32_ok(g, e)) {
        a.nsplit = 1;
        return launch_wres32(a, st);
    }
    if (mode == 0 && a.vec4 && halo16_ok(g, e)) {
        a.nsplit = 1;
        return wres16_ok(g) ? launch_wres16(a, st) : launch_halo16(a, st);
    }
    {
        const int cfg = stream_b6_cfg(g, e);
        const long long xb = (long long)a.M * g->ldx * 4;
        if (cfg && mode == 0 && a.vec4 && a.rsrc_ok && xb < 0x7FFFFFF0LL && aligned16(x) && aligned16(w2) &&
            ldw % 4 == 0) {
            a.x_bytes = (int)xb;
            a.nsplit = 1;
            return launch_stream_b6(a, cfg, st);
        }
    }
    {
        const int nt = stream_nt(g, e);
        const long long xb = (long long)a.M * g->ldx * 4;
        if (nt && mode == 0 && a.vec4 && xb < 0x7FFFFFF0LL && aligned16(x) && aligned16(w2) && ldw % 4 == 0) {
            a.x_bytes = (int)xb;
            a.nsplit = 1;
            return launch_stream(a, nt, g->Ci / 8, 0, st);
        }
    }
    {
        const int cfg = stream_hf_cfg(g, e);
        const long long xb = (long long)a.M * g->ldx * 2;
        if (cfg && mode == 0 && a.rsrc_ok && xb < 0x7FFFFFF0LL && aligned16(x) && aligned16(w2) && ldw % 4 == 0 &&
            (reinterpret_cast<uintptr_t>(y) & 7) == 0 && (reinterpret_cast<uintptr_t>(e->res) & 7) == 0 &&
            (reinterpret_cast<uintptr_t>(e->aux0) & 7) == 0 && (reinterpret_cast<uintptr_t>(e->out2) & 7) == 0) {
            a.x_bytes = (int)xb;
            a.nsplit = 1;
            return launch_stream_hf(a, cfg, st);
        }
    }
    // no other kernel implements SA_BWD with an fp16 Y (its epi_store4 instantiations leave the case out)
    HY_REQUIRE(!(e->kind == HYRES_EPI_SA_BWD && ((e->io_f16 & 2) || e->act == HYRES_ACT_PRELU_MASK)), HYRES_E_ARG,
               "conv: an fp16-Y or PReLU-mask SA_BWD input-gradient needs the streaming kernels (alignment / size / "
               "split mode)");
    {
        const int nt = stream_h_nt(g, e);
        const long long xb = (long long)a.M * g->ldx * 2;
        if (nt && mode == 0 && xb < 0x7FFFFFF0LL && aligned16(x) && aligned16(w2) && ldw % 4 == 0 &&
            (reinterpret_cast<uintptr_t>(y) & 7) == 0) {
            a.x_bytes = (int)xb;
            a.nsplit = 1;
            return launch_stream_h(a, nt, g->Ci / 16, st);
        }
    }
    int rc;
    switch (ch.tile) {
        case 0: rc = launch_fwd<2, 2, 2, 2>(a, mode, st); break;
        case 1: rc = launch_fwd<2, 1, 2, 2>(a, mode, st); break;
        case 3: rc = launch_fwd<1, 2, 2, 2>(a, mode, st); break;
        case 4: rc = launch_fwd<1, 1, 2, 2>(a, mode, st); break;
        default: rc = launch_fwd<1, 1, 4, 1>(a, mode, st); break;
    }
    if (rc || a.nsplit == 1) return rc;
    long long total = (long long)a.M * g->Co * g->nphase;
    const bool yh = (e->io_f16 & 2) != 0;
    if (a.vec4) {
        int blocks = (int)std::min<long long>((total / 4 + 255) / 256, 8192);
        if (yh) hipLaunchKernelGGL(conv_splitk_reduce4_kernel<true>, dim3(blocks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(conv_splitk_reduce4_kernel<false>, dim3(blocks), dim3(256), 0, st, a);
        return HY_LAUNCH_CHECK("conv_splitk_reduce4_kernel");
    }
    int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
    if (yh) hipLaunchKernelGGL(conv_splitk_reduce_kernel<true>, dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(conv_splitk_reduce_kernel<false>, dim3(blocks), dim3(256), 0, st, a);
    return HY_LAUNCH_CHECK("conv_splitk_reduce_kernel");
}

int hyres_conv_kernel_name(const hyres_conv_geom* g, const hyres_epilogue* e, int split, char* buf, int n) {
    HY_REQUIRE(g && e && buf && n > 0, HYRES_E_ARG, "conv_kernel_name: bad args");
    const ConvChoice ch = choose_conv(g, e, true);
    if (ch.narrow) {
        snprintf(buf, n, "%s<%d, %d>", narrow_strip_ok(g) ? "conv_narrow_strip_kernel" : "conv_narrow_kernel",
                 std::min(g->Co, 4), g->Ci == 64 ? 1 : 2);
        return 0;
    }
    if (ch.mode == 0 && wres32_ok(g, e)) {
        snprintf(buf, n, wres_bf6() ? "conv3x3_wres_bf6_kernel" : "conv3x3_wres_f32_kernel");
        return 0;
    }
    if (ch.mode == 0 && halo16_ok(g, e)) {
        snprintf(buf, n, "%s<%d>", wres16_ok(g) ? "conv3x3_wres_f16_kernel" : "conv3x3_halo_f16_kernel", e->io_f16 & 3);
        return 0;
    }
    {
        const int cfg = stream_b6_cfg(g, e);
        if (cfg && ch.mode == 0) {
            snprintf(buf, n, "conv1x1_stream_b6_kernel<%d, %d, %d, %s>", cfg & 15, (cfg >> 4) & 15, cfg >> 8,
                     g_tune[11] == 0 ? "false" : "true");
            return 0;
        }
    }
    {
        const int nt = stream_nt(g, e);
        if (nt && ch.mode == 0) {
            snprintf(buf, n, "conv1x1_stream_kernel<%d, %d%s>", nt, g->Ci / 8, e->f16_operands ? ", true" : "");
            return 0;
        }
        const int chf = stream_hf_cfg(g, e);
        if (chf && ch.mode == 0) {
            snprintf(buf, n, "conv1x1_stream_hf_kernel<%d, %d, %d>", chf & 15, (chf >> 4) & 15, chf >> 8);
            return 0;
        }
        const int nth = stream_h_nt(g, e);
        if (nth && ch.mode == 0) {  // (the launch also checks pointer alignment; the label assumes it)
            snprintf(buf, n, "conv1x1_stream_h_kernel<%d, %d>", nth, g->Ci / 16);
            return 0;
        }
    }
    static const char* tiles[5] = {"2, 2, 2, 2", "2, 1, 2, 2", "1, 1, 4, 1", "1, 2, 2, 2", "1, 1, 2, 2"};
    const bool f16 = e->f16_operands && ch.mode != 2;
    if (e->io_f16 & 3) {
        snprintf(buf, n, "conv_fwd_h_kernel<%s, %d, %s, %d>", tiles[ch.tile], ch.mode, split ? "true" : "false",
                 e->io_f16 & 3);
        return 0;
    }
    if (g_tune[7] == 1 && !f16 && ch.mode != 2) {
        const long long M = (long long)g->B * g->Hq * g->Wq;
        const bool db = ch.tile == 4 && (g_tune[20] == 1 || (g_tune[20] < 0 && M <= 16384));
        snprintf(buf, n, "%s<%s, %d, %s>", db ? "conv_fwd_b6db_kernel" : "conv_fwd_b6_kernel", tiles[ch.tile], ch.mode,
                 split ? "true" : "false");
        return 0;
    }
    snprintf(buf, n, "conv_fwd_kernel<%s, %d, %s, %s>", tiles[ch.tile], ch.mode, split ? "true" : "false",
             f16 ? "true" : "false");
    return 0;
}

int hyres_wgrad_desc_conv2d(hyres_wgrad_desc* d, int B, int H, int W, int Ci, int ldx, int Co, int ldy,
                            int KH, int KW, int stride, int pad, int dil) {
    HY_REQUIRE(d && KH * KW <= HYRES_MAX_TAPS, HYRES_E_ARG, "bad wgrad args");
    *d = hyres_wgrad_desc{};
    const int Ho = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
    const int Wo = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
    d->B = B; d->Hq = Ho; d->Wq = Wo;
    d->M = Co; d->ldp = ldy;
    d->N = Ci; d->ldq = ldx; d->Hqq = H; d->Wqq = W; d->sq = stride;
    d->ntaps = KH * KW;
    for (int kh = 0; kh < KH; ++kh)
        for (int kw = 0; kw < KW; ++kw) {
            d->dh[kh * KW + kw] = kh * dil - pad;
            d->dw[kh * KW + kw] = kw * dil - pad;
        }
    d->sm = Ci * KH * KW; d->sn = KH * KW; d->st = 1;
    return ok();
}

int hyres_wgrad_desc_deconv2d(hyres_wgrad_desc* d, int B, int H, int W, int Ci, int ldx, int Co, int ldy,
                              int K, int pad) {
    HY_REQUIRE(d && K * K <= HYRES_MAX_TAPS, HYRES_E_ARG, "bad wgrad args");
    *d = hyres_wgrad_desc{};
    d->B = B; d->Hq = H; d->Wq = W;
    d->M = Ci; d->ldp = ldx;
    d->N = Co; d->ldq = ldy; d->Hqq = 2 * H; d->Wqq = 2 * W; d->sq = 2;
    d->ntaps = K * K;
    for (int kh = 0; kh < K; ++kh)
        for (int kw = 0; kw < K; ++kw) {
            d->dh[kh * K + kw] = kh - pad;
            d->dw[kh * K + kw] = kw - pad;
        }
    d->sm = Co * K * K; d->sn = K * K; d->st = 1;
    return ok();
}

}  // extern "C"
