// Weight gradients (and bias column sums) for every Conv2d / ConvTranspose2d / GDN of the HyRES hot path on
// CDNA4 (gfx950): dW[t][m][n] = sum_q P[q][m] * Q[shift_t(q)][n] over the batch's pixels, split-K over pixel
// ranges into [nsplit][ntaps][M][N] slabs reduced in a fixed order (deterministic, no atomics).
#include "conv_common.h"

namespace hyres {


// ------------------------------------------------------------------------------------------------
// weight gradient:  out[t][m][n] = sum_q P[q][m] * Q[shift_t(q)][n]      (K = pixels q)
//   * a block owns one (m-tile, n-tile, group of NT taps, pixel split); the P chunk is staged once
//     and reused by all NT taps, only the shifted Q chunk is re-gathered per tap (L1/L2-hot);
//   * ``tapn``: taps folded into the column dimension (c = t*N + n) for N <= 16 (3-channel images),
//     so a 32-wide MFMA column tile is not 90% padding;
//   * blocks of one pixel split are consecutive in logical order and mapped onto one XCD so their
//     shared P/Q rows hit that XCD's L2;
//   * split-K partials go to a [nsplit][ntaps][M][N] slab, reduced deterministically.
// ------------------------------------------------------------------------------------------------
struct WgradArgs {
    hyres_wgrad_desc d;
    const float* p;
    const float* q;
    float* slab;  // [nsplit][ntaps][M][N]
    int chunks_per_split;
    int nchunks;
    int mtiles, ntiles, ngroups;
    int nblocks;  // logical blocks (grid padded to a multiple of 8 for the XCD remap)
    int tapn;
    float* bias_slab;  // [nsplit][M] column sums of P (the bias gradient) or NULL
};

template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int TM, int TN, int WAVES_M, int WAVES_N, int NT, bool VP, bool VQ, bool SQ>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradArgs a) {
    constexpr int BM = 32 * TM * WAVES_M;
    constexpr int BN = 32 * TN * WAVES_N;
    constexpr int PP = BM + 4, PQ = BN + 4;
    // double-buffered P/Q chunks (one barrier per step) when both fit the 64 KB static LDS
    constexpr bool DB = (BM + BN) <= 192;
    constexpr int NBUF = DB ? 2 : 1;
    __shared__ __attribute__((aligned(16))) float Psm[NBUF * KT * PP];
    __shared__ __attribute__((aligned(16))) float Qsm[NBUF * KT * PQ];
    float* Ps = Psm;
    float* Qs = Qsm;
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    // XCD-aware order: hardware block b runs on XCD b % 8; give each XCD a contiguous logical range
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int HqWq = d.Hq * d.Wq;
    const long long Qtot = (long long)d.B * HqWq;
    const bool tapn = a.tapn != 0;

    constexpr int P_V = VP ? (KT * BM / 4 / 256) : (KT * BM / 256);
    constexpr int Q_V = VQ ? (KT * BN / 4 / 256) : (KT * BN / 256);
    static_assert(P_V >= 1 && Q_V >= 1, "tile too small");
    float4 rp[VP ? P_V : 1], rq[VQ ? Q_V : 1];
    float sp[VP ? 1 : P_V], sq[VQ ? 1 : Q_V];

    // per-thread Q rows/columns (fixed for the whole kernel) and the pixel decode of the current chunk
    int q_row[Q_V], q_col[Q_V], q_tap[Q_V];
#pragma unroll
    for (int i = 0; i < Q_V; ++i) {
        const int e = tid + 256 * i;
        q_row[i] = VQ ? e / (BN / 4) : e / BN;
        const int c = n0 + (VQ ? (e % (BN / 4)) * 4 : e % BN);
        if (!VQ && tapn) {
            q_tap[i] = c / d.N;
            q_col[i] = c - q_tap[i] * d.N;
        } else {
            q_tap[i] = 0;
            q_col[i] = c;
        }
    }
    int q_b[Q_V], q_i[Q_V], q_j[Q_V];
    // pixel decode of each thread's Q rows: divisions once (first chunk of the split), then stepped by KT
    // pixels per chunk in raster order (q_b = -1 past the end)
    auto decode_rows = [&](int kc) {
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const long long qq = (long long)kc * KT + q_row[i];
            if (qq < Qtot) {
                q_b[i] = (int)(qq / HqWq);
                const int r = (int)(qq - (long long)q_b[i] * HqWq);
                q_i[i] = r / d.Wq;
                q_j[i] = r - q_i[i] * d.Wq;
            } else {
                q_b[i] = -1; q_i[i] = 0; q_j[i] = 0;
            }
        }
    };
    auto step_rows = [&]() {
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            if (q_b[i] < 0) continue;
            int j = q_j[i] + KT, ii = q_i[i], b = q_b[i];
            while (j >= d.Wq) { j -= d.Wq; ++ii; }
            while (ii >= d.Hq) { ii -= d.Hq; ++b; }
            q_j[i] = j; q_i[i] = ii; q_b[i] = b < d.B ? b : -1;
        }
    };
    auto load_p = [&](int kc) {
        const long long k0 = (long long)kc * KT;
        if constexpr (VP) {
#pragma unroll
            for (int i = 0; i < P_V; ++i) {
                const int e = tid + 256 * i;
                const int row = e / (BM / 4), c = (e % (BM / 4)) * 4;
                const long long qq = k0 + row;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (qq < Qtot && m0 + c < d.M) v = ld4(a.p + qq * d.ldp + m0 + c);
                rp[i] = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < P_V; ++i) {
                const int e = tid + 256 * i;
                const int row = e / BM, c = e % BM;
                const long long qq = k0 + row;
                float v = 0.f;
                if (qq < Qtot && m0 + c < d.M) v = a.p[qq * d.ldp + m0 + c];
                sp[i] = v;
            }
        }
    };
    auto load_q = [&](int t) {
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const int tt = tapn ? q_tap[i] : t;
            bool ok = q_b[i] >= 0 && q_col[i] < d.N && tt < d.ntaps;
            long long off = 0;
            if (ok) {
                const int ih = q_i[i] * d.sq + d.dh[tt], iw = q_j[i] * d.sq + d.dw[tt];
                ok = ih >= 0 && ih < d.Hqq && iw >= 0 && iw < d.Wqq;
                off = ((long long)(q_b[i] * d.Hqq + ih) * d.Wqq + iw) * d.ldq + q_col[i];
            }
            if constexpr (VQ) {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ok) v = ld4(a.q + off);
                if constexpr (SQ) { v.x *= v.x; v.y *= v.y; v.z *= v.z; v.w *= v.w; }
                rq[i] = v;
            } else {
                float v = ok ? a.q[off] : 0.f;
                if constexpr (SQ) v *= v;
                sq[i] = v;
            }
        }
    };
    auto store_p = [&]() {
        if constexpr (VP) {
#pragma unroll
            for (int i = 0; i < P_V; ++i) {
                const int e = tid + 256 * i;
                const int row = e / (BM / 4), c = (e % (BM / 4)) * 4;
                *reinterpret_cast<float4*>(&Ps[row * PP + c]) = rp[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < P_V; ++i) {
                const int e = tid + 256 * i;
                Ps[(e / BM) * PP + e % BM] = sp[i];
            }
        }
    };
    auto store_q = [&]() {
        if constexpr (VQ) {
#pragma unroll
            for (int i = 0; i < Q_V; ++i) {
                const int e = tid + 256 * i;
                *reinterpret_cast<float4*>(&Qs[q_row[i] * PQ + (e % (BN / 4)) * 4]) = rq[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < Q_V; ++i) {
                const int e = tid + 256 * i;
                Qs[q_row[i] * PQ + e % BN] = sq[i];
            }
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int lr = lane & 31, lh = lane >> 5;
    floatx16 acc[NT][TM][TN];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int k = 0; k < TN; ++k)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[j][i][k][r] = 0.f;

    // bias gradient = column sums of P over all pixels: one column tile / tap group per split does it
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float bsum = 0.f;
    const int kc_begin = split * a.chunks_per_split;
    const int kc_end = min(a.nchunks, kc_begin + a.chunks_per_split);
    if (kc_begin < kc_end) {
        decode_rows(kc_begin);
        load_p(kc_begin);
        load_q(t0);
    }
    if constexpr (DB) {
        // prologue: first step's operands in buffer 0; then per step: prefetch the next step's operands
        // into registers, MFMAs on the current buffers, store the prefetch into the other buffers, ONE barrier
        if (kc_begin < kc_end) {
            store_p();
            store_q();
        }
        __syncthreads();
        int pcur = 0, qcur = 0;
        for (int kc = kc_begin; kc < kc_end; ++kc) {
            static_for<NT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                Ps = Psm + pcur * (KT * PP);
                Qs = Qsm + qcur * (KT * PQ);
                const bool next_tap = j + 1 < NT;
                const bool next_chunk = !next_tap && kc + 1 < kc_end;
                if (next_tap) {
                    load_q(t0 + j + 1);
                } else if (next_chunk) {
                    step_rows();
                    load_p(kc + 1);
                    load_q(t0);
                }
                if (j == 0 && do_bias && tid < BM) {
#pragma unroll 8
                    for (int k = 0; k < KT; ++k) bsum += Ps[k * PP + tid];
                }
#pragma unroll
                for (int s = 0; s < KT / 2; ++s) {
                    const int k = lh * (KT / 2) + s;
                    float af[TM], bf[TN];
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm) af[tm] = Ps[k * PP + wm * TM * 32 + tm * 32 + lr];
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) bf[tn] = Qs[k * PQ + wn * TN * 32 + tn * 32 + lr];
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn)
                            acc[j][tm][tn] =
                                __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm], bf[tn], acc[j][tm][tn], 0, 0, 0);
                }
                if (next_tap || next_chunk) {
                    Qs = Qsm + (qcur ^ 1) * (KT * PQ);
                    store_q();
                    if (next_chunk) {
                        Ps = Psm + (pcur ^ 1) * (KT * PP);
                        store_p();
                    }
                }
                __syncthreads();
                qcur ^= 1;
                if (!next_tap) pcur ^= 1;
            });
        }
    } else {
        for (int kc = kc_begin; kc < kc_end; ++kc) {
            static_for<NT>([&](auto J) {
                constexpr int j = decltype(J)::value;
                __syncthreads();
                if (j == 0) store_p();
                store_q();
                __syncthreads();
                if (j == 0 && do_bias && tid < BM) {
    #pragma unroll 8
                    for (int k = 0; k < KT; ++k) bsum += Ps[k * PP + tid];
                }
                if (j + 1 < NT) {
                    load_q(t0 + j + 1);
                } else if (kc + 1 < kc_end) {
                    step_rows();
                    load_p(kc + 1);
                    load_q(t0);
                }
    #pragma unroll
                for (int s = 0; s < KT / 2; ++s) {
                    const int k = lh * (KT / 2) + s;
                    float af[TM], bf[TN];
    #pragma unroll
                    for (int tm = 0; tm < TM; ++tm) af[tm] = Ps[k * PP + wm * TM * 32 + tm * 32 + lr];
    #pragma unroll
                    for (int tn = 0; tn < TN; ++tn) bf[tn] = Qs[k * PQ + wn * TN * 32 + tn * 32 + lr];
    #pragma unroll
                    for (int tm = 0; tm < TM; ++tm)
    #pragma unroll
                        for (int tn = 0; tn < TN; ++tn)
                            acc[j][tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm], bf[tn], acc[j][tm][tn], 0, 0, 0);
                }
            });
        }
    }
    if (do_bias && tid < BM && m0 + tid < d.M) a.bias_slab[(long long)split * d.M + m0 + tid] = bsum;
    // slab store [split][t][M][N]
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int c = n0 + wn * TN * 32 + tn * 32 + lr;
            int t = t0 + j, n = c;
            if (tapn) { t = c / d.N; n = c - t * d.N; }
            if (n >= d.N || t >= d.ntaps) continue;
            float* out = a.slab + ((long long)split * d.ntaps + t) * MN + n;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (m < d.M) out[(long long)m * d.N] = acc[j][tm][tn][r];
                }
        }
    });
}


// ------------------------------------------------------------------------------------------------
// Halo-staged weight gradient for KxK convolutions / transposed convolutions at Q stride SQ = 1 or 2 (K = 3:
// one block does all 9 taps; K = 5: one kernel row of 5 taps per block) whose base rows are a multiple of
// 32 pixels, so a 32-pixel K chunk is one row segment (b, i, j0..j0+31). Per chunk the block stages P
// (32 px x 64 m) and ONE Q halo tile (KR rows x (31*SQ + K) px x 64 n) in LDS, double-buffered, and every
// tap reads its B operand from the halo at its (dh, dw) shift (pixel k at column k*SQ + dw). The generic kernel instead gathers a shifted 32-px Q chunk per tap (9 global loads
// and 9 barriers per chunk, the latency of each exposed at 2 blocks per CU); here it is one load of
// 3 x 34 px per chunk and one barrier per 9 x 16 MFMAs. 64 x 64 tiles, 4 waves of 32 x 32.
// ------------------------------------------------------------------------------------------------
// 1x1 weight gradient (stride 1, fp32, 16B-aligned P/Q): dW[m][n] = sum_p P[p][m] Q[p][n] over the split's
// pixel range. P and Q rows of one 32-pixel chunk are the same pixels, so both load as contiguous float4
// rows (no tap shift / pixel decode); double-buffered [pixel][channel] LDS tiles, one barrier per chunk;
// the bias gradient (column sums of P) rides on the A operand already in registers (one VALU add per
// MFMA step in the wn == 0 waves) instead of a serial LDS pass per chunk.
// G > 1: G groups of 4 waves per block, each over its own contiguous share of the block's pixel range with its
// own LDS tiles, their tiles summed through LDS before the one slab write: the same grid of waves writes 1/G of
// the split slabs (and the reduce reads 1/G), at 2 x (for G = 2) the LDS per block.
template <int TM, int TN, int WAVES_M, int WAVES_N, int G = 1>
__global__ __launch_bounds__(256 * G) void wgrad1x1_kernel(const WgradArgs a) {
    constexpr int BM = 32 * TM * WAVES_M, BN = 32 * TN * WAVES_N;
    constexpr int PP = BM + 4, PQ = BN + 4;
    constexpr int P_V = KT * BM / 4 / 256, Q_V = KT * BN / 4 / 256;
    static_assert(P_V >= 1 && Q_V >= 1, "tile too small");
    static_assert(G == 1 || G * 2 * KT * PP >= BM * BN + BM, "LDS for the group combine");
    __shared__ __attribute__((aligned(16))) float Psm_all[G * 2 * KT * PP];
    __shared__ __attribute__((aligned(16))) float Qsm_all[G * 2 * KT * PQ];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x & 255, grp = threadIdx.x >> 8;
    float* const Psm = Psm_all + grp * (2 * KT * PP);
    float* const Qsm = Qsm_all + grp * (2 * KT * PQ);
    // G > 1 (512 threads, LDS-limited to 1-2 blocks per CU): the blocks take the whole VGPR file of their SIMDs, as
    // every persistent 512-thread kernel does (DESIGN §4 "Cross-kernel interference": the observed hogs were 512-thread,
    // LDS-limited blocks leaving a hole other kernels' waves ran in, with or without v_cvt_pk). 1 block per CU: 2 waves
    // x 256; 2 blocks: 4 waves x 128. Costs nothing: LDS, not registers, sets the occupancy.
    if constexpr (G > 1) {
        constexpr int lds_bytes = (int)sizeof(float) * G * 2 * KT * (PP + PQ);
        constexpr int blocks = 163840 / lds_bytes;
        static_assert(blocks >= 1 && blocks <= 2, "wgrad1x1_kernel<G>1>: 1 or 2 blocks per CU");
        if constexpr (blocks == 2) asm volatile("" ::: "v127");
        else asm volatile("" ::: "v255");
    }
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int split = rr;
    const int m0 = mt * BM, n0 = nt * BN;
    const long long Qtot = (long long)d.B * d.Hq * d.Wq;
    float4 rp[P_V], rq[Q_V];
    auto load = [&](int kc) {
        const long long k0 = (long long)kc * KT;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            const int e = tid + 256 * i;
            const int row = e / (BM / 4), c = (e % (BM / 4)) * 4;
            rp[i] = (k0 + row < Qtot && m0 + c < d.M) ? ld4(a.p + (k0 + row) * d.ldp + m0 + c)
                                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const int e = tid + 256 * i;
            const int row = e / (BN / 4), c = (e % (BN / 4)) * 4;
            rq[i] = (k0 + row < Qtot && n0 + c < d.N) ? ld4(a.q + (k0 + row) * d.ldq + n0 + c)
                                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](int buf) {
        float* Ps = Psm + buf * (KT * PP);
        float* Qs = Qsm + buf * (KT * PQ);
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            const int e = tid + 256 * i;
            *reinterpret_cast<float4*>(&Ps[(e / (BM / 4)) * PP + (e % (BM / 4)) * 4]) = rp[i];
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const int e = tid + 256 * i;
            *reinterpret_cast<float4*>(&Qs[(e / (BN / 4)) * PQ + (e % (BN / 4)) * 4]) = rq[i];
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
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && wn == 0;
    float bsum[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) bsum[i] = 0.f;
    // the block's chunks [kb0, ke0), this group's contiguous share [kb, ke); every group runs `iters` barrier
    // steps (a group with fewer chunks idles through its last one)
    const int kb0 = split * a.chunks_per_split;
    const int ke0 = min(a.nchunks, kb0 + a.chunks_per_split);
    const int share = (max(ke0 - kb0, 0) + G - 1) / G;
    const int kb = min(ke0, kb0 + grp * share), ke = min(ke0, kb + share);
    const int iters = share;
    if (kb < ke) {
        load(kb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < iters; ++it) {
        const int kc = kb + it;
        const bool live = kc < ke;
        const bool next = kc + 1 < ke;
        if (next) load(kc + 1);  // in flight during this chunk's MFMAs
        if (live) {
            const float* Ps = Psm + cur * (KT * PP);
            const float* Qs = Qsm + cur * (KT * PQ);
#pragma unroll
            for (int s2 = 0; s2 < KT / 2; ++s2) {
                const int k = 2 * s2 + lh;
                float av[TM], bv[TN];
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) av[tm] = Ps[k * PP + wm * TM * 32 + tm * 32 + lr];
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) bv[tn] = Qs[k * PQ + wn * TN * 32 + tn * 32 + lr];
                if (do_bias) {
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm) bsum[tm] += av[tm];
                }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
            }
        }
        if (next) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if constexpr (G > 1) {
        // groups 1.. hand their tiles (accumulator layout, lane-major) and bias sums to group 0 through LDS;
        // group 0 adds them in group order (deterministic) before the slab write
        float* red = Psm_all;  // the loop ended with a barrier; the combine area spans groups 1.. of the LDS
        constexpr int TILE = BM * BN;
        for (int g2 = 1; g2 < G; ++g2) {
            if (grp == g2) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            red[(((wave * TM + tm) * TN + tn) * 16 + r) * 64 + lane] = acc[tm][tn][r];
                if (do_bias) {
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm) red[TILE + (wave * TM + tm) * 64 + lane] = bsum[tm];
                }
            }
            __syncthreads();
            if (grp == 0) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            acc[tm][tn][r] += red[(((wave * TM + tm) * TN + tn) * 16 + r) * 64 + lane];
                if (do_bias) {
#pragma unroll
                    for (int tm = 0; tm < TM; ++tm) bsum[tm] += red[TILE + (wave * TM + tm) * 64 + lane];
                }
            }
            __syncthreads();
        }
        if (grp != 0) return;
    }
    if (do_bias) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const float t = bsum[tm] + __shfl_xor(bsum[tm], 32);  // the two lane halves cover even / odd pixels
            const int m = m0 + wm * TM * 32 + tm * 32 + lr;
            if (lh == 0 && m < d.M) a.bias_slab[(long long)split * d.M + m] = t;
        }
    }
    const long long MN = (long long)d.M * d.N;
    float* out = a.slab + (long long)split * MN;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * TN * 32 + tn * 32 + lr;
            if (n >= d.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N + n] = acc[tm][tn][r];
            }
        }
}

// G groups of 256 threads of one block accumulated the same output tile over disjoint pixel ranges: add groups
// 1..G-1 into group 0's floatx16 acc[NT] in group order (deterministic), CH taps per pass through `red`
// (RED floats of LDS; thread-major so every wave's stores and loads are conflict-free). All threads call it.
template <int NT, int G, int RED>
__device__ __forceinline__ void combine_groups(floatx16 (&acc)[NT], float* red, int tid, int gq) {
    constexpr int CH = RED / (16 * 256) < NT ? RED / (16 * 256) : NT;
    static_assert(CH >= 1, "LDS too small for one tap");
    constexpr int NCH = (NT + CH - 1) / CH;
    static_for<NCH>([&](auto C) {
        constexpr int c0 = decltype(C)::value * CH;
        for (int g2 = 1; g2 < G; ++g2) {
            if (gq == g2)
                static_for<NT>([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    if constexpr (j >= c0 && j < c0 + CH) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) red[((j - c0) * 16 + r) * 256 + tid] = acc[j][r];
                    }
                });
            __syncthreads();
            if (gq == 0)
                static_for<NT>([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    if constexpr (j >= c0 && j < c0 + CH) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[j][r] += red[((j - c0) * 16 + r) * 256 + tid];
                    }
                });
            __syncthreads();
        }
    });
}

// G = 2 (round 3): two 4-wave groups per 512-thread block share one pixel split (each its own contiguous half of
// the split's chunks and its own LDS buffers: 1 block of 8 waves per CU instead of 2 of 4) and are summed through
// LDS before the slab write, so the same waves write and the deferred reduce reads half the split slab.
template <int KR, int KW, int SQ, int DIL = 1, int G = 1>
__global__ __launch_bounds__(256 * G, G == 1 ? 2 : 1) void wgrad_halo_kernel(const WgradArgs a, int dhg, int dwg) {
    // DIL: tap spacing (2: MultiScaleRefine's dilated 3x3, enhancement.py:44-51): the KR halo rows are DIL
    // rows apart, the halo columns span 31*SQ + DIL*(KW-1) + 1 pixels
    constexpr int BM = 64, BN = 64, NT = KR * KW, HC = 31 * SQ + DIL * (KW - 1) + 1;  // halo columns of a 32-px chunk
    constexpr int PP = BM + 4, PQ = BN + 4;
    constexpr int PSZ = KT * PP, HSZ = KR * HC * PQ;
    constexpr int P_V = KT * BM / 4 / 256;
    constexpr int H_E = KR * HC * (BN / 4);
    constexpr int H_V = (H_E + 255) / 256;
    __shared__ __attribute__((aligned(16))) float smem_all[G * 2 * (PSZ + HSZ)];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x & 255, gq = threadIdx.x >> 8;
    float* const smem = smem_all + gq * (2 * (PSZ + HSZ));
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int dh0 = dhg + grp * KR * DIL;  // the group's first kernel row offset, first column offset dwg
    const int cpr = d.Wq / 32;
    float4 rp[P_V], rh[H_V];
    auto load = [&](int kc) {
        const int b = kc / (d.Hq * cpr);
        const int rem = kc - b * d.Hq * cpr;
        const int i = rem / cpr;
        const int j0 = (rem - i * cpr) * 32;
        const long long q0 = (long long)kc * 32;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            const int e = tid + 256 * q;
            const int row = e / (BM / 4), c = (e % (BM / 4)) * 4;
            rp[q] = m0 + c < d.M ? ld4(a.p + (q0 + row) * d.ldp + m0 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            const int pix = e / (BN / 4), c = (e % (BN / 4)) * 4;
            const int hr = pix / HC, hc = pix - (pix / HC) * HC;
            const int ih = i * SQ + dh0 + DIL * hr, iw = j0 * SQ + dwg + hc;
            const bool ok = e < H_E && (unsigned)ih < (unsigned)d.Hqq && (unsigned)iw < (unsigned)d.Wqq && n0 + c < d.N;
            rh[q] = ok ? ld4(a.q + ((long long)(b * d.Hqq + ih) * d.Wqq + iw) * d.ldq + n0 + c)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    // bias gradient = column sums of P, accumulated from the staging registers (this thread's channel
    // quad (tid % 16) * 4 is fixed) and reduced once at the end: a per-chunk LDS column pass in one wave
    // held every barrier back by that wave's extra work (256^2 3x3: 676 vs 617 us without bias)
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto store = [&](int buf) {
        float* Ps = smem + buf * (PSZ + HSZ);
        float* Hs = Ps + PSZ;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            const int e = tid + 256 * q;
            if (do_bias) { bsum.x += rp[q].x; bsum.y += rp[q].y; bsum.z += rp[q].z; bsum.w += rp[q].w; }
            *reinterpret_cast<float4*>(&Ps[(e / (BM / 4)) * PP + (e % (BM / 4)) * 4]) = rp[q];
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            if (e < H_E) *reinterpret_cast<float4*>(&Hs[(e / (BN / 4)) * PQ + (e % (BN / 4)) * 4]) = rh[q];
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;
    floatx16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    // the split's chunks [kb0, ke0), this group's contiguous share [kb, ke); every group runs `iters` barrier
    // steps (a group with fewer chunks idles through its last ones)
    const int kb0 = split * a.chunks_per_split;
    const int ke0 = min(a.nchunks, kb0 + a.chunks_per_split);
    const int share = (max(ke0 - kb0, 0) + G - 1) / G;
    const int kb = min(ke0, kb0 + gq * share), ke = min(ke0, kb + share);
    if (kb < ke) {
        load(kb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < share; ++it) {
        const int kc = kb + it;
        const bool next = kc + 1 < ke;
        if (next) load(kc + 1);  // next chunk in flight during this chunk's NT x 16 MFMAs
        if (kc < ke) {
            const float* Ps = smem + cur * (PSZ + HSZ);
            const float* Hs = Ps + PSZ;
            static_for<NT>([&](auto J) {
                constexpr int t = decltype(J)::value;
                constexpr int hr = t / KW, hc = t % KW;
#pragma unroll
                for (int s2 = 0; s2 < KT / 2; ++s2) {
                    const int k = lh * (KT / 2) + s2;
                    const float af = Ps[k * PP + wm * 32 + lr];
                    const float bf = Hs[(hr * HC + k * SQ + DIL * hc) * PQ + wn * 32 + lr];
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, acc[t], 0, 0, 0);
                }
            });
        }
        if (next) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem_all);  // the loop ended with a barrier
        red[threadIdx.x] = bsum;
        __syncthreads();
        if (threadIdx.x < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < 256 * G / (BM / 4); ++r) {
                const float4 v = red[threadIdx.x + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
        __syncthreads();
    }
    if constexpr (G > 1) {
        combine_groups<NT, G, G * 2 * (PSZ + HSZ)>(acc, smem_all, tid, gq);
        if (gq != 0) return;
    }
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int n = n0 + wn * 32 + lr;
        if (n < d.N) {
            float* out = a.slab + ((long long)split * d.ntaps + t0 + j) * MN + n;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N] = acc[j][r];
            }
        }
    });
}


// ------------------------------------------------------------------------------------------------
// AMP weight gradient (train.sh --mixed-precision): the same GEMM dW[t][m][n] = sum_q P[q][m] Q_t[q][n]
// with P and Q rounded to fp16 when staged and consumed by v_mfma_f32_32x32x16_f16 (fp32 accumulation,
// fp32 bias sums from the unrounded P).  Chunks of KTH = 64 pixels are staged exactly as they arrive
// from HBM — [k][channel] rows, 4 channels (8 bytes) per ds_write_b64 — and read back transposed with
// ds_read_b64_tr_b16, which hands each lane the 8 consecutive k of its row/column the MFMA wants.  Row
// pitch = BM + 32 halves: the four rows of one transposed read land on disjoint banks.  Double-buffered
// (one barrier per tap step).  Requires the vector path (M, N, ldp, ldq % 4 == 0) and no tap folding.
// ------------------------------------------------------------------------------------------------
constexpr int KTH = 64;

// a staged operand quad: raw halves when the operand is fp16 in HBM (kept unconverted until the LDS store, so
// the prefetch of the next chunk does not wait for its data), fp32 otherwise
template <bool H>
using quad_t = std::conditional_t<H, half4_t, float4>;
template <bool H>
__device__ __forceinline__ quad_t<H> ldq4(const float* p, long long i) {
    if constexpr (H) return *reinterpret_cast<const half4_t*>(reinterpret_cast<const _Float16*>(p) + i);
    else return ld4(p + i);
}
template <bool H>
__device__ __forceinline__ quad_t<H> zq4() {
    if constexpr (H) return half4_t{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    else return make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ float4 q2f(const float4& v) { return v; }
__device__ __forceinline__ float4 q2f(const half4_t& v) {
    return make_float4((float)v.x, (float)v.y, (float)v.z, (float)v.w);
}
__device__ __forceinline__ half4_t q2h(const half4_t& v) { return v; }
__device__ __forceinline__ half4_t q2h(const float4& v) {
    return half4_t{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
}
typedef __fp16 fp16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 halfx4_t __attribute__((ext_vector_type(4)));
typedef _Float16 halfx8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ halfx4_t lds_tr4(const _Float16* p) {
    fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_t*)(p));
    return __builtin_bit_cast(halfx4_t, v);
}

// ONE: a 1x1 stride-1 gradient on the base grid (Q row = P row): Q rows load like P rows, no pixel decode.
// IOH: operands stored fp16 in HBM (AMP training's saved activations): bit 0 P, bit 1 Q (8-byte loads of 4
// channels; the fp16 -> fp32 -> fp16 round trip into LDS is exact).
template <int TM, int TN, int WAVES_M, int WAVES_N, int NT, bool SQ, bool ONE = false, int IOH = 0>
__global__ __launch_bounds__(256) void wgrad_f16_kernel(const WgradArgs a) {
    constexpr bool PH = (IOH & 1) != 0, QH = (IOH & 2) != 0;
    constexpr int BM = 32 * TM * WAVES_M;
    constexpr int BN = 32 * TN * WAVES_N;
    constexpr int PP = BM + 32, PQ = BN + 32;  // halves
    __shared__ __attribute__((aligned(16))) _Float16 Psm[2 * KTH * PP];
    __shared__ __attribute__((aligned(16))) _Float16 Qsm[2 * KTH * PQ];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int HqWq = d.Hq * d.Wq;
    const long long Qtot = (long long)d.B * HqWq;

    constexpr int P_V = KTH * BM / 4 / 256, Q_V = KTH * BN / 4 / 256;
    static_assert(P_V >= 1 && Q_V >= 1, "tile too small");
    quad_t<PH> rp[P_V];
    quad_t<QH> rq[Q_V];
    // fixed per-thread channel quad (256 % (B/4) == 0): rows are tid/(B/4) + i*256/(B/4)
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);
    const int qc = (tid % (BN / 4)) * 4, qrow0 = tid / (BN / 4);
    constexpr int PRS = 256 / (BM / 4), QRS = 256 / (BN / 4);
    int q_b[Q_V], q_i[Q_V], q_j[Q_V];
    auto decode_rows = [&](int kc) {
        if constexpr (ONE) return;
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const long long qq = (long long)kc * KTH + qrow0 + i * QRS;
            if (qq < Qtot) {
                q_b[i] = (int)(qq / HqWq);
                const int r = (int)(qq - (long long)q_b[i] * HqWq);
                q_i[i] = r / d.Wq;
                q_j[i] = r - q_i[i] * d.Wq;
            } else {
                q_b[i] = -1; q_i[i] = 0; q_j[i] = 0;
            }
        }
    };
    auto step_rows = [&]() {
        if constexpr (ONE) return;
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            if (q_b[i] < 0) continue;
            int j = q_j[i] + KTH, ii = q_i[i], b = q_b[i];
            while (j >= d.Wq) { j -= d.Wq; ++ii; }
            while (ii >= d.Hq) { ii -= d.Hq; ++b; }
            q_j[i] = j; q_i[i] = ii; q_b[i] = b < d.B ? b : -1;
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto load_p = [&](int kc) {
        const long long k0 = (long long)kc * KTH;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            const long long qq = k0 + prow0 + i * PRS;
            rp[i] = (qq < Qtot && m0 + pc < d.M) ? ldq4<PH>(a.p, qq * d.ldp + m0 + pc) : zq4<PH>();
        }
    };
    int cur_kc = 0;  // ONE: the chunk load_q fetches (Q rows = P rows)
    auto load_q = [&](int t) {
        if constexpr (ONE) {
            const long long k0 = (long long)cur_kc * KTH;
#pragma unroll
            for (int i = 0; i < Q_V; ++i) {
                const long long qq = k0 + qrow0 + i * QRS;
                rq[i] = (qq < Qtot && n0 + qc < d.N) ? ldq4<QH>(a.q, qq * d.ldq + n0 + qc) : zq4<QH>();
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            quad_t<QH> v = zq4<QH>();
            if (q_b[i] >= 0 && n0 + qc < d.N && t < d.ntaps) {
                const int ih = q_i[i] * d.sq + d.dh[t], iw = q_j[i] * d.sq + d.dw[t];
                if (ih >= 0 && ih < d.Hqq && iw >= 0 && iw < d.Wqq)
                    v = ldq4<QH>(a.q, ((long long)(q_b[i] * d.Hqq + ih) * d.Wqq + iw) * d.ldq + n0 + qc);
            }
            rq[i] = v;  // SQ: squared at the LDS store
        }
    };
    auto store_p = [&](_Float16* Ps) {
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            if (do_bias) {
                const float4 f = q2f(rp[i]);
                bsum.x += f.x; bsum.y += f.y; bsum.z += f.z; bsum.w += f.w;
            }
            *reinterpret_cast<half4_t*>(&Ps[(prow0 + i * PRS) * PP + pc]) = q2h(rp[i]);
        }
    };
    auto store_q = [&](_Float16* Qs) {
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            half4_t h;
            if constexpr (SQ) {
                const float4 f = q2f(rq[i]);
                h = q2h(make_float4(f.x * f.x, f.y * f.y, f.z * f.z, f.w * f.w));
            } else {
                h = q2h(rq[i]);
            }
            *reinterpret_cast<half4_t*>(&Qs[(qrow0 + i * QRS) * PQ + qc]) = h;
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    // transposed-read address of this lane: half h = lane>>5 takes k rows 8h..8h+7 of each 16-k step; in
    // its 16-lane group g, lane 4q+p supplies row (.. + q), columns 16g + 4p .. +3
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    floatx16 acc[NT][TM][TN];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int k = 0; k < TN; ++k)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[j][i][k][r] = 0.f;

    const int kc_begin = split * a.chunks_per_split;
    const int kc_end = min(a.nchunks, kc_begin + a.chunks_per_split);
    if (kc_begin < kc_end) {
        decode_rows(kc_begin);
        load_p(kc_begin);
        cur_kc = kc_begin;
        load_q(t0);
        store_p(Psm);
        store_q(Qsm);
    }
    __syncthreads();
    int pcur = 0, qcur = 0;
    for (int kc = kc_begin; kc < kc_end; ++kc) {
        static_for<NT>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const _Float16* Ps = Psm + pcur * (KTH * PP);
            const _Float16* Qs = Qsm + qcur * (KTH * PQ);
            const bool next_tap = j + 1 < NT;
            const bool next_chunk = !next_tap && kc + 1 < kc_end;
            if (next_tap) {
                load_q(t0 + j + 1);
            } else if (next_chunk) {
                step_rows();
                load_p(kc + 1);
                cur_kc = kc + 1;
                load_q(t0);
            }
#pragma unroll
            for (int s = 0; s < KTH / 16; ++s) {
                halfx8_t af[TM], bf[TN];
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    const _Float16* src = Ps + (16 * s + tr_row) * PP + wm * TM * 32 + tm * 32 + tr_col;
                    const halfx4_t lo = lds_tr4(src), hi = lds_tr4(src + 4 * PP);
                    af[tm] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                }
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const _Float16* src = Qs + (16 * s + tr_row) * PQ + wn * TN * 32 + tn * 32 + tr_col;
                    const halfx4_t lo = lds_tr4(src), hi = lds_tr4(src + 4 * PQ);
                    bf[tn] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                }
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[j][tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[tm], bf[tn], acc[j][tm][tn], 0, 0, 0);
            }
            if (next_tap || next_chunk) {
                store_q(Qsm + (qcur ^ 1) * (KTH * PQ));
                if (next_chunk) store_p(Psm + (pcur ^ 1) * (KTH * PP));
            }
            __syncthreads();
            qcur ^= 1;
            if (!next_tap) pcur ^= 1;
        });
    }
    if (do_bias) {
        // fp32 column sums of this thread's rows -> reduce the PRS threads that share a channel quad
        float4* red = reinterpret_cast<float4*>(Psm);  // the loop ended with a barrier
        red[tid] = bsum;
        __syncthreads();
        if (tid < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < PRS; ++r) {
                const float4 v = red[tid + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
    }
    // slab store [split][t][M][N] (accumulator layout of v_mfma_f32_32x32x16_f16 = the 32x32x2 f32 one)
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * TN * 32 + tn * 32 + lr;
            const int t = t0 + j;
            if (n >= d.N || t >= d.ntaps) continue;
            float* out = a.slab + ((long long)split * d.ntaps + t) * MN + n;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (m < d.M) out[(long long)m * d.N] = acc[j][tm][tn][r];
                }
        }
    });
}

// ------------------------------------------------------------------------------------------------
// AMP halo-staged weight gradient: wgrad_halo_kernel's schedule (one 32-pixel row segment of P and ONE
// Q halo tile of KR rows x HC columns per chunk, all KR x KW taps of the group read from the halo at their
// (dh, dw) shift, one barrier per chunk) with wgrad_f16_kernel's operands: both tiles rounded to fp16 when
// staged ([pixel][channel] rows, pitch 64 + 32 halves) and read back transposed with ds_read_b64_tr_b16
// into v_mfma_f32_32x32x16_f16 (fp32 accumulation). The generic f16 kernel gathers a shifted Q chunk per
// tap (one tap per block, 9x the Q loads); here a 3x3 group costs one 3 x 34-pixel halo load per chunk.
// The tap's B rows are halo rows base + k*SQ: the transposed read takes per-lane addresses, so the stride
// is just a pitch of SQ*PQ. Bias gradient = fp32 column sums of the unrounded P (as wgrad_f16_kernel).
// ------------------------------------------------------------------------------------------------
template <int KR, int KW, int SQ, int DIL = 1, int IOH = 0, int G = 1>  // G: as wgrad_halo_kernel
__global__ __launch_bounds__(256 * G, G == 1 ? 2 : 1) void wgrad_halo_f16_kernel(const WgradArgs a, int dhg, int dwg) {
    constexpr bool PH = (IOH & 1) != 0, QH = (IOH & 2) != 0;  // fp16 operands in HBM (wgrad_f16_kernel)
    constexpr int BM = 64, BN = 64, NT = KR * KW, HC = 31 * SQ + DIL * (KW - 1) + 1;
    constexpr int PP = BM + 32, PQ = BN + 32;  // halves
    constexpr int PSZ = KT * PP, HSZ = KR * HC * PQ;
    constexpr int P_V = KT * BM / 4 / 256;  // 2 float4 of P per thread and chunk
    constexpr int H_E = KR * HC * (BN / 4);
    constexpr int H_V = (H_E + 255) / 256;
    static_assert((PSZ + HSZ) % 4 == 0, "8-byte aligned buffers for the transposed reads");
    __shared__ __attribute__((aligned(16))) _Float16 smem_all[G * 2 * (PSZ + HSZ)];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x & 255, gq = threadIdx.x >> 8;
    _Float16* const smem = smem_all + gq * (2 * (PSZ + HSZ));
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int dh0 = dhg + grp * KR * DIL;
    const int cpr = d.Wq / 32;
    // this thread's fixed channel quad of P (256 % (BM/4) == 0): rows tid/16 + 16*q
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);
    quad_t<PH> rp[P_V];
    quad_t<QH> rh[H_V];
    auto load = [&](int kc) {
        const int b = kc / (d.Hq * cpr);
        const int rem = kc - b * d.Hq * cpr;
        const int i = rem / cpr;
        const int j0 = (rem - i * cpr) * 32;
        const long long q0 = (long long)kc * 32;
#pragma unroll
        for (int q = 0; q < P_V; ++q)
            rp[q] = m0 + pc < d.M ? ldq4<PH>(a.p, (q0 + prow0 + 16 * q) * d.ldp + m0 + pc) : zq4<PH>();
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            const int pix = e / (BN / 4), c = (e % (BN / 4)) * 4;
            const int hr = pix / HC, hc = pix - (pix / HC) * HC;
            const int ih = i * SQ + dh0 + DIL * hr, iw = j0 * SQ + dwg + hc;
            const bool ok = e < H_E && (unsigned)ih < (unsigned)d.Hqq && (unsigned)iw < (unsigned)d.Wqq && n0 + c < d.N;
            rh[q] = ok ? ldq4<QH>(a.q, ((long long)(b * d.Hqq + ih) * d.Wqq + iw) * d.ldq + n0 + c) : zq4<QH>();
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto store = [&](int buf) {
        _Float16* Ps = smem + buf * (PSZ + HSZ);
        _Float16* Hs = Ps + PSZ;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            if (do_bias) {
                const float4 f = q2f(rp[q]);
                bsum.x += f.x; bsum.y += f.y; bsum.z += f.z; bsum.w += f.w;
            }
            *reinterpret_cast<half4_t*>(&Ps[(prow0 + 16 * q) * PP + pc]) = q2h(rp[q]);
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            if (e < H_E) *reinterpret_cast<half4_t*>(&Hs[(e / (BN / 4)) * PQ + (e % (BN / 4)) * 4]) = q2h(rh[q]);
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // transposed-read lane address (wgrad_f16_kernel): half lh takes k rows 8lh..8lh+7 of a 16-k step
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    floatx16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int kb0 = split * a.chunks_per_split;
    const int ke0 = min(a.nchunks, kb0 + a.chunks_per_split);
    const int share = (max(ke0 - kb0, 0) + G - 1) / G;
    const int kb = min(ke0, kb0 + gq * share), ke = min(ke0, kb + share);
    if (kb < ke) {
        load(kb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < share; ++it) {
        const int kc = kb + it;
        const bool next = kc + 1 < ke;
        if (next) load(kc + 1);  // next chunk in flight during this chunk's NT x 2 MFMAs per wave
        const _Float16* Ps = smem + cur * (PSZ + HSZ);
        const _Float16* Hs = Ps + PSZ;
#pragma unroll
        for (int s = 0; s < KT / 16; ++s) {
            if (kc >= ke) break;  // this group idles through the split's last step
            const _Float16* pa = Ps + (16 * s + tr_row) * PP + wm * 32 + tr_col;
            const halfx4_t alo = lds_tr4(pa), ahi = lds_tr4(pa + 4 * PP);
            const halfx8_t af = __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7);
            static_for<NT>([&](auto J) {
                constexpr int t = decltype(J)::value;
                constexpr int hr = t / KW, hc = t % KW;
                const _Float16* pb = Hs + (hr * HC + DIL * hc + SQ * (16 * s + tr_row)) * PQ + wn * 32 + tr_col;
                const halfx4_t blo = lds_tr4(pb), bhi = lds_tr4(pb + 4 * SQ * PQ);
                const halfx8_t bf = __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[t], 0, 0, 0);
            });
        }
        if (next) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem_all);  // the loop ended with a barrier
        red[threadIdx.x] = bsum;
        __syncthreads();
        if (threadIdx.x < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < 256 * G / (BM / 4); ++r) {
                const float4 v = red[threadIdx.x + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
        __syncthreads();
    }
    if constexpr (G > 1) {
        combine_groups<NT, G, G * (PSZ + HSZ)>(acc, reinterpret_cast<float*>(smem_all), tid, gq);
        if (gq != 0) return;
    }
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int n = n0 + wn * 32 + lr;
        if (n < d.N) {
            float* out = a.slab + ((long long)split * d.ntaps + t0 + j) * MN + n;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N] = acc[j][r];
            }
        }
    });
}

// ------------------------------------------------------------------------------------------------
// fp32 1x1 weight gradient on the bf16 MFMA ("bf16x6", the default fp32 GEMM): wgrad1x1_kernel's chunking (32-pixel
// chunks, P and Q rows of the same pixels as contiguous float4 rows, double-buffered, one barrier per chunk) with
// the staged tiles split into three bf16 planes in the transposed [pixel][channel] layout of wgrad_f16_kernel (pitch
// B + 32 halves, ds_read_b64_tr_b16) and bf6_mfma products: 2 x 6 v_mfma_f32_32x32x16_bf16 per tile and chunk
// against 16 v_mfma_f32_32x32x2_f32, at an intensity (~21 FLOP/B at 128^2 64 <-> 128) where the fp32 MFMA and HBM
// cost about the same. Bias gradient = fp32 column sums of the unsplit P from the staging registers.
// ------------------------------------------------------------------------------------------------
template <int TM, int TN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(256) void wgrad1x1_bf6_kernel(const WgradArgs a) {
    constexpr int BM = 32 * TM * WAVES_M, BN = 32 * TN * WAVES_N;
    constexpr int PP = BM + 32, PQ = BN + 32;  // bf16 row pitches
    constexpr int PSZ = KT * PP, QSZ = KT * PQ, PLANE = PSZ + QSZ, BUF = 3 * PLANE;
    constexpr int P_V = KT * BM / 4 / 256, Q_V = KT * BN / 4 / 256;
    static_assert(P_V >= 1 && Q_V >= 1, "tile too small");
    static_assert(PLANE % 4 == 0 && 2 * BUF * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int split = rr;
    const int m0 = mt * BM, n0 = nt * BN;
    const long long Qtot = (long long)d.B * d.Hq * d.Wq;
    // fixed per-thread channel quads (256 % (B / 4) == 0): rows tid / (B / 4) + i * 256 / (B / 4)
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);
    const int qc = (tid % (BN / 4)) * 4, qrow0 = tid / (BN / 4);
    constexpr int PRS = 256 / (BM / 4), QRS = 256 / (BN / 4);
    float4 rp[P_V], rq[Q_V];
    auto load = [&](int kc) {
        const long long k0 = (long long)kc * KT;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            const long long row = k0 + prow0 + i * PRS;
            rp[i] = (row < Qtot && m0 + pc < d.M) ? ld4(a.p + row * d.ldp + m0 + pc) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const long long row = k0 + qrow0 + i * QRS;
            rq[i] = (row < Qtot && n0 + qc < d.N) ? ld4(a.q + row * d.ldq + n0 + qc) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto put = [&](__bf16* base, int o, const float4& v) {
        bf16x4_t h, m, l;
        bf6_split4(v, h, m, l);
        *reinterpret_cast<bf16x4_t*>(&base[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&base[PLANE + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&base[2 * PLANE + o]) = l;
    };
    auto store = [&](int buf) {
        __bf16* B0 = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            if (do_bias) { bsum.x += rp[i].x; bsum.y += rp[i].y; bsum.z += rp[i].z; bsum.w += rp[i].w; }
            put(B0, (prow0 + i * PRS) * PP + pc, rp[i]);
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) put(B0, PSZ + (qrow0 + i * QRS) * PQ + qc, rq[i]);
    };
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    auto frag = [&](const __bf16* p, int pitch) {
        const halfx4_t lo = lds_tr4(reinterpret_cast<const _Float16*>(p));
        const halfx4_t hi = lds_tr4(reinterpret_cast<const _Float16*>(p + 4 * pitch));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int kb = split * a.chunks_per_split;
    const int ke = min(a.nchunks, kb + a.chunks_per_split);
    if (kb < ke) {
        load(kb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kc = kb; kc < ke; ++kc) {
        const bool next = kc + 1 < ke;
        if (next) load(kc + 1);  // in flight during this chunk's MFMAs
        const __bf16* Ps = smem + cur * BUF;
        const __bf16* Qs = Ps + PSZ;
#pragma unroll
        for (int s = 0; s < KT / 16; ++s) {
            bf16x8_t af[TM][3], bf[TN][3];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    af[tm][pl] = frag(Ps + pl * PLANE + (16 * s + tr_row) * PP + wm * TM * 32 + tm * 32 + tr_col, PP);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    bf[tn][pl] = frag(Qs + pl * PLANE + (16 * s + tr_row) * PQ + wn * TN * 32 + tn * 32 + tr_col, PQ);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = bf6_mfma(af[tm], bf[tn], acc[tm][tn]);
        }
        if (next) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem);  // the loop ended with a barrier
        red[tid] = bsum;
        __syncthreads();
        if (tid < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < PRS; ++r) {
                const float4 v = red[tid + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
    }
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    float* out = a.slab + (long long)split * MN;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * TN * 32 + tn * 32 + lr;
            if (n >= d.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N + n] = acc[tm][tn][r];
            }
        }
}

// ------------------------------------------------------------------------------------------------
// wgrad1x1_bf6_kernel with its operand loads two chunks ahead (hyres_conv_tuning key 15 = 2). The 1x1 weight
// gradient streams P and Q once (~3 TB/s at one 98 KB block per CU: 24.6 KB of loads in flight per CU, one HBM latency
// per 32-pixel chunk). Here two register sets alternate: chunk k + 2's loads are issued while chunk k's MFMAs run and
// chunk k + 1's registers go to LDS, so two chunks are in flight. Every load is an unconditional raw buffer load
// (out-of-range rows / channels / chunks past the split: an offset past the buffer's end, which returns 0 without
// touching memory): no branch around a load, so the compiler's vmcnt waits count only the older set. Same products in
// the same order as wgrad1x1_bf6_kernel (bit-identical slabs).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wg_rsrc(const void* p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)std::min<long long>(bytes, 0x7FFFFFF0LL),
                                             0x00020000);
}
template <int TM, int TN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(256) void wgrad1x1_bf6_pf2_kernel(const WgradArgs a) {
    constexpr int BM = 32 * TM * WAVES_M, BN = 32 * TN * WAVES_N;
    constexpr int PP = BM + 32, PQ = BN + 32;  // bf16 row pitches
    constexpr int PSZ = KT * PP, QSZ = KT * PQ, PLANE = PSZ + QSZ, BUF = 3 * PLANE;
    constexpr int P_V = KT * BM / 4 / 256, Q_V = KT * BN / 4 / 256;
    static_assert(P_V >= 1 && Q_V >= 1, "tile too small");
    static_assert(PLANE % 4 == 0 && 2 * BUF * 2 <= 160 * 1024, "LDS");
    constexpr int OOR = (int)0x80000000;
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int split = rr;
    const int m0 = mt * BM, n0 = nt * BN;
    const long long Qtot = (long long)d.B * d.Hq * d.Wq;
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);
    const int qc = (tid % (BN / 4)) * 4, qrow0 = tid / (BN / 4);
    constexpr int PRS = 256 / (BM / 4), QRS = 256 / (BN / 4);
    const __amdgpu_buffer_rsrc_t rp_ = wg_rsrc(a.p, Qtot * d.ldp * 4);
    const __amdgpu_buffer_rsrc_t rq_ = wg_rsrc(a.q, Qtot * d.ldq * 4);
    const bool pc_ok = m0 + pc < d.M, qc_ok = n0 + qc < d.N;
    const int kb = split * a.chunks_per_split;
    const int ke = min(a.nchunks, kb + a.chunks_per_split);
    auto load = [&](int kc, float4 (&rp)[P_V], float4 (&rq)[Q_V]) {
        const long long k0 = (long long)kc * KT;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            const long long row = k0 + prow0 + i * PRS;
            const int off = (kc < ke && row < Qtot && pc_ok) ? (int)((row * d.ldp + m0 + pc) * 4) : OOR;
            rp[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp_, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) {
            const long long row = k0 + qrow0 + i * QRS;
            const int off = (kc < ke && row < Qtot && qc_ok) ? (int)((row * d.ldq + n0 + qc) * 4) : OOR;
            rq[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rq_, off, 0, 0));
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto put = [&](__bf16* base, int o, const float4& v) {
        bf16x4_t h, m, l;
        bf6_split4(v, h, m, l);
        *reinterpret_cast<bf16x4_t*>(&base[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&base[PLANE + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&base[2 * PLANE + o]) = l;
    };
    auto store = [&](int buf, const float4 (&rp)[P_V], const float4 (&rq)[Q_V]) {
        __bf16* B0 = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < P_V; ++i) {
            if (do_bias) { bsum.x += rp[i].x; bsum.y += rp[i].y; bsum.z += rp[i].z; bsum.w += rp[i].w; }
            put(B0, (prow0 + i * PRS) * PP + pc, rp[i]);
        }
#pragma unroll
        for (int i = 0; i < Q_V; ++i) put(B0, PSZ + (qrow0 + i * QRS) * PQ + qc, rq[i]);
    };
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    auto frag = [&](const __bf16* p, int pitch) {
        const halfx4_t lo = lds_tr4(reinterpret_cast<const _Float16*>(p));
        const halfx4_t hi = lds_tr4(reinterpret_cast<const _Float16*>(p + 4 * pitch));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float4 pA[P_V], qA[Q_V], pB[P_V], qB[Q_V];
    if (kb < ke) {  // block-uniform
        load(kb, pA, qA);
        load(kb + 1, pB, qB);
        store(0, pA, qA);
    }
    __syncthreads();
    // chunk kc sits in LDS buffer ``cur``; ``hn`` holds chunk kc + 1 (in flight), ``hl`` (stored) receives kc + 2
    auto body = [&](int kc, int cur, float4 (&pl)[P_V], float4 (&ql)[Q_V], const float4 (&pn)[P_V],
                    const float4 (&qn)[Q_V]) {
        load(kc + 2, pl, ql);
        const __bf16* Ps = smem + cur * BUF;
        const __bf16* Qs = Ps + PSZ;
#pragma unroll
        for (int s = 0; s < KT / 16; ++s) {
            bf16x8_t af[TM][3], bf[TN][3];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int pl3 = 0; pl3 < 3; ++pl3)
                    af[tm][pl3] = frag(Ps + pl3 * PLANE + (16 * s + tr_row) * PP + wm * TM * 32 + tm * 32 + tr_col, PP);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int pl3 = 0; pl3 < 3; ++pl3)
                    bf[tn][pl3] = frag(Qs + pl3 * PLANE + (16 * s + tr_row) * PQ + wn * TN * 32 + tn * 32 + tr_col, PQ);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = bf6_mfma(af[tm], bf[tn], acc[tm][tn]);
        }
        if (kc + 1 < ke) store(cur ^ 1, pn, qn);  // block-uniform
        __syncthreads();
    };
    for (int kc = kb; kc < ke; kc += 2) {
        body(kc, 0, pA, qA, pB, qB);
        if (kc + 1 < ke) body(kc + 1, 1, pB, qB, pA, qA);
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem);  // the loop ended with a barrier
        red[tid] = bsum;
        __syncthreads();
        if (tid < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < PRS; ++r) {
                const float4 v = red[tid + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
    }
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    float* out = a.slab + (long long)split * MN;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * TN * 32 + tn * 32 + lr;
            if (n >= d.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N + n] = acc[tm][tn][r];
            }
        }
}

// ------------------------------------------------------------------------------------------------
// fp32 halo-staged weight gradient on the bf16 MFMA ("bf16x6", hyres_conv_tuning key 7 = 1, the default fp32 GEMM):
// wgrad_halo_f16_kernel's schedule and transposed LDS images, with each fp32 operand split when staged into three
// bf16 planes (x = x0 + x1 + x2, 24 significant bits) and every product formed from the six cross products with
// i + j <= 2 in fp32 accumulation (bf6_mfma: per product ~2^-25 relative, below the fp32 MFMA's own rounding).
// Per 32-pixel chunk a wave issues NT x 2 x 6 v_mfma_f32_32x32x16_bf16 (32 cycles each) against NT x 16
// v_mfma_f32_32x32x2_f32 (64 cycles each) in wgrad_halo_kernel: 2.67x fewer MFMA cycles. LDS: 2 buffers x 3 planes
// x (P chunk + Q halo) <= 158 KB, one 4-wave block per CU. Bias gradient = fp32 column sums of the unsplit P.
// ------------------------------------------------------------------------------------------------
template <int KR, int KW, int SQ, int DIL = 1>
__global__ __launch_bounds__(256, 1) void wgrad_halo_bf6_kernel(const WgradArgs a, int dhg, int dwg) {
    constexpr int BM = 64, BN = 64, NT = KR * KW, HC = 31 * SQ + DIL * (KW - 1) + 1;
    constexpr int PP = BM + 32, PQ = BN + 32;  // bf16 row pitches (the transposed reads' conflict-free pitch)
    constexpr int PSZ = KT * PP, HSZ = KR * HC * PQ, PLANE = PSZ + HSZ, BUF = 3 * PLANE;
    constexpr int P_V = KT * BM / 4 / 256;
    constexpr int H_E = KR * HC * (BN / 4);
    constexpr int H_V = (H_E + 255) / 256;
    static_assert(PLANE % 4 == 0, "8-byte aligned planes for the transposed reads");
    static_assert(2 * BUF * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int dh0 = dhg + grp * KR * DIL;
    const int cpr = d.Wq / 32;
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);  // this thread's fixed P channel quad
    float4 rp[P_V], rh[H_V];
    auto load = [&](int kc) {
        const int b = kc / (d.Hq * cpr);
        const int rem = kc - b * d.Hq * cpr;
        const int i = rem / cpr;
        const int j0 = (rem - i * cpr) * 32;
        const long long q0 = (long long)kc * 32;
#pragma unroll
        for (int q = 0; q < P_V; ++q)
            rp[q] = m0 + pc < d.M ? ld4(a.p + (q0 + prow0 + 16 * q) * d.ldp + m0 + pc) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            const int pix = e / (BN / 4), c = (e % (BN / 4)) * 4;
            const int hr = pix / HC, hc = pix - (pix / HC) * HC;
            const int ih = i * SQ + dh0 + DIL * hr, iw = j0 * SQ + dwg + hc;
            const bool ok = e < H_E && (unsigned)ih < (unsigned)d.Hqq && (unsigned)iw < (unsigned)d.Wqq && n0 + c < d.N;
            rh[q] = ok ? ld4(a.q + ((long long)(b * d.Hqq + ih) * d.Wqq + iw) * d.ldq + n0 + c)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto put = [&](__bf16* base, int o, const float4& v) {
        bf16x4_t h, m, l;
        bf6_split4(v, h, m, l);
        *reinterpret_cast<bf16x4_t*>(&base[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&base[PLANE + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&base[2 * PLANE + o]) = l;
    };
    auto store = [&](int buf) {
        __bf16* B0 = smem + buf * BUF;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            if (do_bias) { bsum.x += rp[q].x; bsum.y += rp[q].y; bsum.z += rp[q].z; bsum.w += rp[q].w; }
            put(B0, (prow0 + 16 * q) * PP + pc, rp[q]);
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            if (e < H_E) put(B0, PSZ + (e / (BN / 4)) * PQ + (e % (BN / 4)) * 4, rh[q]);
        }
    };

    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // transposed-read lane address (wgrad_f16_kernel): half lh takes k rows 8lh..8lh+7 of a 16-k step
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    auto frag = [&](const __bf16* p, int pitch) {  // 8 consecutive k of one row / column, transposed read
        const halfx4_t lo = lds_tr4(reinterpret_cast<const _Float16*>(p));
        const halfx4_t hi = lds_tr4(reinterpret_cast<const _Float16*>(p + 4 * pitch));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    floatx16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int kb = split * a.chunks_per_split;
    const int ke = min(a.nchunks, kb + a.chunks_per_split);
    if (kb < ke) {
        load(kb);
        store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int kc = kb; kc < ke; ++kc) {
        const bool next = kc + 1 < ke;
        if (next) load(kc + 1);  // next chunk in flight during this chunk's NT x 12 MFMAs per wave
        const __bf16* Ps = smem + cur * BUF;
        const __bf16* Hs = Ps + PSZ;
#pragma unroll
        for (int s = 0; s < KT / 16; ++s) {
            bf16x8_t af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) af[pl] = frag(Ps + pl * PLANE + (16 * s + tr_row) * PP + wm * 32 + tr_col, PP);
            static_for<NT>([&](auto J) {
                constexpr int t = decltype(J)::value;
                constexpr int hr = t / KW, hc = t % KW;
                const int ob = (hr * HC + DIL * hc + SQ * (16 * s + tr_row)) * PQ + wn * 32 + tr_col;
                bf16x8_t bf[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) bf[pl] = frag(Hs + pl * PLANE + ob, SQ * PQ);
                acc[t] = bf6_mfma(af, bf, acc[t]);
            });
        }
        if (next) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem);  // the loop ended with a barrier
        red[tid] = bsum;
        __syncthreads();
        if (tid < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < 256 / (BM / 4); ++r) {
                const float4 v = red[tid + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
    }
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int n = n0 + wn * 32 + lr;
        if (n < d.N) {
            float* out = a.slab + ((long long)split * d.ntaps + t0 + j) * MN + n;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N] = acc[j][r];
            }
        }
    });
}

// ------------------------------------------------------------------------------------------------
// wgrad_halo_bf6_kernel (one kernel row of taps per block, KR = 1) with its operand loads two chunks ahead
// (hyres_conv_tuning key 16 = 2), as wgrad1x1_bf6_pf2_kernel: two register sets alternate, every load an
// unconditional raw buffer load (an offset past the buffer's end for the halo's out-of-image pixels, channels past N
// and chunks past the split: 0 without a memory access), so no branch sits around a load. Same products in the same
// order (bit-identical slabs).
// ------------------------------------------------------------------------------------------------
// MINB: blocks per CU the LDS allows (2 for the 3-tap rows and the stride-1 5-tap rows, 1 for the stride-2 5x5): the
// register bound keeps the compiler from spending the second block's VGPRs on the second register set
template <int KW, int SQ, int DIL = 1, int MINB = 2>
__global__ __launch_bounds__(256, MINB) void wgrad_halo_bf6_pf2_kernel(const WgradArgs a, int dhg, int dwg) {
    constexpr int KR = 1;
    constexpr int BM = 64, BN = 64, NT = KR * KW, HC = 31 * SQ + DIL * (KW - 1) + 1;
    constexpr int PP = BM + 32, PQ = BN + 32;
    constexpr int PSZ = KT * PP, HSZ = KR * HC * PQ, PLANE = PSZ + HSZ, BUF = 3 * PLANE;
    constexpr int P_V = KT * BM / 4 / 256;
    constexpr int H_E = KR * HC * (BN / 4);
    constexpr int H_V = (H_E + 255) / 256;
    constexpr int OOR = (int)0x80000000;
    static_assert(PLANE % 4 == 0, "8-byte aligned planes for the transposed reads");
    static_assert(2 * BUF * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x;
    const int bid = blockIdx.x;
    const int lb = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);  // XCD-aware order, as wgrad_kernel
    if (lb >= a.nblocks) return;
    int rr = lb;
    const int mt = rr % a.mtiles; rr /= a.mtiles;
    const int nt = rr % a.ntiles; rr /= a.ntiles;
    const int grp = rr % a.ngroups;
    const int split = rr / a.ngroups;
    const int m0 = mt * BM, n0 = nt * BN;
    const int t0 = grp * NT;
    const int dh0 = dhg + grp * KR * DIL;
    const int cpr = d.Wq / 32;
    const int pc = (tid % (BM / 4)) * 4, prow0 = tid / (BM / 4);
    const long long Qtot = (long long)d.B * d.Hq * d.Wq;
    const __amdgpu_buffer_rsrc_t rp_ = wg_rsrc(a.p, Qtot * d.ldp * 4);
    const __amdgpu_buffer_rsrc_t rq_ = wg_rsrc(a.q, (long long)d.B * d.Hqq * d.Wqq * d.ldq * 4);
    const bool pc_ok = m0 + pc < d.M;
    const int kb = split * a.chunks_per_split;
    const int ke = min(a.nchunks, kb + a.chunks_per_split);
    auto load = [&](int kc, float4 (&rp)[P_V], float4 (&rh)[H_V]) {
        const bool live = kc < ke;
        const int kcc = live ? kc : kb;
        const int b = kcc / (d.Hq * cpr);
        const int rem = kcc - b * d.Hq * cpr;
        const int i = rem / cpr;
        const int j0 = (rem - i * cpr) * 32;
        const long long q0 = (long long)kcc * 32;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            const int off = (live && pc_ok) ? (int)(((q0 + prow0 + 16 * q) * d.ldp + m0 + pc) * 4) : OOR;
            rp[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rp_, off, 0, 0));
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            const int pix = e / (BN / 4), c = (e % (BN / 4)) * 4;
            const int hr = pix / HC, hc = pix - (pix / HC) * HC;
            const int ih = i * SQ + dh0 + DIL * hr, iw = j0 * SQ + dwg + hc;
            const bool ok = live && e < H_E && (unsigned)ih < (unsigned)d.Hqq && (unsigned)iw < (unsigned)d.Wqq &&
                            n0 + c < d.N;
            const int off = ok ? (int)(((((long long)b * d.Hqq + ih) * d.Wqq + iw) * d.ldq + n0 + c) * 4) : OOR;
            rh[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rq_, off, 0, 0));
        }
    };
    const bool do_bias = a.bias_slab != nullptr && nt == 0 && grp == 0;
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);
    auto put = [&](__bf16* base, int o, const float4& v) {
        bf16x4_t h, m, l;
        bf6_split4(v, h, m, l);
        *reinterpret_cast<bf16x4_t*>(&base[o]) = h;
        *reinterpret_cast<bf16x4_t*>(&base[PLANE + o]) = m;
        *reinterpret_cast<bf16x4_t*>(&base[2 * PLANE + o]) = l;
    };
    auto store = [&](int buf, const float4 (&rp)[P_V], const float4 (&rh)[H_V]) {
        __bf16* B0 = smem + buf * BUF;
#pragma unroll
        for (int q = 0; q < P_V; ++q) {
            if (do_bias) { bsum.x += rp[q].x; bsum.y += rp[q].y; bsum.z += rp[q].z; bsum.w += rp[q].w; }
            put(B0, (prow0 + 16 * q) * PP + pc, rp[q]);
        }
#pragma unroll
        for (int q = 0; q < H_V; ++q) {
            const int e = tid + 256 * q;
            if (e < H_E) put(B0, PSZ + (e / (BN / 4)) * PQ + (e % (BN / 4)) * 4, rh[q]);
        }
    };
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane >> 2) & 3, lp = lane & 3;
    const int tr_row = 8 * lh + lq, tr_col = 16 * lg + 4 * lp;
    auto frag = [&](const __bf16* p, int pitch) {
        const halfx4_t lo = lds_tr4(reinterpret_cast<const _Float16*>(p));
        const halfx4_t hi = lds_tr4(reinterpret_cast<const _Float16*>(p + 4 * pitch));
        return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    floatx16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float4 pA[P_V], hA[H_V], pB[P_V], hB[H_V];
    if (kb < ke) {  // block-uniform
        load(kb, pA, hA);
        load(kb + 1, pB, hB);
        store(0, pA, hA);
    }
    __syncthreads();
    auto body = [&](int kc, int cur, float4 (&pl)[P_V], float4 (&hl)[H_V], const float4 (&pn)[P_V],
                    const float4 (&hn)[H_V]) {
        load(kc + 2, pl, hl);
        const __bf16* Ps = smem + cur * BUF;
        const __bf16* Hs = Ps + PSZ;
#pragma unroll
        for (int s = 0; s < KT / 16; ++s) {
            bf16x8_t af[3];
#pragma unroll
            for (int pl3 = 0; pl3 < 3; ++pl3)
                af[pl3] = frag(Ps + pl3 * PLANE + (16 * s + tr_row) * PP + wm * 32 + tr_col, PP);
            static_for<NT>([&](auto J) {
                constexpr int t = decltype(J)::value;
                constexpr int hr = t / KW, hc = t % KW;
                const int ob = (hr * HC + DIL * hc + SQ * (16 * s + tr_row)) * PQ + wn * 32 + tr_col;
                bf16x8_t bf[3];
#pragma unroll
                for (int pl3 = 0; pl3 < 3; ++pl3) bf[pl3] = frag(Hs + pl3 * PLANE + ob, SQ * PQ);
                acc[t] = bf6_mfma(af, bf, acc[t]);
            });
        }
        if (kc + 1 < ke) store(cur ^ 1, pn, hn);  // block-uniform
        __syncthreads();
    };
    for (int kc = kb; kc < ke; kc += 2) {
        body(kc, 0, pA, hA, pB, hB);
        if (kc + 1 < ke) body(kc + 1, 1, pB, hB, pA, hA);
    }
    if (do_bias) {  // block-uniform
        float4* red = reinterpret_cast<float4*>(smem);  // the loop ended with a barrier
        red[tid] = bsum;
        __syncthreads();
        if (tid < BM / 4) {
            float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < 256 / (BM / 4); ++r) {
                const float4 v = red[tid + r * (BM / 4)];
                s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
            }
            float* dst = a.bias_slab + (long long)split * d.M + m0 + 4 * tid;
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
            for (int c = 0; c < 4; ++c)
                if (m0 + 4 * tid + c < d.M) dst[c] = sv[c];
        }
    }
    const int lr = lane & 31;
    const long long MN = (long long)d.M * d.N;
    static_for<NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int n = n0 + wn * 32 + lr;
        if (n < d.N) {
            float* out = a.slab + ((long long)split * d.ntaps + t0 + j) * MN + n;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m < d.M) out[(long long)m * d.N] = acc[j][r];
            }
        }
    });
}

// ------------------------------------------------------------------------------------------------
// Thin-operand weight gradient: dW[t][m][n] = sum_q P[q][m] * Q[shift_t(q)][n] with N <= 4 (the 3-channel
// image side: refine conv 3->64 / 64->3 at 256^2 (the latter through the swapped descriptor), g_a's 5x5 s2
// conv 3->128, g_s's deconv 128->3) and M = 64*MW wide channels. An MFMA tile would be >90 % padding and
// the tap-folded MFMA path gathers Q with scalar loads (13-15 TF/s, ~1 TB/s, 240-280 us per layer); here
// the work is VALU FMAs at the HBM rate of P:
//   * a block owns ``rpb`` consecutive base-grid rows (b, i) and one group of TG taps (grid.y);
//   * per row, the Q rows the group's taps touch (<= THIN_ROWS rows x (Wq-1)*sq + tap span columns) are
//     staged once in LDS as float4 (n padded to 4), zero outside the image;
//   * wave w walks pixels j = w, w+4, ...: lane l holds P[q][l + 64*mw] (coalesced rows, the next pixel's
//     row prefetched before this pixel's FMAs), the tap's Q values are one broadcast ds_read_b128;
//   * per-lane accumulators [MW][TG][NC] (+ the P column sums = the bias gradient) are reduced over the
//     block's 4 waves through LDS into the split slab [block][t][m][n]; the deterministic slab reduce of
//     the generic path finishes it.
// ------------------------------------------------------------------------------------------------
constexpr int THIN_ROWS = 5, THIN_SPAN = 264;  // staged window: rows x columns (host check: ncol <= SPAN)
constexpr int THIN_COLS = THIN_SPAN;
constexpr int THIN_STAGE = (THIN_ROWS * THIN_COLS + 255) / 256;  // staged window entries per thread

template <int MW, int NC, int TG, int SQ, bool PH = false>  // PH: P (the wide operand) fp16 in HBM
__global__ __launch_bounds__(256) void wgrad_thin_kernel(const WgradArgs a, int rpb, int dhmin, int dwmin, int nrow,
                                                         int ncol, int win) {
    constexpr int PCH = 64 / MW;            // pixels per P chunk (PCH x 64*MW floats = 16 KB)
    constexpr int PV = PCH * 16 * MW / 256;  // float4 per thread per chunk
    constexpr int PPW = PCH / 4;             // pixels per wave per chunk
    __shared__ __attribute__((aligned(16))) float Qs[THIN_ROWS * THIN_COLS * 4];
    __shared__ __attribute__((aligned(16))) float Ps[PCH * 64 * MW];
    const hyres_wgrad_desc& d = a.d;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int blk = blockIdx.x, grp = blockIdx.y;
    const int t0 = grp * TG;
    const int ntg = min(TG, d.ntaps - t0);
    const int R = d.B * d.Hq;
    const int r0 = blk * rpb, r1 = min(R, r0 + rpb);
    const bool do_bias = a.bias_slab != nullptr && grp == 0;
    const int nst = nrow * THIN_COLS;
    // per-tap window offsets through LDS (an indexed read of the by-value descriptor's tap arrays would
    // copy them to scratch); taps past ntg read any slot: their accumulators are never stored
    __shared__ int toff_s[TG];
    if (tid < TG)
        toff_s[tid] = tid < ntg ? ((d.dh[t0 + tid] - dhmin) * THIN_COLS + (d.dw[t0 + tid] - dwmin)) * 4 : 0;
    __syncthreads();
    int toff[TG];
#pragma unroll
    for (int u = 0; u < TG; ++u) toff[u] = toff_s[u];
    // accumulators as float4 (thin channels in .xyzw): an array of MW*TG vectors stays in registers where
    // a [MW][TG][4] float array (> 32 elements) is demoted to scratch
    float4 acc[MW][TG];
    float bsum[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) {
        bsum[w] = 0.f;
#pragma unroll
        for (int u = 0; u < TG; ++u) acc[w][u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    quad_t<PH> pr4[PV];  // fp16 P: raw halves, converted at the LDS store
    for (int r = r0; r < r1; ++r) {
        const int b = r / d.Hq, i = r - (r / d.Hq) * d.Hq;
        const long long prow = (long long)r * d.Wq * d.ldp;  // element offset of this row's first pixel
        auto load_chunk = [&](int c0) {
#pragma unroll
            for (int k = 0; k < PV; ++k) {
                const int idx = tid + 256 * k;
                const int px = idx / (16 * MW), c4 = idx - (idx / (16 * MW)) * (16 * MW);
                pr4[k] = c0 + px < d.Wq ? ldq4<PH>(a.p, prow + (long long)(c0 + px) * d.ldp + 4 * c4) : zq4<PH>();
            }
        };
        load_chunk(0);
        __syncthreads();  // the previous row's readers of Qs / Ps are done
        // this row's Q window (zero outside the image, past N channels and past column ncol): every load of
        // the window is issued before the first LDS store (a rolled loop serialised one latency per entry)
        {
            float4 qv[THIN_STAGE];
#pragma unroll
            for (int k = 0; k < THIN_STAGE; ++k) {
                const int idx = tid + 256 * k;
                const int rr = idx / THIN_COLS, cc = idx - (idx / THIN_COLS) * THIN_COLS;
                const int ih = i * SQ + dhmin + rr, iw = dwmin + cc;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (idx < nst && cc < ncol && (unsigned)ih < (unsigned)d.Hqq && (unsigned)iw < (unsigned)d.Wqq) {
                    const float* qp = a.q + ((long long)(b * d.Hqq + ih) * d.Wqq + iw) * d.ldq;
                    v.x = qp[0];
                    if (NC > 1 && d.N > 1) v.y = qp[1];
                    if (NC > 2 && d.N > 2) v.z = qp[2];
                    if (NC > 3 && d.N > 3) v.w = qp[3];
                }
                qv[k] = v;
            }
#pragma unroll
            for (int k = 0; k < THIN_STAGE; ++k)
                if (tid + 256 * k < nst) *reinterpret_cast<float4*>(&Qs[(tid + 256 * k) * 4]) = qv[k];
        }
        for (int c0 = 0; c0 < d.Wq; c0 += PCH) {
            if (c0) __syncthreads();  // the previous chunk's readers of Ps are done
#pragma unroll
            for (int k = 0; k < PV; ++k) *reinterpret_cast<float4*>(&Ps[4 * (tid + 256 * k)]) = q2f(pr4[k]);
            __syncthreads();
            if (c0 + PCH < d.Wq) load_chunk(c0 + PCH);  // next chunk in flight during this chunk's FMAs
            if constexpr (MW == 1 && TG == 9 && SQ == 1) {
                // win = 1: one group of the 3x3 taps in row-major order, 2: the same reversed (the swapped descriptor of
                // the 64 -> 3 convs: dh, dw negated); host-checked, Wq <= 256
                auto window = [&](auto REVC) {
                    constexpr bool REV = decltype(REVC)::value;
                    // round 6: the 3 x 3 Q window of the wave's current pixel in registers, sliding one column per
                    // pixel (3 LDS reads per pixel instead of 9: the per-tap broadcast reads and their waits were the
                    // limit, profiles/r6y_pmc_families.txt); logical column c of pixel uu sits in slot (c + uu) % 3.
                    // Same FMAs per accumulator in the same pixel order: bit-identical
                    const int jb = c0 + wave * PPW;
                    float4 qw[3][3];
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            qw[r][c] = *reinterpret_cast<const float4*>(Qs + (r * THIN_COLS + jb + c) * 4);
#pragma unroll
                    for (int uu = 0; uu < PPW; ++uu) {
                        if (jb + uu < d.Wq) {  // wave-uniform
                            const float pv = Ps[(wave * PPW + uu) * 64 + lane];
#pragma unroll
                            for (int r = 0; r < 3; ++r)
#pragma unroll
                                for (int c = 0; c < 3; ++c) {
                                    const float4 q = qw[r][(c + uu) % 3];
                                    float4& A = acc[0][REV ? 8 - (r * 3 + c) : r * 3 + c];
                                    A.x = fmaf(pv, q.x, A.x);
                                    if (NC > 1) A.y = fmaf(pv, q.y, A.y);
                                    if (NC > 2) A.z = fmaf(pv, q.z, A.z);
                                    if (NC > 3) A.w = fmaf(pv, q.w, A.w);
                                }
                            bsum[0] += pv;
                        }
                        if (uu + 1 < PPW) {
#pragma unroll
                            for (int r = 0; r < 3; ++r)
                                qw[r][uu % 3] = *reinterpret_cast<const float4*>(Qs + (r * THIN_COLS + jb + uu + 3) * 4);
                        }
                    }
                };
                if (win == 1) {  // block-uniform
                    window(std::false_type{});
                    continue;
                }
                if (win == 2) {
                    window(std::true_type{});
                    continue;
                }
            }
#pragma unroll 2
            for (int uu = 0; uu < PPW; ++uu) {
                const int pl = wave * PPW + uu;
                const int j = c0 + pl;
                if (j >= d.Wq) break;  // wave-uniform
                float pv[MW];
#pragma unroll
                for (int w = 0; w < MW; ++w) pv[w] = Ps[pl * 64 * MW + 64 * w + lane];
                const float* qg = Qs + j * SQ * 4;
#pragma unroll
                for (int v = 0; v < TG; ++v) {
                    const float4 q = *reinterpret_cast<const float4*>(qg + toff[v]);
#pragma unroll
                    for (int w = 0; w < MW; ++w) {
                        acc[w][v].x = fmaf(pv[w], q.x, acc[w][v].x);
                        if (NC > 1) acc[w][v].y = fmaf(pv[w], q.y, acc[w][v].y);
                        if (NC > 2) acc[w][v].z = fmaf(pv[w], q.z, acc[w][v].z);
                        if (NC > 3) acc[w][v].w = fmaf(pv[w], q.w, acc[w][v].w);
                    }
                }
#pragma unroll
                for (int w = 0; w < MW; ++w) bsum[w] += pv[w];
            }
        }
    }
    float* red = Qs;
    // reduce the 4 waves' partials: one tap at a time through LDS ([wave][MW*NC][64]), wave 0 writes
    const long long MN = (long long)d.M * d.N;
    static_for<TG>([&](auto U) {  // compile-time tap index: acc stays in registers
        constexpr int u = decltype(U)::value;
        if (u < ntg) {
            __syncthreads();
#pragma unroll
            for (int w = 0; w < MW; ++w) {
                const float av[4] = {acc[w][u].x, acc[w][u].y, acc[w][u].z, acc[w][u].w};
#pragma unroll
                for (int n = 0; n < NC; ++n) red[(wave * MW * NC + w * NC + n) * 64 + lane] = av[n];
            }
            __syncthreads();
            if (wave == 0) {
                float* out = a.slab + ((long long)blk * d.ntaps + t0 + u) * MN;
#pragma unroll
                for (int w = 0; w < MW; ++w)
#pragma unroll
                    for (int n = 0; n < NC; ++n) {
                        if (n >= d.N) continue;
                        const int kk = (w * NC + n) * 64 + lane;
                        const float v = red[kk] + red[MW * NC * 64 + kk] + red[2 * MW * NC * 64 + kk] +
                                        red[3 * MW * NC * 64 + kk];
                        out[(long long)(lane + 64 * w) * d.N + n] = v;
                    }
            }
        }
    });
    if (do_bias) {
        __syncthreads();
#pragma unroll
        for (int w = 0; w < MW; ++w) red[(wave * MW + w) * 64 + lane] = bsum[w];
        __syncthreads();
        if (wave == 0)
#pragma unroll
            for (int w = 0; w < MW; ++w) {
                const int k = w * 64 + lane;
                a.bias_slab[(long long)blk * d.M + lane + 64 * w] =
                    red[k] + red[MW * 64 + k] + red[2 * MW * 64 + k] + red[3 * MW * 64 + k];
            }
    }
}

// deterministic split-K reduce: LX float4 lanes x (256 / LX) split groups per block (4*LX outputs per
// block). Few outputs with many splits (1x1 / small weights over a whole batch: nsplit up to 512) take
// LX = 4, so each thread walks nsplit/64 partial rows instead of nsplit/16 and 4x as many blocks run.
template <int LX>
__device__ __forceinline__ void wgrad_reduce_body(int blk, const float* slab, int nsplit, int ntaps, int M, int N,
                                                  float* dst, int sm, int sn, int st, int accumulate) {
    constexpr int G = 256 / LX, OUT = 4 * LX;
    __shared__ float red[G][OUT + 1];
    const long long total = (long long)ntaps * M * N;
    const int lx = threadIdx.x % LX, ly = threadIdx.x / LX;
    const long long base = (long long)blk * OUT + 4 * lx;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((total & 3) == 0) {
        if (base < total)
#pragma unroll 4
            for (int k = ly; k < nsplit; k += G) {
                const float4 v = ld4(slab + k * total + base);
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
    } else {
        for (int k = ly; k < nsplit; k += G) {
            const float* p = slab + k * total + base;
            if (base + 0 < total) s.x += p[0];
            if (base + 1 < total) s.y += p[1];
            if (base + 2 < total) s.z += p[2];
            if (base + 3 < total) s.w += p[3];
        }
    }
    red[ly][4 * lx + 0] = s.x;
    red[ly][4 * lx + 1] = s.y;
    red[ly][4 * lx + 2] = s.z;
    red[ly][4 * lx + 3] = s.w;
    __syncthreads();
    if (threadIdx.x < OUT) {
        const long long idx = (long long)blk * OUT + threadIdx.x;
        if (idx < total) {
            float v = 0.f;
#pragma unroll 16
            for (int g = 0; g < G; ++g) v += red[g][threadIdx.x];
            const int n = (int)(idx % N);
            const long long r = idx / N;
            const int m = (int)(r % M);
            const int t = (int)(r / M);
            float* p = dst + (long long)m * sm + (long long)n * sn + (long long)t * st;
            *p = accumulate ? (*p + v) : v;
        }
    }
}

template <int LX>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* slab, int nsplit, int ntaps, int M, int N,
                                                           float* dst, int sm, int sn, int st, int accumulate) {
    wgrad_reduce_body<LX>(blockIdx.x, slab, nsplit, ntaps, M, N, dst, sm, sn, st, accumulate);
}

// weight-gradient slab reduce and the bias-gradient partials ([nsplit][M]) in one launch
template <int LX>
__global__ __launch_bounds__(256) void wgrad_bias_reduce_kernel(const float* slab, int nsplit, int ntaps, int M, int N,
                                                                float* dst, int sm, int sn, int st, int accumulate,
                                                                int nb_w, const float* bslab, float* dbias) {
    if ((int)blockIdx.x < nb_w)
        wgrad_reduce_body<LX>(blockIdx.x, slab, nsplit, ntaps, M, N, dst, sm, sn, st, accumulate);
    else
        wgrad_reduce_body<LX>(blockIdx.x - nb_w, bslab, nsplit, 1, M, 1, dbias, 1, 0, 0, accumulate);
}

// Deferred reduces of a whole gradient segment in one launch (hyres_wgrad_reduce_jobs): the job table rides in
// the kernel arguments (captured by value in a HIP graph, no device table to keep alive); block b belongs to the
// first job whose block range ends past b. Each job runs the per-layer reduce body with the layer's own lane
// layout, so every output sums its partials in exactly the order wgrad_reduce_kernel does.
struct WgradJobBatch {
    hyres_wgrad_job j[HYRES_WGRAD_MAX_JOBS];
    int end[HYRES_WGRAD_MAX_JOBS];  // exclusive prefix sums of the jobs' block counts
    int n;
};

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(const WgradJobBatch b) {
    const int blk = blockIdx.x;
    int k = 0;
    while (k < b.n - 1 && blk >= b.end[k]) ++k;
    const int local = blk - (k ? b.end[k - 1] : 0);
    const hyres_wgrad_job& j = b.j[k];
    if (j.lanes == 16)
        wgrad_reduce_body<16>(local, j.slab, j.nsplit, j.ntaps, j.M, j.N, j.dst, j.sm, j.sn, j.st, j.accumulate);
    else if (j.lanes == 8)
        wgrad_reduce_body<8>(local, j.slab, j.nsplit, j.ntaps, j.M, j.N, j.dst, j.sm, j.sn, j.st, j.accumulate);
    else
        wgrad_reduce_body<4>(local, j.slab, j.nsplit, j.ntaps, j.M, j.N, j.dst, j.sm, j.sn, j.st, j.accumulate);
}

// lanes per block row for the reduce: keep ~>= 1024 blocks when the split count is large
static int reduce_lx(long long total, int nsplit) {
    if (nsplit <= 64 || (total + 63) / 64 >= 1024) return 16;
    if ((total + 31) / 32 >= 1024) return 8;
    return 4;
}

// Column sums of a [P][C] (pixel stride ld) matrix, deterministic two-pass.
// Pass 1: a block owns a row range; its 256 threads are laid out TR x TC over (rows, channel groups of
// VEC floats) so every wave reads whole contiguous rows; the TR partial rows are folded through LDS.
template <int VEC, bool H = false>  // H: x stored fp16 (AMP fp16 gradients), fp32 sums
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* x, int P, int C, int ld,
                                                             int rows_per_block, float* part) {
    __shared__ float red[256 * VEC];
    const int groups = C / VEC;                       // channel groups
    const int TC = groups < 256 ? groups : 256;        // threads across channels
    const int TR = 256 / TC;                           // threads across rows
    const int tc = threadIdx.x % TC, tr = threadIdx.x / TC;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(P, r0 + rows_per_block);
    for (int g0 = 0; g0 < groups; g0 += TC) {
        const int gi = g0 + tc;
        float acc[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
        if (tr < TR && gi < groups) {
            for (int r = r0 + tr; r < r1; r += TR) {
                const long long o = (long long)r * ld + gi * VEC;
                if constexpr (VEC == 4) {
                    float4 q = ldv4<H>(x, o);
                    acc[0] += q.x; acc[1] += q.y; acc[2] += q.z; acc[3] += q.w;
                } else {
                    acc[0] += ldv<H>(x, o);
                }
            }
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) red[threadIdx.x * VEC + v] = acc[v];
        __syncthreads();
        if (tr == 0 && gi < groups) {
            for (int k = 1; k < TR; ++k)
#pragma unroll
                for (int v = 0; v < VEC; ++v) acc[v] += red[(k * TC + tc) * VEC + v];
#pragma unroll
            for (int v = 0; v < VEC; ++v) part[(long long)blockIdx.x * C + gi * VEC + v] = acc[v];
        }
        __syncthreads();
    }
}

}  // namespace hyres

using namespace hyres;

namespace hyres {


struct WgradPlan {
    int TMc, TNc, WMc, WNc, NT, BM, BN, mtiles, ntiles, ngroups, nchunks, nsplit, cps, tapn, nblocks;
    int halo, hk, hdh, hdw, hdil;  // wgrad_halo_kernel: K, first tap's (dh, dw), tap spacing
    int g1x1;                      // wgrad1x1_kernel: 4-wave groups per block
    int hg;                        // wgrad_halo(_f16)_kernel: 4-wave groups per block
};

// wgrad_halo_kernel applies: fp32, dense KxK taps (K = 3 or 5, dilation 1; K = 3 with dilation 2), Q stride
// 1 or 2 (5x5 only), base rows of a multiple of 32 pixels, both operands >= 32 channels on the float4 path.
// *dil = the tap spacing.
static bool halo_ok(const hyres_wgrad_desc* d, int* K, int* dil) {
    if (d->square_q || (d->sq != 1 && d->sq != 2)) return false;
    if (d->Wq % 32 != 0 || d->M < 32 || d->N < 32 || d->M % 4 || d->N % 4 || d->ldp % 4 || d->ldq % 4) return false;
    const int k = d->ntaps == 9 ? 3 : d->ntaps == 25 ? 5 : 0;
    if (!k || (d->sq == 2 && k != 5)) return false;  // stride 2 only for the 5x5 (de)convs (3x3 s2: 123 KB LDS)
    const int D = d->dw[1] - d->dw[0];
    if (D != 1 && !(D == 2 && k == 3 && d->sq == 1)) return false;
    for (int t = 0; t < d->ntaps; ++t)
        if (d->dh[t] != d->dh[0] + D * (t / k) || d->dw[t] != d->dw[0] + D * (t % k)) return false;
    *K = k;
    *dil = D;
    return true;
}

static bool wgrad_f16_ok(const hyres_wgrad_desc* d);

static WgradPlan wgrad_plan(const hyres_wgrad_desc* d) {
    WgradPlan p{};
    p.NT = 1;
    int hk = 0, hdil = 1;
    const bool halo = halo_ok(d, &hk, &hdil);  // fp32 or (AMP) f16 halo kernel: 32-pixel chunks either way
    const int kt = (wgrad_f16_ok(d) && !halo) ? KTH : KT;
    p.tapn = (d->N <= 16 && d->ntaps > 1 && !d->square_q) ? 1 : 0;
    const int ncols = p.tapn ? d->ntaps * d->N : d->N;
    if (p.tapn) {
        if (ncols <= 32) { p.TMc = 1; p.TNc = 1; p.WMc = 4; p.WNc = 1; }
        else { p.TMc = 1; p.TNc = 1; p.WMc = 2; p.WNc = 2; }
    } else if (d->M >= 128 && d->N >= 128) { p.TMc = 2; p.TNc = 2; p.WMc = 2; p.WNc = 2; }
    else if (d->M >= 128 && d->N >= 64 && d->ntaps == 1) { p.TMc = 2; p.TNc = 1; p.WMc = 2; p.WNc = 2; }
    else if (d->M <= 32) { p.TMc = 1; p.TNc = 1; p.WMc = 1; p.WNc = 4; }
    else if (d->N <= 32) { p.TMc = 1; p.TNc = 1; p.WMc = 4; p.WNc = 1; }
    else {
        p.TMc = 1; p.TNc = 1; p.WMc = 2; p.WNc = 2;
        // fp32: group 9 / 5 taps per block (operand reuse); f16: one tap per block column group (measured
        // faster on every f16 geometry of the step: the f16 main loop is short, more blocks hide it better)
        p.NT = (d->ntaps % 9 == 0) ? 9 : (d->ntaps % 5 == 0) ? 5 : 1;
        if (kt == KTH || g_tune[5] == 1) p.NT = 1;
    }
    p.BM = 32 * p.TMc * p.WMc; p.BN = 32 * p.TNc * p.WNc;
    p.mtiles = ceil_div(d->M, p.BM); p.ntiles = ceil_div(ncols, p.BN);
    p.ngroups = p.tapn ? 1 : ceil_div(d->ntaps, p.NT);
    p.nchunks = ceil_div((long long)d->B * d->Hq * d->Wq, kt);
    if (halo) {
        p.halo = 1;
        p.hk = hk;
        p.hdil = hdil;
        p.hdh = d->dh[0];
        p.hdw = d->dw[0];
        p.tapn = 0;
        p.TMc = p.TNc = 1; p.WMc = p.WNc = 2;
        p.BM = p.BN = 64;
        p.mtiles = ceil_div(d->M, 64); p.ntiles = ceil_div(d->N, 64);
        // 3x3: one kernel row of 3 taps per block, or all 9 taps per block (one 3-row halo per chunk) — rows of 3
        // give 3x the tiles, so a third of the pixel splits and of the split slab for the same grid. Default: rows
        // for dilation 1 (AMP step 21.56 -> 21.34 ms, fp32 42.82 -> 42.68 ms over 3 alternating repeats each;
        // 128^2 fp32 kernel 235 -> 208 us), all 9 taps for the dilated 3x3s (256^2: 678 vs 797 us fp32, 152 vs 219 us
        // f16: their halo rows are 2 apart, so a row group re-stages most of the chunk; profiles/r3r_rows_ab.txt,
        // r3y_rows_fp32_ab.txt)
        const int rows = hdil == 2 ? 3 : 1;
        p.NT = p.hk == 3 ? (rows == 1 ? 3 : 9) : 5;
        p.ngroups = d->ntaps / p.NT;
    }
    const long long tiles = (long long)p.mtiles * p.ntiles * p.ngroups;
    // ~2048 blocks (swept on MI355X: 1024 -> 2048 is -0.6 % step time; fewer splits hurt), >= 8 chunks
    // (256 pixels; f16: 4 chunks of 64) per split, <= 512 splits (hyres_conv_tuning keys 3, 4, 6 override them for
    // sweeps). Small grids (<= 16384 pixels, the 32^2 region at
    // bs 16): ~4096 blocks, fp32 multi-tap splits down to 4 chunks. The split count is capped so that the partial
    // slab stays <= 16 M floats (64 MB): for the wide 1x1 layers (M x N ~ 0.5 M) the slab write + reduce
    // otherwise costs more than the parallelism buys (scripts/tile_sweep.py --wgrad)
    const long long Q = (long long)d->B * d->Hq * d->Wq;
    const bool small = Q <= 16384;
    const int tb = g_tune[3] > 0 ? g_tune[3] : (small ? 4096 : 2048);
    const int mc0 = g_tune[4] > 0 ? g_tune[4] : ((small && kt == KT && d->ntaps > 1) ? 4 : 8);
    const int mc = std::max(1, mc0 * KT / kt);
    // <= 256 splits (<= 64 on the small grids): past that the split slab's write + reduce costs more than the
    // extra blocks buy — step 32.79 -> 32.54 ms, AMP 19.10 -> 18.76 ms against 512 everywhere (isolated, kernel +
    // reduce: 128^2 3x3 64->64 143 -> 137 us, 32^2 3x3 96->96 51.6 -> 43.4 us; one exception measured, 256^2 1x1
    // 64->64 132 -> 160 us, but 512 splits for the 1x1s only gave no step gain; profiles/r5z_wgrad_split_ab.txt)
    const int ms = g_tune[6] > 0 ? g_tune[6] : (small ? 64 : 256);
    const long long slab_cap = std::max<long long>(4, (16LL << 20) / ((long long)d->ntaps * d->M * d->N));
    const long long want = std::min<long long>(std::max<long long>(1, (tb + tiles - 1) / tiles), slab_cap);
    const long long maxsplit = std::max<long long>(1, p.nchunks / mc);
    p.nsplit = (int)std::min<long long>(std::min<long long>(want, maxsplit), ms);
    if (p.halo) {
        // whole rounds only: the halo kernel runs 2 blocks per CU (3 for 5x5 stride 1); a partial last round
        // of long split-K blocks costs as much as a full one, so drop it (e.g. 800 -> 500 blocks)
        // (the bf16x6 kernel: 1 block per CU when it stages all 9 taps' halo, 158 KB of LDS)
        const bool b6_9 = f32_gemm_bf6() && !wgrad_f16_ok(d) && p.NT == 9;
        const long long cap = 256LL * (b6_9 ? 1 : (p.hk == 5 && d->sq == 1) ? 3 : 2);
        if (tiles * p.nsplit > cap) p.nsplit = (int)std::max<long long>(1, (tiles * p.nsplit / cap) * cap / tiles);
        // and fill a partial single round when that grows the slab by <= 25 % (128^2 3x3: 455 -> 512)
        else if (cap / tiles <= maxsplit && 4 * (cap / tiles) <= 5LL * p.nsplit) p.nsplit = (int)(cap / tiles);
    }
    // 1x1 stride-1 fp32 gradients (wgrad1x1_kernel) outside the small grids: 2 groups of 4 waves per block share
    // one split's pixels, so the same waves write half the slab. Isolated 128^2 64<->128: 65 -> 62 us; on the 32^2
    // grids it lost (24.6 -> 30.5 us: half the blocks). (Two groups per block for the halo kernels — half their
    // split slab — won isolated but lost in the live step, 40.0 -> 41.1 ms: the 146 KB block keeps the concurrent
    // branches' blocks off its CU; profiles/r3o_halo_groups.txt. Removed in round 4.)
    p.hg = 1;
    p.g1x1 = 1;
    if (!small && !halo && kt == KT && !f32_gemm_bf6() && !p.tapn && !d->square_q && d->ntaps == 1 && d->dh[0] == 0 &&
        d->dw[0] == 0 && d->sq == 1 && d->Hqq == d->Hq && d->Wqq == d->Wq && p.ngroups == 1 && p.nsplit >= 2) {
        p.g1x1 = 2;
        p.nsplit = (p.nsplit + 1) / 2;
    }
    p.cps = ceil_div(p.nchunks, p.nsplit);
    p.nsplit = ceil_div(p.nchunks, p.cps);
    p.nblocks = (int)(tiles * p.nsplit);
    return p;
}

// f16 operands only on the vector path without tap folding (the 3-channel layers stay fp32)
static bool wgrad_f16_ok(const hyres_wgrad_desc* d) {
    const bool tapn = d->N <= 16 && d->ntaps > 1 && !d->square_q;
    return d->f16_operands && !tapn && d->M % 4 == 0 && d->N % 4 == 0 && d->ldp % 4 == 0 && d->ldq % 4 == 0 &&
           d->M >= 32 && d->N >= 32;
}

// Small-M stride-1 gradients are computed transposed with negated shifts so that the 3-channel
// operand becomes the (tap-folded) column side:  out[t][m][n] = sum_q' Q[q'][n] * P[q' - shift_t][m].
static bool wgrad_swap(const hyres_wgrad_desc* d) {
    return d->M <= 16 && d->N > 16 && d->ntaps > 1 && d->sq == 1 && d->Hqq == d->Hq && d->Wqq == d->Wq &&
           !d->square_q;
}

static hyres_wgrad_desc wgrad_swapped(const hyres_wgrad_desc* d) {
    hyres_wgrad_desc e = *d;
    e.M = d->N; e.ldp = d->ldq;
    e.N = d->M; e.ldq = d->ldp;
    for (int t = 0; t < d->ntaps; ++t) { e.dh[t] = -d->dh[t]; e.dw[t] = -d->dw[t]; }
    e.sm = d->sn; e.sn = d->sm;
    e.io_f16 = ((d->io_f16 & 1) << 1) | ((d->io_f16 >> 1) & 1);
    return e;
}

// fp16 operands (desc.io_f16) the chosen kernel reads natively: the f16 MFMA kernels either or both (AMP training:
// the saved activation and, with fp16 activation gradients, the gradient), the thin kernel a fp16 P; every other
// fp16 operand is converted into fp32 scratch before the launch (hyres_wgrad_workspace_bytes reserves it)
static int wgrad_native_io(const hyres_wgrad_desc* d, bool thin) {
    const int io = d->io_f16 & 3;
    if (!io) return 0;
    if (wgrad_f16_ok(d)) return io;
    if (thin) return io & 1;
    return 0;
}

static long long wgrad_cvt_floats(const hyres_wgrad_desc* d, int native) {
    const int cvt = (d->io_f16 & 3) & ~native;
    long long n = 0;
    if (cvt & 1) n += (long long)d->B * d->Hq * d->Wq * d->M + 8;  // + 16-byte alignment slack
    if (cvt & 2) n += (long long)d->B * d->Hqq * d->Wqq * d->N + 8;
    return n;
}

// fp16 [P][C] (pixel stride ld) -> contiguous fp32 [P][C]
__global__ void half_to_float_2d_kernel(const _Float16* src, int ld, float* dst, long long P, int C) {
    const long long n = P * C;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const long long p = i / C;
        dst[i] = (float)src[p * ld + (i - p * C)];
    }
}

// thin-operand weight-gradient plan (wgrad_thin_kernel): N <= 4, M in {64, 128}, the staged Q window fits
struct ThinPlan {
    int mw, nc, tg, ngroups, rpb, nblk, dhmin, dwmin, nrow, ncol, sq, win;
};

static bool thin_plan(const hyres_wgrad_desc* d, ThinPlan* tp) {
    if (d->N > 4 || (d->M != 64 && d->M != 128) || d->square_q || d->ntaps < 1 || d->ntaps > 25)
        return false;
    int hmin = 1 << 30, hmax = -(1 << 30), wmin = 1 << 30, wmax = -(1 << 30);
    for (int t = 0; t < d->ntaps; ++t) {
        hmin = std::min(hmin, d->dh[t]); hmax = std::max(hmax, d->dh[t]);
        wmin = std::min(wmin, d->dw[t]); wmax = std::max(wmax, d->dw[t]);
    }
    ThinPlan p{};
    p.dhmin = hmin; p.dwmin = wmin;
    p.nrow = hmax - hmin + 1;
    p.ncol = (d->Wq - 1) * d->sq + (wmax - wmin) + 1;
    if (p.nrow > THIN_ROWS || p.ncol > THIN_SPAN || (d->sq != 1 && d->sq != 2)) return false;
    if (d->ldp % 4 != 0) return false;  // P chunks staged as float4
    p.mw = d->M / 64;
    p.nc = d->N == 3 ? 3 : 4;
    p.sq = d->sq;
    p.tg = d->ntaps <= 9 ? 9 : (p.mw == 1 ? 25 : 13);
    p.ngroups = ceil_div(d->ntaps, p.tg);
    const int R = d->B * d->Hq;
    p.rpb = std::max(1, ceil_div(R * p.ngroups, 1024));  // ~1024 blocks (4 per CU)
    p.nblk = ceil_div(R, p.rpb);
    // the sliding-window loop (hyres_conv_tuning key 23, default 1): the 3x3 taps in row-major order, one group
    const bool w3 = g_tune[23] != 0 && p.mw == 1 && p.tg == 9 && p.sq == 1 && d->ntaps == 9 && d->Wq <= 256;
    bool fwd = w3, rev = w3;
    for (int t = 0; t < 9 && w3; ++t) {
        fwd = fwd && d->dh[t] == t / 3 - 1 && d->dw[t] == t % 3 - 1;
        rev = rev && d->dh[t] == 1 - t / 3 && d->dw[t] == 1 - t % 3;
    }
    p.win = fwd ? 1 : rev ? 2 : 0;
    *tp = p;
    return true;
}

static void launch_thin(const WgradArgs& a, const ThinPlan& p, bool ph, hipStream_t st) {
    const dim3 grid(p.nblk, p.ngroups);
    auto go = [&](auto mw, auto nc, auto tg) {
        constexpr int MW_ = decltype(mw)::value, NC_ = decltype(nc)::value, TG_ = decltype(tg)::value;
        if (p.sq == 1) {
            if (ph) hipLaunchKernelGGL((wgrad_thin_kernel<MW_, NC_, TG_, 1, true>), grid, dim3(256), 0, st, a, p.rpb,
                                       p.dhmin, p.dwmin, p.nrow, p.ncol, p.win);
            else hipLaunchKernelGGL((wgrad_thin_kernel<MW_, NC_, TG_, 1>), grid, dim3(256), 0, st, a, p.rpb, p.dhmin,
                                    p.dwmin, p.nrow, p.ncol, p.win);
        } else {
            if (ph) hipLaunchKernelGGL((wgrad_thin_kernel<MW_, NC_, TG_, 2, true>), grid, dim3(256), 0, st, a, p.rpb,
                                       p.dhmin, p.dwmin, p.nrow, p.ncol, p.win);
            else hipLaunchKernelGGL((wgrad_thin_kernel<MW_, NC_, TG_, 2>), grid, dim3(256), 0, st, a, p.rpb, p.dhmin,
                                    p.dwmin, p.nrow, p.ncol, p.win);
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I9 = std::integral_constant<int, 9>;
    using I13 = std::integral_constant<int, 13>;
    using I25 = std::integral_constant<int, 25>;
    if (p.mw == 1) {
        if (p.nc == 3) { if (p.tg == 9) go(I1{}, I3{}, I9{}); else go(I1{}, I3{}, I25{}); }
        else { if (p.tg == 9) go(I1{}, I4{}, I9{}); else go(I1{}, I4{}, I25{}); }
    } else {
        if (p.nc == 3) { if (p.tg == 9) go(I2{}, I3{}, I9{}); else go(I2{}, I3{}, I13{}); }
        else { if (p.tg == 9) go(I2{}, I4{}, I9{}); else go(I2{}, I4{}, I13{}); }
    }
}

template <int TM, int TN, int WM_, int WN_, int NT>
static void launch_wgrad(const WgradArgs& a, bool vp, bool vq, bool sqr, dim3 grid, hipStream_t st) {
    if (vp && vq && sqr) hipLaunchKernelGGL((wgrad_kernel<TM, TN, WM_, WN_, NT, true, true, true>), grid, dim3(256), 0, st, a);
    else if (vp && vq) hipLaunchKernelGGL((wgrad_kernel<TM, TN, WM_, WN_, NT, true, true, false>), grid, dim3(256), 0, st, a);
    else if (vp) hipLaunchKernelGGL((wgrad_kernel<TM, TN, WM_, WN_, NT, true, false, false>), grid, dim3(256), 0, st, a);
    else if (vq) hipLaunchKernelGGL((wgrad_kernel<TM, TN, WM_, WN_, NT, false, true, false>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((wgrad_kernel<TM, TN, WM_, WN_, NT, false, false, false>), grid, dim3(256), 0, st, a);
}

}  // namespace hyres

extern "C" {

static long long wgrad_slab_floats(const hyres_wgrad_desc* e, const WgradPlan& p) {
    return (long long)p.nsplit * e->ntaps * (long long)e->M * e->N;
}

long long hyres_wgrad_workspace_bytes(const hyres_wgrad_desc* d) {
    const bool swap = wgrad_swap(d);
    hyres_wgrad_desc e = swap ? wgrad_swapped(d) : *d;
    WgradPlan p = wgrad_plan(&e);
    // + the bias-gradient partials: [nsplit][M] in the kernel, or colsum partials when swapped
    auto need = [&](const WgradPlan& q) {
        const long long bias = swap ? hyres_colsum_workspace_bytes(d->B * d->Hq * d->Wq, d->M) / 4 + 4
                                    : (long long)q.nsplit * e.M + 4;
        return (wgrad_slab_floats(&e, q) + bias + wgrad_cvt_floats(&e, wgrad_native_io(&e, false))) * 4;
    };
    long long bytes = need(p);
    ThinPlan tp;
    if (thin_plan(&e, &tp)) {  // one slab row per thin block (the launch may still take the generic path
        WgradPlan q = p;       // when P is not 16-byte aligned: cover both)
        q.nsplit = tp.nblk;
        bytes = std::max(bytes, need(q));
    }
    return bytes;
}

// Launch the weight-gradient GEMM (and, for the swapped small-M layers, the bias column sums) and describe the
// split-K slab reduce that remains as jobs[0] (weight) and jobs[1] (the [nsplit][M] bias partials, if any).
static int wgrad_issue(const hyres_wgrad_desc* d0, const float* pp, const float* qq, float* dst, float* dbias,
                       void* ws, long long ws_bytes, hyres_stream_t s, hyres_wgrad_job* jobs, int* njobs) {
    *njobs = 0;
    HY_REQUIRE(d0 && pp && qq && dst, HYRES_E_ARG, "wgrad: NULL");
    const long long need = hyres_wgrad_workspace_bytes(d0);
    HY_REQUIRE(ws && ws_bytes >= need, HYRES_E_WORKSPACE, "wgrad: workspace %lld < %lld", ws_bytes, need);
    const float* p_orig = pp;
    const bool swap = wgrad_swap(d0);
    hyres_wgrad_desc dd = swap ? wgrad_swapped(d0) : *d0;
    const hyres_wgrad_desc* d = &dd;
    if (swap) std::swap(pp, qq);
    WgradPlan p = wgrad_plan(d);
    ThinPlan tp;
    const bool thin = thin_plan(d, &tp) && aligned16(pp);
    if (thin) p.nsplit = tp.nblk;
    float* bias_ws = (float*)ws + wgrad_slab_floats(d, p);
    int io = dd.io_f16 & 3;
    {
        // fp16 operands the chosen kernel cannot read: contiguous fp32 copies after the slab and bias partials
        // (the plan does not depend on the operand dtype or pixel stride beyond the checks below)
        const int native = wgrad_native_io(d, thin);
        const int cvt = io & ~native;
        auto al4 = [](long long n) { return (n + 3) & ~3LL; };
        float* cws = (float*)ws + al4(wgrad_slab_floats(d, p) + (swap ? hyres_colsum_workspace_bytes(d0->B * d0->Hq * d0->Wq,
                                                                                                      d0->M) / 4 + 4
                                                                      : (long long)p.nsplit * d->M + 4));
        hipStream_t st0 = as_stream(s);
        if (cvt & 1) {
            const long long P = (long long)dd.B * dd.Hq * dd.Wq;
            hipLaunchKernelGGL(half_to_float_2d_kernel, dim3((unsigned)std::min<long long>((P * dd.M + 255) / 256, 8192)),
                               dim3(256), 0, st0, (const _Float16*)pp, dd.ldp, cws, P, dd.M);
            pp = cws; dd.ldp = dd.M; cws += al4(P * dd.M);
        }
        if (cvt & 2) {
            const long long P = (long long)dd.B * dd.Hqq * dd.Wqq;
            hipLaunchKernelGGL(half_to_float_2d_kernel, dim3((unsigned)std::min<long long>((P * dd.N + 255) / 256, 8192)),
                               dim3(256), 0, st0, (const _Float16*)qq, dd.ldq, cws, P, dd.N);
            qq = cws; dd.ldq = dd.N;
        }
        if (cvt) {
            int rc0 = HY_LAUNCH_CHECK("half_to_float_2d");
            if (rc0) return rc0;
        }
        io &= native;
        dd.io_f16 = io;
    }
    const bool vp = (d->M % 4 == 0) && (d->ldp % 4 == 0) && aligned16(pp);
    const bool vq = !p.tapn && (d->N % 4 == 0) && (d->ldq % 4 == 0) && aligned16(qq);
    HY_REQUIRE(!d->square_q || (vp && vq), HYRES_E_SHAPE, "wgrad: square_q needs the vector path");
    // the plan (chunk size, split count, workspace) assumed the f16 kernel: its operands must be aligned
    HY_REQUIRE(!wgrad_f16_ok(d) || (vp && vq), HYRES_E_ALIGN, "wgrad(f16): P/Q must be 16-byte aligned");
    HY_REQUIRE(!p.halo || (vp && vq), HYRES_E_ALIGN, "wgrad(halo): P/Q must be 16-byte aligned");
    WgradArgs a;
    a.d = *d; a.p = pp; a.q = qq; a.slab = (float*)ws; a.chunks_per_split = p.cps; a.nchunks = p.nchunks;
    a.mtiles = p.mtiles; a.ntiles = p.ntiles; a.ngroups = p.ngroups; a.nblocks = p.nblocks; a.tapn = p.tapn;
    a.bias_slab = (dbias && !swap) ? bias_ws : nullptr;
    dim3 grid(ceil_div(p.nblocks, 8) * 8);
    hipStream_t st = as_stream(s);
    const bool sqr = d->square_q != 0;
    const bool one = !thin && !p.halo && !wgrad_f16_ok(d) && !sqr && !p.tapn && vp && vq &&
                     d->ntaps == 1 && d->dh[0] == 0 && d->dw[0] == 0 && d->sq == 1 && d->Hqq == d->Hq &&
                     d->Wqq == d->Wq && p.ngroups == 1;
    const bool pf2 = g_tune[15] == 2 && (long long)d->B * d->Hq * d->Wq * std::max(d->ldp, d->ldq) * 4 < 0x7FFFFFF0LL;
    if (one && f32_gemm_bf6() && pf2) {  // loads two chunks ahead (key 15 = 2)
        if (p.TMc == 2 && p.TNc == 2) hipLaunchKernelGGL((wgrad1x1_bf6_pf2_kernel<2, 2, 2, 2>), grid, dim3(256), 0, st, a);
        else if (p.TMc == 2) hipLaunchKernelGGL((wgrad1x1_bf6_pf2_kernel<2, 1, 2, 2>), grid, dim3(256), 0, st, a);
        else if (p.WMc == 1) hipLaunchKernelGGL((wgrad1x1_bf6_pf2_kernel<1, 1, 1, 4>), grid, dim3(256), 0, st, a);
        else if (p.WNc == 1) hipLaunchKernelGGL((wgrad1x1_bf6_pf2_kernel<1, 1, 4, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad1x1_bf6_pf2_kernel<1, 1, 2, 2>), grid, dim3(256), 0, st, a);
    } else if (one && f32_gemm_bf6()) {  // bf16x6 products (the plan keeps one 4-wave group per block for it)
        if (p.TMc == 2 && p.TNc == 2) hipLaunchKernelGGL((wgrad1x1_bf6_kernel<2, 2, 2, 2>), grid, dim3(256), 0, st, a);
        else if (p.TMc == 2) hipLaunchKernelGGL((wgrad1x1_bf6_kernel<2, 1, 2, 2>), grid, dim3(256), 0, st, a);
        else if (p.WMc == 1) hipLaunchKernelGGL((wgrad1x1_bf6_kernel<1, 1, 1, 4>), grid, dim3(256), 0, st, a);
        else if (p.WNc == 1) hipLaunchKernelGGL((wgrad1x1_bf6_kernel<1, 1, 4, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad1x1_bf6_kernel<1, 1, 2, 2>), grid, dim3(256), 0, st, a);
    } else if (one) {
        auto w1 = [&](auto gc) {
            constexpr int G_ = decltype(gc)::value;
            const dim3 blk(256 * G_);
            if (p.TMc == 2 && p.TNc == 2) hipLaunchKernelGGL((wgrad1x1_kernel<2, 2, 2, 2, G_>), grid, blk, 0, st, a);
            else if (p.TMc == 2) hipLaunchKernelGGL((wgrad1x1_kernel<2, 1, 2, 2, G_>), grid, blk, 0, st, a);
            else if (p.WMc == 1) hipLaunchKernelGGL((wgrad1x1_kernel<1, 1, 1, 4, G_>), grid, blk, 0, st, a);
            else if (p.WNc == 1) hipLaunchKernelGGL((wgrad1x1_kernel<1, 1, 4, 1, G_>), grid, blk, 0, st, a);
            else hipLaunchKernelGGL((wgrad1x1_kernel<1, 1, 2, 2, G_>), grid, blk, 0, st, a);
        };
        if (p.g1x1 == 2) w1(std::integral_constant<int, 2>{});
        else w1(std::integral_constant<int, 1>{});
    } else if (thin) {
        launch_thin(a, tp, (io & 1) != 0, st);
    } else if (p.halo && wgrad_f16_ok(d)) {
        auto halo16 = [&](auto ioc, auto gc) {
            constexpr int IO_ = decltype(ioc)::value, G_ = decltype(gc)::value;
            const dim3 blk(256 * G_);
            if (p.hk == 3 && p.NT == 3 && p.hdil == 2)
                hipLaunchKernelGGL((wgrad_halo_f16_kernel<1, 3, 1, 2, IO_, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3 && p.NT == 3)
                hipLaunchKernelGGL((wgrad_halo_f16_kernel<1, 3, 1, 1, IO_, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3 && p.hdil == 2)
                hipLaunchKernelGGL((wgrad_halo_f16_kernel<3, 3, 1, 2, IO_, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3)
                hipLaunchKernelGGL((wgrad_halo_f16_kernel<3, 3, 1, 1, IO_, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (d->sq == 1)  // 5x5 stride 1: one group (3 blocks per CU)
                hipLaunchKernelGGL((wgrad_halo_f16_kernel<1, 5, 1, 1, IO_>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
            else hipLaunchKernelGGL((wgrad_halo_f16_kernel<1, 5, 2, 1, IO_, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
        };
        auto halo16g = [&](auto ioc) { halo16(ioc, std::integral_constant<int, 1>{}); };
        if (io == 1) halo16g(std::integral_constant<int, 1>{});
        else if (io == 2) halo16g(std::integral_constant<int, 2>{});
        else if (io == 3) halo16g(std::integral_constant<int, 3>{});
        else halo16g(std::integral_constant<int, 0>{});
    } else if (p.halo && f32_gemm_bf6() && g_tune[16] == 2 && (p.NT == 3 || (p.NT == 5 && g_tune[22] != 0)) &&
               (long long)d->B * d->Hqq * d->Wqq * d->ldq * 4 < 0x7FFFFFF0LL &&
               (long long)d->B * d->Hq * d->Wq * d->ldp * 4 < 0x7FFFFFF0LL) {  // loads two chunks ahead (key 16 = 2)
        if (p.hk == 3 && p.hdil == 2)
            hipLaunchKernelGGL((wgrad_halo_bf6_pf2_kernel<3, 1, 2>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (p.hk == 3)
            hipLaunchKernelGGL((wgrad_halo_bf6_pf2_kernel<3, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (d->sq == 1)
            hipLaunchKernelGGL((wgrad_halo_bf6_pf2_kernel<5, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else hipLaunchKernelGGL((wgrad_halo_bf6_pf2_kernel<5, 2, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
    } else if (p.halo && f32_gemm_bf6()) {  // fp32 operands (fp16 ones were converted above), bf16x6 products
        if (p.hk == 3 && p.NT == 3 && p.hdil == 2)
            hipLaunchKernelGGL((wgrad_halo_bf6_kernel<1, 3, 1, 2>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (p.hk == 3 && p.NT == 3)
            hipLaunchKernelGGL((wgrad_halo_bf6_kernel<1, 3, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (p.hk == 3 && p.hdil == 2)
            hipLaunchKernelGGL((wgrad_halo_bf6_kernel<3, 3, 1, 2>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (p.hk == 3)
            hipLaunchKernelGGL((wgrad_halo_bf6_kernel<3, 3, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else if (d->sq == 1)
            hipLaunchKernelGGL((wgrad_halo_bf6_kernel<1, 5, 1, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
        else hipLaunchKernelGGL((wgrad_halo_bf6_kernel<1, 5, 2, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
    } else if (p.halo) {
        auto halo32 = [&](auto gc) {
            constexpr int G_ = decltype(gc)::value;
            const dim3 blk(256 * G_);
            if (p.hk == 3 && p.NT == 3 && p.hdil == 2)
                hipLaunchKernelGGL((wgrad_halo_kernel<1, 3, 1, 2, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3 && p.NT == 3)
                hipLaunchKernelGGL((wgrad_halo_kernel<1, 3, 1, 1, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3 && p.hdil == 2)
                hipLaunchKernelGGL((wgrad_halo_kernel<3, 3, 1, 2, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (p.hk == 3)
                hipLaunchKernelGGL((wgrad_halo_kernel<3, 3, 1, 1, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
            else if (d->sq == 1)  // 5x5 stride 1: one group (3 blocks per CU)
                hipLaunchKernelGGL((wgrad_halo_kernel<1, 5, 1>), grid, dim3(256), 0, st, a, p.hdh, p.hdw);
            else hipLaunchKernelGGL((wgrad_halo_kernel<1, 5, 2, 1, G_>), grid, blk, 0, st, a, p.hdh, p.hdw);
        };
        halo32(std::integral_constant<int, 1>{});
    } else if (wgrad_f16_ok(d)) {
        const bool one16 = !sqr && d->ntaps == 1 && d->dh[0] == 0 && d->dw[0] == 0 && d->sq == 1 &&
                           d->Hqq == d->Hq && d->Wqq == d->Wq && p.ngroups == 1;
        auto f16io = [&](auto tm, auto tn, auto wm_, auto wn_, auto ntc, auto ioc) {
            constexpr int TM_ = decltype(tm)::value, TN_ = decltype(tn)::value;
            constexpr int WM2 = decltype(wm_)::value, WN2 = decltype(wn_)::value, NT_ = decltype(ntc)::value;
            constexpr int IO_ = decltype(ioc)::value;
            if (sqr) {
                // GDN: Q = x (fp16 in AMP training), P = the norm gradient (fp16 with AMP fp16 gradients)
                hipLaunchKernelGGL((wgrad_f16_kernel<TM_, TN_, WM2, WN2, NT_, true, false, IO_>), grid, dim3(256), 0, st,
                                   a);
            } else if (NT_ == 1 && one16) {
                hipLaunchKernelGGL((wgrad_f16_kernel<TM_, TN_, WM2, WN2, 1, false, true, IO_>), grid, dim3(256), 0, st,
                                   a);
            } else {
                hipLaunchKernelGGL((wgrad_f16_kernel<TM_, TN_, WM2, WN2, NT_, false, false, IO_>), grid, dim3(256), 0,
                                   st, a);
            }
        };
        auto f16 = [&](auto tm, auto tn, auto wm_, auto wn_, auto ntc) {
            if (io == 1) f16io(tm, tn, wm_, wn_, ntc, std::integral_constant<int, 1>{});
            else if (io == 2) f16io(tm, tn, wm_, wn_, ntc, std::integral_constant<int, 2>{});
            else if (io == 3) f16io(tm, tn, wm_, wn_, ntc, std::integral_constant<int, 3>{});
            else f16io(tm, tn, wm_, wn_, ntc, std::integral_constant<int, 0>{});
        };
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I4 = std::integral_constant<int, 4>;
        if (p.TMc == 2 && p.TNc == 2) f16(I2{}, I2{}, I2{}, I2{}, I1{});
        else if (p.TMc == 2) f16(I2{}, I1{}, I2{}, I2{}, I1{});
        else if (p.WMc == 1) f16(I1{}, I1{}, I1{}, I4{}, I1{});
        else if (p.WNc == 1) f16(I1{}, I1{}, I4{}, I1{}, I1{});
        else if (p.NT == 9) f16(I1{}, I1{}, I2{}, I2{}, std::integral_constant<int, 9>{});
        else if (p.NT == 5) f16(I1{}, I1{}, I2{}, I2{}, std::integral_constant<int, 5>{});
        else f16(I1{}, I1{}, I2{}, I2{}, I1{});
    } else if (p.TMc == 2 && p.TNc == 2) launch_wgrad<2, 2, 2, 2, 1>(a, vp, vq, sqr, grid, st);
    else if (p.TMc == 2) launch_wgrad<2, 1, 2, 2, 1>(a, vp, vq, sqr, grid, st);
    else if (p.WMc == 1) launch_wgrad<1, 1, 1, 4, 1>(a, vp, vq, sqr, grid, st);
    else if (p.WNc == 1) launch_wgrad<1, 1, 4, 1, 1>(a, vp, vq, sqr, grid, st);
    else if (p.NT == 9) launch_wgrad<1, 1, 2, 2, 9>(a, vp, vq, sqr, grid, st);
    else if (p.NT == 5) launch_wgrad<1, 1, 2, 2, 5>(a, vp, vq, sqr, grid, st);
    else launch_wgrad<1, 1, 2, 2, 1>(a, vp, vq, sqr, grid, st);
    int rc = HY_LAUNCH_CHECK("wgrad_kernel");
    if (rc) return rc;
    const long long total = (long long)d->ntaps * d->M * d->N;
    const int lx = reduce_lx(total, p.nsplit);
    jobs[0] = hyres_wgrad_job{(const float*)ws, dst, p.nsplit, d->ntaps, d->M, d->N, d->sm, d->sn, d->st,
                              d->accumulate, lx, 0};
    *njobs = 1;
    if (dbias && !swap) {  // [nsplit][M] partials = a [nsplit][1][M][1] slab, reduced with the weight's layout
        jobs[1] = hyres_wgrad_job{(const float*)bias_ws, dbias, p.nsplit, 1, d->M, 1, 1, 0, 0, d->accumulate, lx, 0};
        *njobs = 2;
    }
    if (dbias && swap) {  // P (= dY) is the tap-folded side here: plain column sums (own workspace after the slab)
        const int P = d0->B * d0->Hq * d0->Wq;
        if (d0->io_f16 & 1)
            return hyres_colsum_f16(p_orig, P, d0->M, d0->ldp, dbias, d0->accumulate, bias_ws,
                                    hyres_colsum_workspace_bytes(P, d0->M), s);
        return hyres_colsum(p_orig, P, d0->M, d0->ldp, dbias, d0->accumulate, bias_ws,
                            hyres_colsum_workspace_bytes(P, d0->M), s);
    }
    return 0;
}

int hyres_conv_wgrad(const hyres_wgrad_desc* d, const float* pp, const float* qq, float* dst, float* dbias,
                     void* ws, long long ws_bytes, hyres_stream_t s) {
    hyres_wgrad_job jobs[2];
    int nj = 0;
    int rc = wgrad_issue(d, pp, qq, dst, dbias, ws, ws_bytes, s, jobs, &nj);
    if (rc || nj == 0) return rc;
    const hyres_wgrad_job& w = jobs[0];
    const long long total = (long long)w.ntaps * w.M * w.N;
    const int outb = 4 * w.lanes;
    hipStream_t st = as_stream(s);
    auto reduce = [&](auto lxc) {
        constexpr int LX = decltype(lxc)::value;
        if (nj == 2) {  // the [nsplit][M] bias partials reduced by the same launch
            const hyres_wgrad_job& b = jobs[1];
            const int nb_w = (int)ceil_div(total, outb);
            hipLaunchKernelGGL(wgrad_bias_reduce_kernel<LX>, dim3(nb_w + ceil_div(b.M, outb)), dim3(256), 0, st,
                               w.slab, w.nsplit, w.ntaps, w.M, w.N, w.dst, w.sm, w.sn, w.st, w.accumulate, nb_w,
                               b.slab, b.dst);
            return HY_LAUNCH_CHECK("wgrad_bias_reduce_kernel");
        }
        hipLaunchKernelGGL(wgrad_reduce_kernel<LX>, dim3(ceil_div(total, outb)), dim3(256), 0, st, w.slab, w.nsplit,
                           w.ntaps, w.M, w.N, w.dst, w.sm, w.sn, w.st, w.accumulate);
        return HY_LAUNCH_CHECK("wgrad_reduce_kernel");
    };
    if (w.lanes == 16) return reduce(std::integral_constant<int, 16>{});
    if (w.lanes == 8) return reduce(std::integral_constant<int, 8>{});
    return reduce(std::integral_constant<int, 4>{});
}

int hyres_conv_wgrad_deferred(const hyres_wgrad_desc* d, const float* pp, const float* qq, float* dst,
                              float* dbias, void* ws, long long ws_bytes, hyres_wgrad_job* jobs, int* njobs,
                              hyres_stream_t s) {
    HY_REQUIRE(jobs && njobs, HYRES_E_ARG, "wgrad_deferred: NULL job output");
    return wgrad_issue(d, pp, qq, dst, dbias, ws, ws_bytes, s, jobs, njobs);
}

int hyres_wgrad_reduce_jobs(const hyres_wgrad_job* jobs, int n, hyres_stream_t s) {
    HY_REQUIRE(n >= 0 && (n == 0 || jobs), HYRES_E_ARG, "wgrad_reduce_jobs: bad job list");
    hipStream_t st = as_stream(s);
    for (int i0 = 0; i0 < n; i0 += HYRES_WGRAD_MAX_JOBS) {
        WgradJobBatch b{};
        b.n = std::min(HYRES_WGRAD_MAX_JOBS, n - i0);
        long long blocks = 0;
        for (int k = 0; k < b.n; ++k) {
            const hyres_wgrad_job& j = jobs[i0 + k];
            HY_REQUIRE(j.slab && j.dst && j.nsplit >= 1 && j.ntaps >= 1 && j.M >= 1 && j.N >= 1 &&
                           (j.lanes == 4 || j.lanes == 8 || j.lanes == 16),
                       HYRES_E_ARG, "wgrad_reduce_jobs: bad job %d", i0 + k);
            b.j[k] = j;
            blocks += ceil_div((long long)j.ntaps * j.M * j.N, 4 * j.lanes);
            HY_REQUIRE(blocks < (1LL << 31), HYRES_E_SHAPE, "wgrad_reduce_jobs: too many blocks");
            b.end[k] = (int)blocks;
        }
        hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b);
        const int rc = HY_LAUNCH_CHECK("wgrad_reduce_batch_kernel");
        if (rc) return rc;
    }
    return 0;
}

static int colsum_blocks(int P) {
    // >= 128 rows per block, at most 512 partial rows
    int nb = std::max(1, std::min(ceil_div(P, 128), 512));
    int rows = ceil_div(P, nb);
    return ceil_div(P, rows);
}

long long hyres_colsum_workspace_bytes(int P, int C) { return (long long)colsum_blocks(P) * C * 4; }

static int colsum_impl(const float* x, int P, int C, int ld, float* dst, int accumulate, void* ws, long long ws_bytes,
                       bool h, hyres_stream_t s) {
    HY_REQUIRE(x && dst && P > 0 && C > 0, HYRES_E_ARG, "colsum: bad args");
    const int nb = colsum_blocks(P);
    const int rows = ceil_div(P, nb);
    HY_REQUIRE(ws && ws_bytes >= (long long)nb * C * 4, HYRES_E_WORKSPACE, "colsum: workspace");
    hipStream_t st = as_stream(s);
    const bool vec = (C % 4 == 0) && (ld % 4 == 0) && aligned16(x);
    if (vec && h)
        hipLaunchKernelGGL((colsum_partial_kernel<4, true>), dim3(nb), dim3(256), 0, st, x, P, C, ld, rows, (float*)ws);
    else if (h)
        hipLaunchKernelGGL((colsum_partial_kernel<1, true>), dim3(nb), dim3(256), 0, st, x, P, C, ld, rows, (float*)ws);
    else if (vec)
        hipLaunchKernelGGL(colsum_partial_kernel<4>, dim3(nb), dim3(256), 0, st, x, P, C, ld, rows, (float*)ws);
    else
        hipLaunchKernelGGL(colsum_partial_kernel<1>, dim3(nb), dim3(256), 0, st, x, P, C, ld, rows, (float*)ws);
    int rc = HY_LAUNCH_CHECK("colsum_partial");
    if (rc) return rc;
    // the [nb][C] partials = a [nb][1][C][1] slab: the parallel deterministic split reduce (round 3; the former
    // colsum_final walked nb/4 partial rows serially per thread: 24 us per launch on C = 64)
    const int lx = reduce_lx(C, nb);
    if (lx == 16)
        hipLaunchKernelGGL(wgrad_reduce_kernel<16>, dim3(ceil_div(C, 64)), dim3(256), 0, st, (const float*)ws, nb, 1, C,
                           1, dst, 1, 0, 0, accumulate);
    else if (lx == 8)
        hipLaunchKernelGGL(wgrad_reduce_kernel<8>, dim3(ceil_div(C, 32)), dim3(256), 0, st, (const float*)ws, nb, 1, C,
                           1, dst, 1, 0, 0, accumulate);
    else
        hipLaunchKernelGGL(wgrad_reduce_kernel<4>, dim3(ceil_div(C, 16)), dim3(256), 0, st, (const float*)ws, nb, 1, C,
                           1, dst, 1, 0, 0, accumulate);
    return HY_LAUNCH_CHECK("colsum_reduce");
}

int hyres_colsum(const float* x, int P, int C, int ld, float* dst, int accumulate, void* ws,
                 long long ws_bytes, hyres_stream_t s) {
    return colsum_impl(x, P, C, ld, dst, accumulate, ws, ws_bytes, false, s);
}
int hyres_colsum_f16(const void* x, int P, int C, int ld, float* dst, int accumulate, void* ws,
                     long long ws_bytes, hyres_stream_t s) {
    return colsum_impl((const float*)x, P, C, ld, dst, accumulate, ws, ws_bytes, true, s);
}

}  // extern "C"
