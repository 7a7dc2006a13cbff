// Internal declarations shared by the convolution (conv.hip) and weight-gradient (wgrad.hip) units.
#pragma once
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

namespace hyres {

constexpr int KT = 32;  // K chunk (floats)

// tile / split-K overrides set through hyres_conv_tuning (conv.hip; -1 = the planners' heuristics)
extern int g_tune[HYRES_TUNE_KEYS];

// fp32 GEMMs on the bf16 MFMA (hyres_conv_tuning key 7 = 1, the default): "bf16x6"
inline bool f32_gemm_bf6() { return g_tune[7] == 1; }

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

// fp32 -> three bf16 pieces h + m + l (24 significant bits, remainder <= 2^-25 |x|): the bf16x6 fp32 GEMM's operands
__device__ __forceinline__ void bf6_split4(float4 v, bf16x4_t& h, bf16x4_t& m, bf16x4_t& l) {
    const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const __bf16 a = (__bf16)x[i];
        const float r1 = x[i] - (float)a;
        const __bf16 b = (__bf16)r1;
        h[i] = a;
        m[i] = b;
        l[i] = (__bf16)(r1 - (float)b);
    }
}

// acc += a * b to fp32 accuracy from the three-piece operands: the six cross products with i + j <= 2, the
// smallest first
__device__ __forceinline__ floatx16 bf6_mfma(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], floatx16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}


}  // namespace hyres
