// Internal helpers shared by the libhyres_hip translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "hyres_hip.h"

namespace hyres {

int set_error(int code, const char* fmt, ...);
int ok();

inline hipStream_t as_stream(hyres_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error((int)e, "%s: %s", what, hipGetErrorString(e));
    return ok();
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

typedef _Float16 half4_t __attribute__((ext_vector_type(4)));

// activation element / float4 access: fp32, or fp16 storage in HBM (H, autocast inference) with fp32 arithmetic
template <bool H>
__device__ __forceinline__ float ldv(const float* p, long long i) {
    if constexpr (H) return (float)reinterpret_cast<const _Float16*>(p)[i];
    else return p[i];
}
template <bool H>
__device__ __forceinline__ void stv(float* p, long long i, float v) {
    if constexpr (H) reinterpret_cast<_Float16*>(p)[i] = (_Float16)v;
    else p[i] = v;
}
template <bool H>
__device__ __forceinline__ float4 ldv4(const float* p, long long i) {
    if constexpr (H) {
        const half4_t h = *reinterpret_cast<const half4_t*>(reinterpret_cast<const _Float16*>(p) + i);
        return make_float4((float)h.x, (float)h.y, (float)h.z, (float)h.w);
    } else {
        return ld4(p + i);
    }
}
template <bool H>
__device__ __forceinline__ void stv4(float* p, long long i, float4 v) {
    if constexpr (H) {
        const half4_t h = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
        *reinterpret_cast<half4_t*>(reinterpret_cast<_Float16*>(p) + i) = h;
    } else {
        *reinterpret_cast<float4*>(p + i) = v;
    }
}

}  // namespace hyres

#define HY_REQUIRE(cond, code, ...)                                  \
    do {                                                             \
        if (!(cond)) return ::hyres::set_error((code), __VA_ARGS__); \
    } while (0)

#define HY_LAUNCH_CHECK(name) ::hyres::launch_status(name)
