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

}  // namespace hyres

#define HY_REQUIRE(cond, code, ...)                                  \
    do {                                                             \
        if (!(cond)) return ::hyres::set_error((code), __VA_ARGS__); \
    } while (0)

#define HY_LAUNCH_CHECK(name) ::hyres::launch_status(name)
