// Shared helpers for the gfx950 kernels of libedgedet.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/edgedet.h"

namespace edgedet {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ host-side error channel
void set_error(const std::string& msg);
const char* get_error();

#define EDGEDET_CHECK_HIP(expr)                                                              \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            ::edgedet::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));       \
            return -2;                                                                       \
        }                                                                                    \
    } while (0)

#define EDGEDET_REQUIRE(cond, msg)                                                           \
    do {                                                                                     \
        if (!(cond)) {                                                                       \
            ::edgedet::set_error(std::string("edgedet: ") + (msg));                          \
            return -1;                                                                       \
        }                                                                                    \
    } while (0)

#define EDGEDET_LAUNCH_CHECK()                                                               \
    do {                                                                                     \
        hipError_t _e = hipGetLastError();                                                   \
        if (_e != hipSuccess) {                                                              \
            ::edgedet::set_error(std::string("kernel launch: ") + hipGetErrorString(_e));  \
            return -3;                                                                       \
        }                                                                                    \
    } while (0)

// ------------------------------------------------------------------ activations
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2, ACT_HSWISH = 3, ACT_HSIGMOID = 4, ACT_SIGMOID = 5 };

// Same operation order as ATen's CPU kernels (hardswish: x * min(max(x + 3, 0), 6) / 6;
// hardsigmoid: min(max(x + 3, 0), 6) / 6).
__device__ __forceinline__ float apply_act(float v, int act) {
    switch (act) {
        case ACT_RELU: return v > 0.f ? v : 0.f;
        case ACT_RELU6: return fminf(fmaxf(v, 0.f), 6.f);
        case ACT_HSWISH: return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
        case ACT_HSIGMOID: return fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
        case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
        default: return v;
    }
}

// ------------------------------------------------------------------ fast unsigned division
// q = n / d for n < 2^31 via multiply-high (Granlund–Montgomery, round-up variant).
struct FastDiv {
    uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    f.s = s;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (__umulhi(n, f.m) + n) >> f.s;
}

// float -> uint32 whose unsigned order equals the float order (NaN excluded)
__device__ __forceinline__ uint32_t float_key(float x) {
    uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Block-wide copy into LDS with U independent loads in flight per thread: dst[t] = src(t), t < n.
// (A plain strided loop issues one load per iteration and waits for it before the store: one memory
// round trip per element, the dominant cost of small latency-bound kernels.)
template <int NT, int U, typename T, typename F>
__device__ __forceinline__ void stage_lds(T* dst, int n, F src) {
    for (int base = threadIdx.x; base < n; base += NT * U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = base + NT * u;
            v[u] = src(t < n ? t : n - 1);  // clamped index: every load is issued unconditionally
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + NT * u < n) dst[base + NT * u] = v[u];
    }
}

}  // namespace edgedet
