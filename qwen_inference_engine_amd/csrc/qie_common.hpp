// qie_common.hpp — shared device/host helpers for the qie HIP kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/qie/qie_types.h"

namespace qie {

// ----------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...);

#define QIE_HIP(expr)                                                          \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess)                                                  \
            return ::qie::fail((int)_e, "%s:%d %s -> %s", __FILE__, __LINE__,  \
                               #expr, hipGetErrorString(_e));                  \
    } while (0)

#define QIE_LAUNCH_CHECK()                                                     \
    do {                                                                       \
        hipError_t _e = hipGetLastError();                                     \
        if (_e != hipSuccess)                                                  \
            return ::qie::fail((int)_e, "%s:%d launch -> %s", __FILE__,        \
                               __LINE__, hipGetErrorString(_e));               \
    } while (0)

#define QIE_REQUIRE(cond, ...)                                                 \
    do {                                                                       \
        if (!(cond)) return ::qie::fail(-22, __VA_ARGS__);                     \
    } while (0)

constexpr int kWave = 64;

// ------------------------------------------------------------- bf16 helpers
__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Round-to-nearest-even f32 -> bf16 (== __float2bfloat16 for finite values;
// gfx950 lowers the __bf16 cast to v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// Selection key of the reference's arg-max / top-k (logit_decode.cu:15-33,
// 149-274): larger value wins; among equal values the winner maximises
// bitrev8(idx mod 256), then minimises idx.  0 means "no candidate"
// (NaN and -inf are never selected by the reference: strict > from -INF).
__device__ __forceinline__ uint64_t sel_key(float v, uint32_t idx) {
    if (!(v > -INFINITY)) return 0ull;
    uint32_t u = __float_as_uint(v);
    uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    uint32_t br = __builtin_bitreverse32(idx & 0xffu) >> 24;
    return ((uint64_t)ord << 32) | ((uint64_t)br << 24) | (uint64_t)((~idx) & 0xffffffu);
}
__device__ __forceinline__ int32_t key_idx(uint64_t key) {
    return key == 0ull ? -1 : (int32_t)((~(uint32_t)key) & 0xffffffu);
}
__device__ __forceinline__ float key_val(uint64_t key) {
    uint32_t ord = (uint32_t)(key >> 32);
    uint32_t u = (ord & 0x80000000u) ? (ord & 0x7fffffffu) : ~ord;
    return __uint_as_float(u);
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Device properties cached per process (CU count for persistent grids).
int device_cu_count();

}  // namespace qie
