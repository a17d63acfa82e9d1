// qie_common.hpp — shared device/host helpers for the qie HIP kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/qie/qie_types.h"

struct qie_kv_cache;

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

#ifndef QIE_TRY
#define QIE_TRY(expr)                                                          \
    do {                                                                       \
        const int _rc = (expr);                                                \
        if (_rc) return _rc;                                                   \
    } while (0)
#endif

constexpr int kWave = 64;

// ------------------------------------------------------------- dev knobs
// A/B and timing knobs (environment variables, kernel debug early exits) exist only in the
// development build (`make DEV=1` -> lib/dev/libqie.so; tools point QIE_LIB at it).  The
// shipped library compiles every knob to its default and the debug branches away.
#ifdef QIE_DEV
inline int dev_env(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}
#define QIE_DBG(expr) (expr)
#else
inline int dev_env(const char*, int dflt) { return dflt; }
#define QIE_DBG(expr) false
#endif

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
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (same RNE as f2bf; the scalar
// form converts each half separately and merges with a shift and an or)
typedef __bf16 qie_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float qie_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((qie_f32x2_t{lo, hi}), qie_bf16x2_t));
}

// ------------------------------------------------------ fp8 (OCP e4m3fn) weights
// A quantised weight row = e4m3 codes times a power-of-two row scale, so every
// dequantised value (3 mantissa bits x 2^k) is exactly a bf16: the fp8 engine computes
// the same products as a bf16 model whose weights are those dequantised values
// (tests/oracle run exactly that).  Encode: round to nearest even, saturate at 448.
__host__ __device__ inline uint8_t e4m3_encode(float v) {
    const uint32_t sign = v < 0.f ? 0x80u : 0u;
    float a = fabsf(v);
    if (!(a > 0.f)) return (uint8_t)sign;                 // +-0 (NaN never produced upstream)
    if (a >= 448.f) return (uint8_t)(sign | 0x7Eu);       // saturate (max finite 1.75 * 2^8)
    if (a < 0.015625f) {                                  // subnormal range: step 2^-9
        const uint32_t m = (uint32_t)rintf(a * 512.f);    // 0..8; 8 == 2^-6, code 0x08 (normal)
        return (uint8_t)(sign | m);
    }
    int e;
    const float f = frexpf(a, &e);                        // a = f * 2^e, f in [0.5, 1)
    int E = e - 1;                                        // a = (2 f) * 2^E, 2f in [1, 2)
    uint32_t m3 = (uint32_t)rintf((2.f * f - 1.f) * 8.f); // 0..8
    if (m3 == 8) { m3 = 0; E += 1; }
    uint32_t code = ((uint32_t)(E + 7) << 3) | m3;
    if (code > 0x7Eu) code = 0x7Eu;
    return (uint8_t)(sign | code);
}
__host__ __device__ inline float e4m3_decode(uint8_t b) {
    const int ex = (b >> 3) & 0xF, man = b & 7;
    const float v = ex == 0 ? (float)man * 0.001953125f : ldexpf(1.f + (float)man * 0.125f, ex - 7);
    return (b & 0x80) ? -v : v;
}
// power-of-two row scale: the smallest 2^k with amax / 2^k <= 448
__host__ __device__ inline float e4m3_row_scale(float amax) {
    if (!(amax > 0.f)) return 1.f;
    int e;
    frexpf(amax / 448.f, &e);                             // amax / 448 = f * 2^e, f in [0.5, 1)
    float s = ldexpf(1.f, e);                             // s >= amax / 448
    if (ldexpf(1.f, e - 1) * 448.f >= amax) s = ldexpf(1.f, e - 1);
    if (s * 448.f < amax) s *= 2.f;                       // exact checks: the division rounded
    // never below the smallest normal: the scale's exponent field is the MFMA's e8m0 operand
    // (read from the float bits), and a subnormal s would read as exponent 0
    const float smin = ldexpf(1.f, -126);
    return s < smin ? smin : s;
}
// 4 packed codes -> 4 floats (v_cvt_pk_f32_fp8; gfx950 "fp8" is OCP e4m3fn — checked
// against e4m3_decode for all 256 codes by tests/test_gpu_fp8.py)
__device__ __forceinline__ void fp8x4_to_f32(uint32_t w, float* f) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
    f[0] = lo[0];
    f[1] = lo[1];
    f[2] = hi[0];
    f[3] = hi[1];
}

// four e4m3 codes -> four bf16, two per instruction (gfx950 v_cvt_scalef32_pk_bf16_fp8,
// scale 1.0).  Every e4m3 value, subnormals included, is a bf16, so the conversion is exact;
// tests/test_gpu_fp8.py::test_fp8_decode_bf16_all_codes checks all 256 codes against the
// e4m3fn table (qie_debug_fp8_decode_bf16).  Half the VALU of fp8 -> f32 -> bf16.
__device__ __forceinline__ uint2 fp8x4_to_bf16x4(uint32_t w) {
    const auto lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w, 1.0f, false);
    const auto hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w, 1.0f, true);
    return make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
}

// A uniform pointer as an opaque register value: per-lane selects between
// laundered pointers stay v_cndmask on values instead of being folded into a per-lane
// load of the kernel-argument slot (which costs a vmcnt(0) round trip).
template <class T>
__device__ __forceinline__ const T* launder_ptr(const T* p) {
    asm volatile("" : "+v"(p));
    return p;
}

__device__ __forceinline__ uint64_t launder_u64(uint64_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

// ------------------------------------------------------- KV cache addressing
// qie_kv_cache in kernel form.  A (layer, kv head) run holds `run` consecutive tokens:
// max_ctx of one sequence (contiguous) or page_tokens of one page (paged).  The run of
// (lg = layer*nkv + kv head) starts at base + lg*run*hd; kv_tok adds the offset of
// token `tok` of sequence `seq` (paged: through the block table, page = tok >> shift).
struct KvMap {
    const int32_t* table;   // paged: [n_seq][max_pages]; null: contiguous
    int64_t stride;         // elements between sequences (contiguous) / pages (paged)
    int run;                // tokens per (layer, kv head) run
    int shift;              // paged: log2(page_tokens)
    int max_pages;
};

template <bool PG>
__device__ __forceinline__ int64_t kv_tok(const KvMap& k, int64_t seq, int tok, int hd) {
    if constexpr (PG)
        return (int64_t)k.table[seq * k.max_pages + (tok >> k.shift)] * k.stride +
               (int64_t)(tok & ((1 << k.shift) - 1)) * hd;
    else
        return seq * k.stride + (int64_t)tok * hd;
}
// Validated KvMap of a public cache descriptor (k_misc.hip); `who` names the caller.
int kv_map_make(const qie_kv_cache* c, KvMap* out, const char* who);

// run-relative offset of the first element of (layer, kv head) lg
__host__ __device__ __forceinline__ int64_t kv_run_off(const KvMap& k, int64_t lg, int hd) {
    return lg * k.run * (int64_t)hd;
}

// ------------------------------------------------------ cross-lane reductions
// __shfl_xor lowers to ds_bpermute_b32 (an LDS round trip, ~100 cycles); chains of
// them serialised the decode attention.  These use DPP row ops (folded into the
// VALU op, e.g. v_add_f32_dpp) within 16-lane rows and gfx950's
// v_permlane16/32_swap across rows — no LDS traffic.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// every lane gets op over the N-lane aligned group it belongs to (N in 2,4,8,16):
// xor 1, xor 2 (quad_perm), then mirrored halves (row_half_mirror) and rows (row_mirror).
template <int N>
__device__ __forceinline__ float group_sum(float v) {
    if constexpr (N >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    if constexpr (N >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    if constexpr (N >= 8) v += dpp_f<0x141>(v);  // row_half_mirror
    if constexpr (N >= 16) v += dpp_f<0x140>(v); // row_mirror
    return v;
}
template <int N>
__device__ __forceinline__ float group_max(float v) {
    if constexpr (N >= 2) v = fmaxf(v, dpp_f<0xB1>(v));
    if constexpr (N >= 4) v = fmaxf(v, dpp_f<0x4E>(v));
    if constexpr (N >= 8) v = fmaxf(v, dpp_f<0x141>(v));
    if constexpr (N >= 16) v = fmaxf(v, dpp_f<0x140>(v));
    return v;
}
// op with lane ^ 16 / lane ^ 32 (v_permlane16_swap / v_permlane32_swap on two copies).
// Inline asm: the __builtin_amdgcn_permlane*_swap builtins with both operands equal are
// miscompiled by this toolchain (both results read from the same register).  The s_nops
// cover the VALU-write -> permlane-read hazard and the result read after it.
template <int W>
__device__ __forceinline__ void lane_swap(float& a, float& b) {
    if constexpr (W == 16)
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    else
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xor16_sum(float v) { float a = v, b = v; lane_swap<16>(a, b); return a + b; }
__device__ __forceinline__ float xor32_sum(float v) { float a = v, b = v; lane_swap<32>(a, b); return a + b; }
__device__ __forceinline__ float xor16_max(float v) { float a = v, b = v; lane_swap<16>(a, b); return fmaxf(a, b); }
__device__ __forceinline__ float xor32_max(float v) { float a = v, b = v; lane_swap<32>(a, b); return fmaxf(a, b); }
__device__ __forceinline__ float wave_sum(float v) { return xor32_sum(xor16_sum(group_sum<16>(v))); }
__device__ __forceinline__ float wave_max(float v) { return xor32_max(xor16_max(group_max<16>(v))); }
// 64-bit max (selection keys) keeps the generic shuffle path (rare, end of kernels).
__device__ __forceinline__ unsigned long long wave_max(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long t = __shfl_xor(v, o, 64);
        v = t > v ? t : v;
    }
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

// Per-sequence RoPE row of the current decode position (engine-owned, see DecodeAttnParams::rc):
// float [B][rope_cur_stride(hd)] = {tag (the position, int bits), 7 pad, cos[hd / 2], sin[hd / 2]}
__host__ __device__ constexpr int rope_cur_stride(int hd) { return 8 + hd; }
// the decode attention launches of this host thread read this table (null: none)
void set_decode_rope_cur(const float* rc);

// Peer-backend tagged exchange (comm.hip): rank r's partial of generation e sits in every
// rank's buffer at tagged slot [e & 1][r] as 8-byte words {tag = e + 1, f32 value}, so a
// reader polls the data itself (no flag, no release fence: each word is one atomic store).
constexpr int64_t kPeerTagCap = 1 << 20;   // bytes per tagged (parity, rank) slot
constexpr int kPeerTagMaxWorld = 8;
// What a producer kernel needs to push its fp32 outputs straight into the tagged slots.
struct PeerPush {
    char* tb[kPeerTagMaxWorld];   // every rank's tagged region base
    const unsigned* gen;          // this rank's generation word
    int world, rank;
};
__device__ __forceinline__ uint64_t* peer_tag_slot(char* tb, unsigned e, int src) {
    return reinterpret_cast<uint64_t*>(tb + (int64_t)((e & 1) * kPeerTagMaxWorld + src) * kPeerTagCap);
}
// The M = 1 GEMV launches of this host thread push their F32-epilogue outputs (null: none);
// gemv_push_taken() reports whether the last launch did.
void set_gemv_push(const PeerPush* pp);
bool gemv_push_taken();

// Device properties cached per process (CU count for persistent grids).
int device_cu_count();

}  // namespace qie
