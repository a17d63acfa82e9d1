// k_misc.hip — error plumbing, embedding gather, row RMSNorm, q/k post-projection
// (qk-norm + RoPE + KV append), elementwise ops, synthetic weight fill.
//
// Reference kernels restated for gfx950 (wave64, 16-byte vector accesses):
//   embedding_matrix_func  layers/src/embedded_matrix.cu:5-17
//   rmsNorm                layers/src/normalization.cu:5-25
//   qkNorm                 layers/src/qk_norm.cu:43-79
//   RoPE                   layers/src/RoPE.cu:6-22
//   activation/element_mul layers/src/SiLU.cu:10-23, element_add.cu:4-12
//   residual_add           layers/src/residual_add.cu:7-18
//   kv_copy_layer_to_cache_{prefill,decode} layers/src/include_cuda.cu:165-279
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

#include <cmath>
#include <cstdarg>
#include <cstring>
#include <mutex>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace qie {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int device_cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
            cus[dev] = prop.multiProcessorCount;
        else
            cus[dev] = 256;
    }
    return cus[dev];
}

// ------------------------------------------------------------ embedding
// One block per token row, 16-byte copies (the reference copies one bf16 at a
// time from pinned host memory with one thread per row).
__global__ __launch_bounds__(256) void embedding_kernel(const uint4* __restrict__ E,
                                                        const int32_t* __restrict__ ids,
                                                        uint4* __restrict__ out, int64_t H8) {
    const int64_t t = blockIdx.x;
    const int64_t row = ids[t];
    const uint4* src = E + row * H8;
    uint4* dst = out + t * H8;
    for (int64_t i = threadIdx.x; i < H8; i += blockDim.x) dst[i] = src[i];
}

// ------------------------------------------------------------- RMSNorm
// Block per row; fp32 sum of squares (wave butterfly + LDS), then
//   REF: y = bf16((x / sqrtf(ss/H + eps)) * w)          normalization.cu:5-25
//   HF : y = bf16(w * bf16(x * (1/sqrtf(ss/H + eps))))
__device__ __forceinline__ float block_sum_256(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}

__device__ __forceinline__ uint4 rms_apply8(uint4 xv, uint4 wv, float rms, float inv, int numerics) {
#pragma clang fp contract(off)
    uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w};
    uint32_t ws[4] = {wv.x, wv.y, wv.z, wv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        float a0 = bf_lo(xs[j]), a1 = bf_hi(xs[j]);
        float w0 = bf_lo(ws[j]), w1 = bf_hi(ws[j]);
        float y0, y1;
        if (numerics == QIE_NUMERICS_HF) {
            y0 = w0 * rbf(a0 * inv);
            y1 = w1 * rbf(a1 * inv);
        } else {
            y0 = (a0 / rms) * w0;
            y1 = (a1 / rms) * w1;
        }
        o[j] = pack2(y0, y1);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__global__ __launch_bounds__(256) void rmsnorm_kernel(const uint4* __restrict__ x,
                                                      const uint4* __restrict__ w,
                                                      uint4* __restrict__ y, int64_t H, float eps,
                                                      int numerics) {
    __shared__ float red[4];
    const int64_t H8 = H / 8;
    const uint4* xr = x + blockIdx.x * H8;
    uint4* yr = y + blockIdx.x * H8;
    float ss = 0.f;
    for (int64_t i = threadIdx.x; i < H8; i += 256) {
        uint4 v = xr[i];
        uint32_t a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float l = bf_lo(a[j]), h = bf_hi(a[j]);
            ss += l * l + h * h;
        }
    }
    ss = block_sum_256(ss, red);
    const float rms = sqrtf((ss / (float)H) + eps);
    const float inv = 1.0f / rms;
    for (int64_t i = threadIdx.x; i < H8; i += 256) yr[i] = rms_apply8(xr[i], w[i], rms, inv, numerics);
}

// H <= 2048 V: the row and the norm weights stay in registers, both loaded up front (one
// round trip instead of the loop form's two; the batched decode runs it twice per layer)
template <int V>
__global__ __launch_bounds__(256) void rmsnorm_reg_kernel(const uint4* __restrict__ x, const uint4* __restrict__ w,
                                                          uint4* __restrict__ y, int64_t H, float eps, int numerics) {
    __shared__ float red[4];
    const int64_t H8 = H / 8;
    const uint4* xr = x + blockIdx.x * H8;
    uint4* yr = y + blockIdx.x * H8;
    uint4 xv[V], wv[V];
#pragma unroll
    for (int c = 0; c < V; c++) {
        const int64_t i = threadIdx.x + 256 * c;
        const int64_t ic = i < H8 ? i : H8 - 1;   // clamped: loads stay unconditional
        xv[c] = xr[ic];
        wv[c] = w[ic];
    }
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < V; c++) {
        if (threadIdx.x + 256 * c >= H8) continue;
        const uint32_t a[4] = {xv[c].x, xv[c].y, xv[c].z, xv[c].w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float l = bf_lo(a[j]), h = bf_hi(a[j]);
            ss += l * l + h * h;
        }
    }
    ss = block_sum_256(ss, red);
    const float rms = sqrtf((ss / (float)H) + eps);
    const float inv = 1.0f / rms;
#pragma unroll
    for (int c = 0; c < V; c++) {
        const int64_t i = threadIdx.x + 256 * c;
        if (i < H8) yr[i] = rms_apply8(xv[c], wv[c], rms, inv, numerics);
    }
}

// ------------------------------------------- q/k post-projection + KV append
// Block per row, one wave per head.  Each lane owns one RoPE pair:
//   REF: (2*lane, 2*lane+1) interleaved (RoPE.cu:12-18)
//   HF : (lane, lane + hd/2) rotate_half
// qk-norm (Qwen3 only) is the per-head RMSNorm of qk_norm.cu:43-79.
struct QkvPostArgs {
    const uint16_t* qkv;
    const int32_t* pos;
    int rows_per_seq;
    const uint16_t* q_norm;
    const uint16_t* k_norm;
    const float* cs;
    const float* sn;
    int nq, nkv, hd;
    uint16_t* kc;
    uint16_t* vc;
    KvMap km;
    int layer;
    float eps;
    int numerics;
    uint16_t* q_out;
};

// Round 6: the wave's heads are taken in batches of kQkvBatch whose source pairs are all
// loaded before the first store (the row-at-a-time form waited one memory round trip per head,
// nine in a row per wave at Qwen2-7B widths); the arithmetic per element is unchanged.
constexpr int kQkvBatch = 10;

template <bool PG, bool HF>
__global__ __launch_bounds__(256) void qkv_post_kernel(QkvPostArgs a) {
#pragma clang fp contract(off)
    const int64_t m = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int hd = a.hd, half = hd / 2;
    const int QD = a.nq * hd, KD = a.nkv * hd;
    const int ptot = a.nq + 2 * a.nkv;
    const int p = a.pos[m];
    const int64_t seq = m / a.rows_per_seq;
    const uint16_t* row = a.qkv + m * (int64_t)(QD + 2 * KD);
    const bool active = lane < half;
    const int i0 = HF ? lane : 2 * lane;
    const int i1 = HF ? lane + half : 2 * lane + 1;
    const float c = active ? a.cs[(int64_t)p * half + lane] : 0.f;
    const float s = active ? a.sn[(int64_t)p * half + lane] : 0.f;
    // q, k and v heads are contiguous in the projection row: head h starts at h * hd
    for (int h0 = wave; h0 < ptot; h0 += 4 * kQkvBatch) {
        uint32_t raw[kQkvBatch];   // the lane's pair of head h0 + 4 b: element i0 low, i1 high
#pragma unroll
        for (int b = 0; b < kQkvBatch; b++) {
            const int h = h0 + 4 * b;
            raw[b] = 0;
            if (h < ptot && active) {
                const uint16_t* src = row + h * hd;
                raw[b] = HF ? (uint32_t)src[i0] | ((uint32_t)src[i1] << 16)
                            : reinterpret_cast<const uint32_t*>(src)[lane];
            }
        }
#pragma unroll
        for (int b = 0; b < kQkvBatch; b++) {
            const int h = h0 + 4 * b;
            if (h >= ptot) break;   // wave-uniform
            uint16_t* dst;
            const uint16_t* nw = nullptr;
            bool rope = true;
            if (h < a.nq) {
                dst = a.q_out + m * (int64_t)QD + h * hd;
                nw = a.q_norm;
            } else if (h < a.nq + a.nkv) {
                const int g = h - a.nq;
                dst = a.kc + kv_run_off(a.km, (int64_t)a.layer * a.nkv + g, hd) + kv_tok<PG>(a.km, seq, p, hd);
                nw = a.k_norm;
            } else {
                const int g = h - a.nq - a.nkv;
                dst = a.vc + kv_run_off(a.km, (int64_t)a.layer * a.nkv + g, hd) + kv_tok<PG>(a.km, seq, p, hd);
                rope = false;
            }
            float x0 = active ? bf2f((uint16_t)(raw[b] & 0xffffu)) : 0.f;
            float x1 = active ? bf2f((uint16_t)(raw[b] >> 16)) : 0.f;
            if (rope && nw) {
                float ss = wave_sum(x0 * x0 + x1 * x1);
                float rms = sqrtf((ss / (float)hd) + a.eps);
                if (HF) {
                    float inv = 1.0f / rms;
                    x0 = rbf(bf2f(nw[i0]) * rbf(x0 * inv));
                    x1 = rbf(bf2f(nw[i1]) * rbf(x1 * inv));
                } else {
                    x0 = rbf((x0 / rms) * bf2f(nw[i0]));
                    x1 = rbf((x1 / rms) * bf2f(nw[i1]));
                }
            }
            float y0 = x0, y1 = x1;
            if (rope) {
                if (HF) {
                    y0 = rbf(rbf(x0 * c) + rbf(-x1 * s));
                    y1 = rbf(rbf(x1 * c) + rbf(x0 * s));
                } else {
                    y0 = x0 * c - x1 * s;
                    y1 = x1 * c + x0 * s;
                }
            }
            if (active) {
                if (HF) {
                    dst[i0] = f2bf(y0);
                    dst[i1] = f2bf(y1);
                } else {
                    reinterpret_cast<uint32_t*>(dst)[lane] = pack2(y0, y1);
                }
            }
        }
    }
}

// ------------------------------------------- standalone per-head ops (operator tier)
// qie_qknorm / qie_rope: the reference's separate in-place launches (launch_qknorm,
// launch_rope, launch_rope_single; helpers.cuh:51-55,140-147) for hosts that keep the
// reference layer loop.  Block per row, one wave per head (looped), one lane per pair.
//   qk-norm: lane l owns elements (l, l + hd/2); its x_l^2 + x_{l+hd/2}^2 is the
//     reference's shared-memory tree after the stride-hd/2 step (qk_norm.cu:59-66), the
//     xor butterfly 32..1 then reproduces the remaining strides, and lane 0's sum (the
//     tree's buf[0]) is broadcast — the reference's exact summation order.
//   RoPE: REF interleaved pairs (2l, 2l+1) (RoPE.cu:12-18), HF rotate_half (l, l+hd/2);
//     row r at position pos[r] (pos != NULL) or pos0 + r.
struct HeadOpArgs {
    uint16_t* x;
    int64_t row_stride;
    int nheads, hd;
    const uint16_t* w;
    float eps;
    const float* cs;
    const float* sn;
    const int32_t* pos;
    int pos0;
    int numerics;
    int rope;   // 0: qk-norm, 1: RoPE
};

__device__ __forceinline__ float tree_sum64(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return __shfl(v, 0, 64);
}

__global__ __launch_bounds__(256) void head_op_kernel(HeadOpArgs a) {
#pragma clang fp contract(off)
    const int64_t r = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int hd = a.hd, half = hd / 2;
    const bool hf = a.numerics == QIE_NUMERICS_HF;
    const bool active = lane < half;
    const bool pair_split = hf || !a.rope;   // (l, l + half) pairs
    const int i0 = pair_split ? lane : 2 * lane;
    const int i1 = pair_split ? lane + half : 2 * lane + 1;
    float c = 0.f, s = 0.f;
    if (a.rope && active) {
        const int64_t p = a.pos ? a.pos[r] : (int64_t)a.pos0 + r;
        c = a.cs[p * half + lane];
        s = a.sn[p * half + lane];
    }
    for (int h = wave; h < a.nheads; h += 4) {
        uint16_t* v = a.x + r * a.row_stride + (int64_t)h * hd;
        float x0 = active ? bf2f(v[i0]) : 0.f;
        float x1 = active ? bf2f(v[i1]) : 0.f;
        float y0, y1;
        if (!a.rope) {
            const float rms = sqrtf((tree_sum64(x0 * x0 + x1 * x1) / (float)hd) + a.eps);
            if (hf) {
                const float inv = 1.0f / rms;
                y0 = bf2f(a.w[i0]) * rbf(x0 * inv);
                y1 = bf2f(a.w[i1]) * rbf(x1 * inv);
            } else {
                y0 = (x0 / rms) * bf2f(a.w[i0]);
                y1 = (x1 / rms) * bf2f(a.w[i1]);
            }
        } else if (hf) {
            y0 = rbf(rbf(x0 * c) + rbf(-x1 * s));
            y1 = rbf(rbf(x1 * c) + rbf(x0 * s));
        } else {
            y0 = x0 * c - x1 * s;
            y1 = x1 * c + x0 * s;
        }
        if (active) {
            v[i0] = f2bf(y0);
            v[i1] = f2bf(y1);
        }
    }
}

// K/V rows [rows][nkv * hd] (row stride ld) -> cache positions pos0 + r of sequence `seq`
// (kv_copy_layer_to_cache_prefill / _decode, include_cuda.cu:165-279).  Block per row,
// one 16-byte chunk per thread.
template <bool PG>
__global__ __launch_bounds__(256) void kv_write_kernel(const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
                                                       int64_t ld, int pos0, uint16_t* kc, uint16_t* vc, KvMap km,
                                                       int seq, int layer, int nkv, int hd) {
    const int64_t r = blockIdx.x;
    const int p = pos0 + (int)r;
    const int cph = hd / 8;
    for (int i = threadIdx.x; i < 2 * nkv * cph; i += 256) {
        const int which = i / (nkv * cph), j = i % (nkv * cph), g = j / cph, ch = j % cph;
        const uint16_t* src = (which ? v : k) + r * ld + g * hd + ch * 8;
        uint16_t* dst = (which ? vc : kc) + kv_run_off(km, (int64_t)layer * nkv + g, hd) + kv_tok<PG>(km, seq, p, hd) +
                        ch * 8;
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    }
}

// activation (SiLU.cu:10-23): x = bf16(x * (1 / (1 + expf(-x)))), in place
__global__ __launch_bounds__(256) void silu_kernel(uint4* __restrict__ x, int64_t n8) {
#pragma clang fp contract(off)
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const uint4 g = x[i];
        const uint32_t ga[4] = {g.x, g.y, g.z, g.w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float g0 = bf_lo(ga[j]), g1 = bf_hi(ga[j]);
            o[j] = pack2(g0 * (1.0f / (1.0f + expf(-g0))), g1 * (1.0f / (1.0f + expf(-g1))));
        }
        x[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// element_mul (element_add.cu:4-12): c = bf16(a * b)
__global__ __launch_bounds__(256) void mul_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                  uint4* __restrict__ c, int64_t n8) {
#pragma clang fp contract(off)
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const uint4 x = a[i], y = b[i];
        const uint32_t aa[4] = {x.x, x.y, x.z, x.w}, bb[4] = {y.x, y.y, y.z, y.w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = pack2(bf_lo(aa[j]) * bf_lo(bb[j]), bf_hi(aa[j]) * bf_hi(bb[j]));
        c[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// ----------------------------------------------------------- elementwise
__global__ __launch_bounds__(256) void silu_mul_kernel(const uint4* __restrict__ g,
                                                       const uint4* __restrict__ u,
                                                       uint4* __restrict__ h, int64_t n8) {
#pragma clang fp contract(off)
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        uint4 gv = g[i], uv = u[i];
        uint32_t ga[4] = {gv.x, gv.y, gv.z, gv.w}, ua[4] = {uv.x, uv.y, uv.z, uv.w}, o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float g0 = bf_lo(ga[j]), g1 = bf_hi(ga[j]);
            float a0 = rbf(g0 * (1.0f / (1.0f + expf(-g0))));
            float a1 = rbf(g1 * (1.0f / (1.0f + expf(-g1))));
            o[j] = pack2(bf_lo(ua[j]) * a0, bf_hi(ua[j]) * a1);
        }
        h[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

__global__ __launch_bounds__(256) void resadd_kernel(uint4* __restrict__ x, const uint4* __restrict__ y,
                                                     int64_t n8) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        uint4 a = x[i], b = y[i];
        uint32_t aa[4] = {a.x, a.y, a.z, a.w}, bb[4] = {b.x, b.y, b.z, b.w}, o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = pack2(bf_lo(aa[j]) + bf_lo(bb[j]), bf_hi(aa[j]) + bf_hi(bb[j]));
        x[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// x = bf16(x + bf16(sum)): tensor-parallel residual after the fp32 all-reduce
__global__ __launch_bounds__(256) void resadd_f32_kernel(uint4* __restrict__ x, const float4* __restrict__ s,
                                                         int64_t n8) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const uint4 a = x[i];
        const float4 s0 = s[2 * i], s1 = s[2 * i + 1];
        const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const uint32_t aa[4] = {a.x, a.y, a.z, a.w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            o[j] = pack2(bf_lo(aa[j]) + rbf(sv[2 * j]), bf_hi(aa[j]) + rbf(sv[2 * j + 1]));
        x[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// ------------------------------------------------------ synthetic weights
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t synth_base(uint32_t tensor_id, uint64_t seed) {
    return splitmix64((seed * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)tensor_id << 32));
}

__host__ __device__ __forceinline__ float synth_value(uint64_t base, int64_t i, float scale,
                                                      float offset) {
    uint64_t r = splitmix64(base + (uint64_t)i);
    float u = (float)((int32_t)(r >> 40) - 8388608) * (1.0f / 8388608.0f);
    return offset + u * scale;
}

__global__ __launch_bounds__(256) void synth_kernel(uint32_t* __restrict__ out, int64_t n2,
                                                    uint64_t base, float scale, float offset,
                                                    int64_t n) {
#pragma clang fp contract(off)
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        float a = synth_value(base, 2 * i, scale, offset);
        float b = (2 * i + 1 < n) ? synth_value(base, 2 * i + 1, scale, offset) : 0.f;
        out[i] = pack2(a, b);
    }
}

// ------------------------------------------------------ fp8 weight quantisation
// One block per weight row: amax -> power-of-two scale -> e4m3 codes (qie_common.hpp).
__global__ __launch_bounds__(256) void quantize_fp8_kernel(const uint16_t* __restrict__ w, int64_t cols,
                                                           uint8_t* __restrict__ codes, float* __restrict__ scales) {
    __shared__ float red[4];
    const int64_t r = blockIdx.x;
    const uint16_t* row = w + r * cols;
    float amax = 0.f;
    for (int64_t c = threadIdx.x; c < cols; c += 256) amax = fmaxf(amax, fabsf(bf2f(row[c])));
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s = e4m3_row_scale(amax);
    for (int64_t c = threadIdx.x; c < cols; c += 256) codes[r * cols + c] = e4m3_encode(bf2f(row[c]) / s);
    if (threadIdx.x == 0) scales[r] = s;
}

__global__ void fp8_decode_probe_kernel(float* out) {
    const uint32_t b = threadIdx.x;   // 64 threads x 4 codes
    float f[4];
    fp8x4_to_f32((4 * b) | ((4 * b + 1) << 8) | ((4 * b + 2) << 16) | ((4 * b + 3) << 24), f);
    for (int j = 0; j < 4; j++) out[4 * b + j] = f[j];
}

__global__ void fp8_decode_bf16_probe_kernel(uint16_t* out) {
    const uint32_t b = threadIdx.x;   // 64 threads x 4 codes, through the MFMA GEMV's decode
    const uint2 v = fp8x4_to_bf16x4((4 * b) | ((4 * b + 1) << 8) | ((4 * b + 2) << 16) | ((4 * b + 3) << 24));
    out[4 * b] = (uint16_t)(v.x & 0xffff);
    out[4 * b + 1] = (uint16_t)(v.x >> 16);
    out[4 * b + 2] = (uint16_t)(v.y & 0xffff);
    out[4 * b + 3] = (uint16_t)(v.y >> 16);
}

__global__ __launch_bounds__(256) void synth_slice_kernel(uint16_t* __restrict__ out, int64_t rows, int64_t cols,
                                                          int64_t full_cols, int64_t row0, int64_t col0,
                                                          uint64_t base, float scale, float offset) {
#pragma clang fp contract(off)
    const int64_t n = rows * cols;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols, c = i % cols;
        out[i] = f2bf(synth_value(base, (row0 + r) * full_cols + col0 + c, scale, offset));
    }
}

// rows r of a [rows][cols] bf16 matrix with (row0 + r) % every == 0 times 2^log2f (exact
// while the result stays finite): the synthetic "peaked head" of the parity runs
__global__ __launch_bounds__(256) void scale_rows_pow2_kernel(uint16_t* __restrict__ w, int64_t rows, int64_t cols,
                                                              int64_t row0, int64_t every, float f) {
    const int64_t nsel = (row0 + rows + every - 1) / every - (row0 + every - 1) / every;
    const int64_t first = (row0 + every - 1) / every * every - row0;
    const int64_t n = nsel * cols;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t r = first + (i / cols) * every, c = i % cols;
        w[r * cols + c] = f2bf(bf2f(w[r * cols + c]) * f);
    }
}

static inline uint16_t host_f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)0x7fff;
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

}  // namespace qie

using namespace qie;

namespace qie {
int kv_map_make(const qie_kv_cache* c, KvMap* out, const char* who) {
    QIE_REQUIRE(c && c->k && c->v && c->n_layers > 0 && c->n_kv_heads > 0 && c->head_dim > 0 && c->max_ctx > 0,
                "%s: bad KV cache descriptor", who);
    const int64_t lh = (int64_t)c->n_layers * c->n_kv_heads * c->head_dim;
    KvMap m{};
    if (c->block_table) {
        const int T = c->page_tokens;
        QIE_REQUIRE(T >= 128 && (T & (T - 1)) == 0, "%s: page_tokens %d must be a power of two >= 128", who, T);
        QIE_REQUIRE(c->max_pages >= (c->max_ctx + T - 1) / T, "%s: max_pages %d < ceil(max_ctx %d / %d)", who,
                    c->max_pages, c->max_ctx, T);
        QIE_REQUIRE(c->seq_stride >= lh * T, "%s: page stride %lld < one page", who, (long long)c->seq_stride);
        m.table = c->block_table;
        m.run = T;
        m.shift = __builtin_ctz((unsigned)T);
        m.max_pages = c->max_pages;
    } else {
        m.table = nullptr;
        m.run = c->max_ctx;
        m.shift = 0;
        m.max_pages = 0;
    }
    m.stride = c->seq_stride;
    *out = m;
    return 0;
}
}  // namespace qie

extern "C" {

const char* qie_last_error(void) { return g_last_error.c_str(); }
int qie_abi_version(void) { return QIE_ABI_VERSION; }

int qie_device_count(int* count) {
    QIE_HIP(hipGetDeviceCount(count));
    return 0;
}

int qie_set_device(int device) {
    QIE_HIP(hipSetDevice(device));
    return 0;
}

int qie_malloc(void** ptr, int64_t bytes) {
    QIE_REQUIRE(ptr && bytes >= 0, "qie_malloc: bad arguments");
    QIE_HIP(hipMalloc(ptr, bytes < 16 ? 16 : (size_t)bytes));
    return 0;
}

int qie_free(void* ptr) {
    if (ptr) QIE_HIP(hipFree(ptr));
    return 0;
}

// The stream-less helpers are complete on return: the engine's and the callers' streams are
// non-blocking, so a copy or memset left on the legacy null stream would not be ordered
// before their kernels.
int qie_memcpy_h2d(void* dst, const void* src, int64_t bytes) {
    QIE_HIP(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyHostToDevice));
    QIE_HIP(hipStreamSynchronize(nullptr));
    return 0;
}

int qie_memcpy_d2h(void* dst, const void* src, int64_t bytes) {
    QIE_HIP(hipDeviceSynchronize());
    QIE_HIP(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
    return 0;
}

int qie_memset(void* ptr, int value, int64_t bytes) {
    QIE_HIP(hipMemset(ptr, value, (size_t)bytes));
    QIE_HIP(hipStreamSynchronize(nullptr));
    return 0;
}

int qie_synchronize(void) {
    QIE_HIP(hipDeviceSynchronize());
    return 0;
}

int qie_stream_create(void** stream_out) {
    QIE_REQUIRE(stream_out, "qie_stream_create: null output");
    hipStream_t st = nullptr;
    QIE_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *stream_out = st;
    return 0;
}

int qie_stream_synchronize(void* stream) {
    QIE_HIP(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

int qie_stream_destroy(void* stream) {
    if (stream) QIE_HIP(hipStreamDestroy((hipStream_t)stream));
    return 0;
}

int qie_rope_table_host(float* cos_out, float* sin_out, int32_t n_pos, int32_t head_dim,
                        float theta, int32_t numerics) {
    QIE_REQUIRE(cos_out && sin_out && n_pos > 0 && head_dim > 0 && head_dim % 2 == 0,
                "qie_rope_table_host: bad arguments");
    const int half = head_dim / 2;
    if (numerics == QIE_NUMERICS_HF) {
        for (int i = 0; i < half; i++) {
            float ex = (float)(2 * i) / (float)head_dim;
            float inv = 1.0f / powf(theta, ex);
            for (int p = 0; p < n_pos; p++) {
                float fr = (float)p * inv;
                uint32_t cu = (uint32_t)host_f2bf(cosf(fr)) << 16, su = (uint32_t)host_f2bf(sinf(fr)) << 16;
                std::memcpy(&cos_out[(size_t)p * half + i], &cu, 4);
                std::memcpy(&sin_out[(size_t)p * half + i], &su, 4);
            }
        }
    } else {
        // precompute_cos_sin, layers/src/include.cpp:5-16 (float pow, int*float angle).
        for (int i = 0; i < half; i++) {
            float exponent = 2 * ((float)i / (float)head_dim);
            float th = std::pow(theta, -exponent);
            for (int p = 0; p < n_pos; p++) {
                cos_out[(size_t)p * half + i] = cosf(p * th);
                sin_out[(size_t)p * half + i] = sinf(p * th);
            }
        }
    }
    return 0;
}

int qie_embedding(const void* E, const int32_t* ids, void* out, int64_t n, int64_t H, void* stream) {
    QIE_REQUIRE(E && ids && out && n >= 0 && H > 0 && H % 8 == 0, "qie_embedding: bad arguments");
    if (n == 0) return 0;
    hipLaunchKernelGGL(embedding_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)E, ids, (uint4*)out, H / 8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_rmsnorm(const void* x, const void* w, void* y, int64_t rows, int64_t H, float eps,
                int32_t numerics, void* stream) {
    QIE_REQUIRE(x && w && y && rows >= 0 && H > 0 && H % 8 == 0 && x != y,
                "qie_rmsnorm: bad arguments");
    if (rows == 0) return 0;
    const int64_t v = (H / 8 + 255) / 256;   // 16-B vectors per thread
    auto fn = v <= 1 ? rmsnorm_reg_kernel<1> : v <= 2 ? rmsnorm_reg_kernel<2> : v <= 4 ? rmsnorm_reg_kernel<4>
                                                                                     : rmsnorm_kernel;
    hipLaunchKernelGGL(fn, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, (const uint4*)x, (const uint4*)w,
                       (uint4*)y, H, eps, numerics);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_qkv_post(const void* qkv, int64_t M, const int32_t* pos, int32_t rows_per_seq,
                 const void* q_norm, const void* k_norm, const float* rope_cos,
                 const float* rope_sin, int32_t n_heads, const qie_kv_cache* cache, int32_t layer,
                 float eps, int32_t numerics, void* q_out, void* stream) {
    QIE_REQUIRE(qkv && pos && cache && cache->k && cache->v && rope_cos && rope_sin && q_out &&
                    M >= 0 && rows_per_seq > 0 && n_heads > 0 && cache->n_kv_heads > 0 &&
                    n_heads % cache->n_kv_heads == 0 && layer >= 0 && layer < cache->n_layers,
                "qie_qkv_post: bad arguments");
    QIE_REQUIRE(cache->head_dim % 2 == 0 && cache->head_dim <= 128,
                "qie_qkv_post: head_dim must be even and <= 128");
    if (M == 0) return 0;
    QkvPostArgs a;
    a.qkv = (const uint16_t*)qkv;
    a.pos = pos;
    a.rows_per_seq = rows_per_seq;
    a.q_norm = (const uint16_t*)q_norm;
    a.k_norm = (const uint16_t*)k_norm;
    a.cs = rope_cos;
    a.sn = rope_sin;
    a.nq = n_heads;
    a.nkv = cache->n_kv_heads;
    a.hd = cache->head_dim;
    a.kc = (uint16_t*)cache->k;
    a.vc = (uint16_t*)cache->v;
    QIE_TRY(kv_map_make(cache, &a.km, "qie_qkv_post"));
    a.layer = layer;
    a.eps = eps;
    a.numerics = numerics;
    a.q_out = (uint16_t*)q_out;
    const bool hf = numerics == QIE_NUMERICS_HF;
    auto fn = a.km.table ? (hf ? qkv_post_kernel<true, true> : qkv_post_kernel<true, false>)
                         : (hf ? qkv_post_kernel<false, true> : qkv_post_kernel<false, false>);
    hipLaunchKernelGGL(fn, dim3((unsigned)M), dim3(256), 0, (hipStream_t)stream, a);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_memcpy_d2d(void* dst, const void* src, int64_t bytes, void* stream) {
    QIE_REQUIRE(dst && src && bytes >= 0, "qie_memcpy_d2d: bad arguments");
    if (bytes == 0) return 0;
    QIE_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

int qie_qknorm(void* x, int64_t rows, int64_t row_stride, int32_t n_heads, int32_t head_dim, const void* w,
               float eps, int32_t numerics, void* stream) {
    QIE_REQUIRE(w, "qie_qknorm: null weight");
    HeadOpArgs a{};
    a.x = (uint16_t*)x; a.row_stride = row_stride; a.nheads = n_heads; a.hd = head_dim;
    a.w = (const uint16_t*)w; a.eps = eps; a.numerics = numerics; a.rope = 0;
    QIE_REQUIRE(a.x && rows >= 0 && n_heads > 0 && head_dim > 0 && head_dim % 2 == 0 && head_dim <= 128 &&
                    row_stride >= (int64_t)n_heads * head_dim,
                "qie_qknorm: bad arguments (head_dim even and <= 128, row_stride >= n_heads * head_dim)");
    if (rows == 0) return 0;
    hipLaunchKernelGGL(head_op_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, a);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_rope(void* x, int64_t rows, int64_t row_stride, int32_t n_heads, int32_t head_dim, const int32_t* pos,
             int32_t pos0, const float* rope_cos, const float* rope_sin, int32_t numerics, void* stream) {
    QIE_REQUIRE(rope_cos && rope_sin && pos0 >= 0, "qie_rope: bad tables / position");
    HeadOpArgs a{};
    a.x = (uint16_t*)x; a.row_stride = row_stride; a.nheads = n_heads; a.hd = head_dim;
    a.cs = rope_cos; a.sn = rope_sin; a.pos = pos; a.pos0 = pos0; a.numerics = numerics; a.rope = 1;
    QIE_REQUIRE(a.x && rows >= 0 && n_heads > 0 && head_dim > 0 && head_dim % 2 == 0 && head_dim <= 128 &&
                    row_stride >= (int64_t)n_heads * head_dim,
                "qie_rope: bad arguments (head_dim even and <= 128, row_stride >= n_heads * head_dim)");
    if (rows == 0) return 0;
    hipLaunchKernelGGL(head_op_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, a);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_kv_write(const void* k, const void* v, int64_t rows, int64_t ld, int32_t pos0, const qie_kv_cache* cache,
                 int32_t seq, int32_t layer, void* stream) {
    QIE_REQUIRE(k && v && cache && rows >= 0 && pos0 >= 0 && seq >= 0 && layer >= 0 && layer < cache->n_layers,
                "qie_kv_write: bad arguments");
    QIE_REQUIRE(pos0 + rows <= cache->max_ctx, "qie_kv_write: positions %d..%lld exceed max_ctx %d", pos0,
                (long long)(pos0 + rows - 1), cache->max_ctx);
    QIE_REQUIRE(cache->head_dim % 8 == 0 && ld >= (int64_t)cache->n_kv_heads * cache->head_dim && ld % 8 == 0 &&
                    ((uintptr_t)k % 16) == 0 && ((uintptr_t)v % 16) == 0,
                "qie_kv_write: rows must be 16-byte aligned with ld >= n_kv_heads * head_dim, ld % 8 == 0");
    if (rows == 0) return 0;
    KvMap km;
    QIE_TRY(kv_map_make(cache, &km, "qie_kv_write"));
    hipLaunchKernelGGL((km.table ? kv_write_kernel<true> : kv_write_kernel<false>), dim3((unsigned)rows), dim3(256), 0,
                       (hipStream_t)stream, (const uint16_t*)k, (const uint16_t*)v, ld, pos0, (uint16_t*)cache->k,
                       (uint16_t*)cache->v, km, seq, layer, cache->n_kv_heads, cache->head_dim);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_silu(void* x, int64_t n, void* stream) {
    QIE_REQUIRE(x && n >= 0 && n % 8 == 0, "qie_silu: bad arguments (n % 8 == 0)");
    if (n == 0) return 0;
    const int64_t n8 = n / 8;
    hipLaunchKernelGGL(silu_kernel, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, (uint4*)x, n8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_mul(const void* a, const void* b, void* c, int64_t n, void* stream) {
    QIE_REQUIRE(a && b && c && n >= 0 && n % 8 == 0, "qie_mul: bad arguments (n % 8 == 0)");
    if (n == 0) return 0;
    const int64_t n8 = n / 8;
    hipLaunchKernelGGL(mul_kernel, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const uint4*)a, (const uint4*)b, (uint4*)c, n8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_silu_mul(const void* gate, const void* up, void* h, int64_t n, void* stream) {
    QIE_REQUIRE(gate && up && h && n >= 0 && n % 8 == 0, "qie_silu_mul: bad arguments");
    if (n == 0) return 0;
    int64_t n8 = n / 8;
    unsigned grid = (unsigned)std::min<int64_t>((n8 + 255) / 256, 8192);
    hipLaunchKernelGGL(silu_mul_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)gate, (const uint4*)up, (uint4*)h, n8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_residual_add(void* x, const void* y, int64_t n, void* stream) {
    QIE_REQUIRE(x && y && n >= 0 && n % 8 == 0, "qie_residual_add: bad arguments");
    if (n == 0) return 0;
    int64_t n8 = n / 8;
    unsigned grid = (unsigned)std::min<int64_t>((n8 + 255) / 256, 8192);
    hipLaunchKernelGGL(resadd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint4*)x,
                       (const uint4*)y, n8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_residual_add_f32(void* x, const float* sum, int64_t n, void* stream) {
    QIE_REQUIRE(x && sum && n >= 0 && n % 8 == 0 && ((uintptr_t)sum % 16) == 0,
                "qie_residual_add_f32: bad arguments");
    if (n == 0) return 0;
    const int64_t n8 = n / 8;
    const unsigned grid = (unsigned)std::min<int64_t>((n8 + 255) / 256, 8192);
    hipLaunchKernelGGL(resadd_f32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint4*)x,
                       (const float4*)sum, n8);
    QIE_LAUNCH_CHECK();
    return 0;
}

int64_t qie_fp8_weight_bytes(int64_t rows, int64_t cols) { return rows * cols + rows * 4; }

// Per-row activation quantisation (QIE_LINEAR_ACT_FP8): one block per row, amax pass then
// the code pass (the row's second read hits L2); codes by v_cvt_pk_fp8_f32 (round to nearest
// even; |x / s| <= 448 by the scale, so its saturation never acts) — checked bit for bit
// against the oracle's table restatement of e4m3 rounding (tests/test_gpu_fp8.py).
__global__ __launch_bounds__(256) void quantize_rows_fp8_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                                int64_t cols, uint8_t* __restrict__ q, int64_t ldq,
                                                                uint8_t* __restrict__ exps) {
    __shared__ float red[4];
    const int64_t r = blockIdx.x, c8 = cols / 8;
    const uint4* xr = reinterpret_cast<const uint4*>(x + r * ldx);
    float amax = 0.f;
    for (int64_t i = threadIdx.x; i < c8; i += 256) {
        const uint4 v = xr[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) amax = fmaxf(amax, fmaxf(fabsf(bf_lo(w[j])), fabsf(bf_hi(w[j]))));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s = e4m3_row_scale(amax);
    const float inv = 1.0f / s;   // exact: a power of two
    if (threadIdx.x == 0) exps[r] = (uint8_t)((__float_as_uint(s) >> 23) & 0xffu);
    uint2* qr = reinterpret_cast<uint2*>(q + r * ldq);
    for (int64_t i = threadIdx.x; i < c8; i += 256) {
        const uint4 v = xr[i];
        int lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf_lo(v.x) * inv, bf_hi(v.x) * inv, 0, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf_lo(v.y) * inv, bf_hi(v.y) * inv, lo, true);
        int hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf_lo(v.z) * inv, bf_hi(v.z) * inv, 0, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf_lo(v.w) * inv, bf_hi(v.w) * inv, hi, true);
        qr[i] = make_uint2((uint32_t)lo, (uint32_t)hi);
    }
}

int qie_quantize_rows_fp8(const void* x, int64_t ldx, int64_t rows, int64_t cols, void* q, int64_t ldq, void* exps,
                          void* stream) {
    QIE_REQUIRE(x && q && exps && rows >= 0 && cols > 0 && cols % 8 == 0 && ldx >= cols && ldx % 8 == 0 &&
                    ldq >= cols && ldq % 16 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)q % 16) == 0,
                "qie_quantize_rows_fp8: bad arguments (cols %% 8, ldx %% 8, ldq %% 16, 16-B aligned buffers)");
    if (rows == 0) return 0;
    hipLaunchKernelGGL(quantize_rows_fp8_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)x, ldx, cols, (uint8_t*)q, ldq, (uint8_t*)exps);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_quantize_fp8(const void* w_bf16, int64_t rows, int64_t cols, void* out, void* stream) {
    QIE_REQUIRE(w_bf16 && out && rows > 0 && cols > 0 && cols % 16 == 0 && ((uintptr_t)out % 16) == 0,
                "qie_quantize_fp8: bad arguments (cols must be a multiple of 16, out 16-B aligned)");
    uint8_t* codes = (uint8_t*)out;
    hipLaunchKernelGGL(quantize_fp8_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)w_bf16, cols, codes, (float*)(codes + rows * cols));
    QIE_LAUNCH_CHECK();
    return 0;
}

// fp8 weight -> bf16 rows (exact: e4m3 value x power-of-two scale has <= 4 significant
// bits).  One thread per 16 codes, grid-stride; 16-B loads, 2 x 16-B stores.
__global__ void dequantize_fp8_kernel(const uint4* codes, const float* scales, int64_t cols16, int64_t n16,
                                      uint4* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 q = codes[i];
        const float sc = scales[i / cols16];
        float f[16];
        fp8x4_to_f32(q.x, f);
        fp8x4_to_f32(q.y, f + 4);
        fp8x4_to_f32(q.z, f + 8);
        fp8x4_to_f32(q.w, f + 12);
        out[2 * i] = make_uint4(pack2(f[0] * sc, f[1] * sc), pack2(f[2] * sc, f[3] * sc), pack2(f[4] * sc, f[5] * sc),
                                pack2(f[6] * sc, f[7] * sc));
        out[2 * i + 1] = make_uint4(pack2(f[8] * sc, f[9] * sc), pack2(f[10] * sc, f[11] * sc),
                                    pack2(f[12] * sc, f[13] * sc), pack2(f[14] * sc, f[15] * sc));
    }
}

int qie_dequantize_fp8(const void* w_fp8, int64_t rows, int64_t cols, void* out_bf16, void* stream) {
    QIE_REQUIRE(w_fp8 && out_bf16 && rows > 0 && cols > 0 && cols % 16 == 0 && ((uintptr_t)w_fp8 % 16) == 0 &&
                    ((uintptr_t)out_bf16 % 16) == 0,
                "qie_dequantize_fp8: bad arguments (cols % 16 == 0, 16-B aligned buffers)");
    const uint8_t* codes = (const uint8_t*)w_fp8;
    const int64_t n16 = rows * cols / 16;
    const unsigned grid = (unsigned)std::min<int64_t>((n16 + 255) / 256, (int64_t)device_cu_count() * 16);
    hipLaunchKernelGGL(dequantize_fp8_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)codes,
                       (const float*)(codes + rows * cols), cols / 16, n16, (uint4*)out_bf16);
    QIE_LAUNCH_CHECK();
    return 0;
}

// plain [rows][cols] fp8 codes -> the 16-row tiled layout (qie_ops.h); one thread per 16-B
// piece of the output: output piece (t, j, l) <- row 16 t + l % 16, columns 64 j + 16 (l / 16)
__global__ __launch_bounds__(256) void fp8_tile16_kernel(const uint4* in, int64_t cols16, int64_t units,
                                                         int64_t n16, uint4* out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const int64_t l = i & 63, blk = i >> 6;
        const int64_t t = blk / units, j = blk % units;
        const int64_t row = 16 * t + (l & 15);
        out[i] = in[row * cols16 + 4 * j + (l >> 4)];
    }
}

int qie_fp8_tile16(const void* w_fp8, int64_t rows, int64_t cols, void* out, void* stream) {
    QIE_REQUIRE(w_fp8 && out && w_fp8 != out && rows > 0 && rows % 16 == 0 && cols > 0 && cols % 64 == 0 &&
                    ((uintptr_t)w_fp8 % 16) == 0 && ((uintptr_t)out % 16) == 0,
                "qie_fp8_tile16: bad arguments (rows %% 16 == 0, cols %% 64 == 0, distinct 16-B aligned buffers)");
    const int64_t n16 = rows * cols / 16;
    const unsigned grid = (unsigned)std::min<int64_t>((n16 + 255) / 256, (int64_t)device_cu_count() * 16);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(fp8_tile16_kernel, dim3(grid), dim3(256), 0, st, (const uint4*)w_fp8, cols / 16, cols / 64, n16,
                       (uint4*)out);
    QIE_LAUNCH_CHECK();
    // the row scales are unchanged
    QIE_HIP(hipMemcpyAsync((uint8_t*)out + rows * cols, (const uint8_t*)w_fp8 + rows * cols, (size_t)rows * 4,
                           hipMemcpyDeviceToDevice, st));
    return 0;
}

int qie_quantize_fp8_host(const void* w_bf16, int64_t rows, int64_t cols, void* out) {
    QIE_REQUIRE(w_bf16 && out && rows > 0 && cols > 0 && cols % 16 == 0, "qie_quantize_fp8_host: bad arguments");
    const uint16_t* w = (const uint16_t*)w_bf16;
    uint8_t* codes = (uint8_t*)out;
    float* scales = (float*)(codes + rows * cols);
    auto h2f = [](uint16_t h) {
        uint32_t u = (uint32_t)h << 16;
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    };
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows; r++) {
        float amax = 0.f;
        for (int64_t c = 0; c < cols; c++) amax = std::max(amax, std::fabs(h2f(w[r * cols + c])));
        const float s = e4m3_row_scale(amax);
        for (int64_t c = 0; c < cols; c++) codes[r * cols + c] = e4m3_encode(h2f(w[r * cols + c]) / s);
        scales[r] = s;
    }
    return 0;
}

int qie_debug_fp8_decode(float* out_dev) {
    QIE_REQUIRE(out_dev, "qie_debug_fp8_decode: null output");
    hipLaunchKernelGGL(fp8_decode_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)0, out_dev);
    QIE_LAUNCH_CHECK();
    QIE_HIP(hipDeviceSynchronize());
    return 0;
}

int qie_debug_fp8_decode_bf16(uint16_t* out_dev) {
    QIE_REQUIRE(out_dev, "qie_debug_fp8_decode_bf16: null output");
    hipLaunchKernelGGL(fp8_decode_bf16_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)0, out_dev);
    QIE_LAUNCH_CHECK();
    QIE_HIP(hipDeviceSynchronize());
    return 0;
}

int qie_synthetic_fill_slice(void* dev, int64_t rows, int64_t cols, int64_t full_cols, int64_t row0,
                             int64_t col0, uint32_t tensor_id, uint64_t seed, float scale, float offset,
                             void* stream) {
    QIE_REQUIRE(dev && rows >= 0 && cols >= 0 && row0 >= 0 && col0 >= 0 && col0 + cols <= full_cols,
                "qie_synthetic_fill_slice: bad arguments");
    const int64_t n = rows * cols;
    if (n == 0) return 0;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(synth_slice_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint16_t*)dev, rows,
                       cols, full_cols, row0, col0, synth_base(tensor_id, seed), scale, offset);
    QIE_LAUNCH_CHECK();
    return 0;
}

uint32_t qie_tensor_id(const char* name) {
    uint32_t h = 2166136261u;
    for (const unsigned char* p = (const unsigned char*)name; *p; ++p) {
        h ^= *p;
        h *= 16777619u;
    }
    return h;
}

int qie_synthetic_fill(void* dev, int64_t n, uint32_t tensor_id, uint64_t seed, float scale,
                       float offset, void* stream) {
    QIE_REQUIRE(dev && n >= 0 && ((uintptr_t)dev % 4) == 0, "qie_synthetic_fill: bad arguments");
    if (n == 0) return 0;
    QIE_REQUIRE(n % 2 == 0, "qie_synthetic_fill: n must be even");
    int64_t n2 = n / 2;
    unsigned grid = (unsigned)std::min<int64_t>((n2 + 255) / 256, 16384);
    hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint32_t*)dev,
                       n2, synth_base(tensor_id, seed), scale, offset, n);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_scale_rows_pow2(void* w, int64_t rows, int64_t cols, int64_t row0, int64_t every, int32_t log2f,
                        void* stream) {
    QIE_REQUIRE(w && rows >= 0 && cols > 0 && row0 >= 0 && every > 0 && log2f >= -32 && log2f <= 32,
                "qie_scale_rows_pow2: bad arguments");
    const int64_t nsel = (row0 + rows + every - 1) / every - (row0 + every - 1) / every;
    if (nsel <= 0 || log2f == 0) return 0;
    const unsigned grid = (unsigned)std::min<int64_t>((nsel * cols + 255) / 256, 4096);
    hipLaunchKernelGGL(scale_rows_pow2_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint16_t*)w, rows, cols,
                       row0, every, ldexpf(1.0f, log2f));
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_synthetic_fill_host(void* host, int64_t n, uint32_t tensor_id, uint64_t seed, float scale,
                            float offset) {
    QIE_REQUIRE(host && n >= 0, "qie_synthetic_fill_host: bad arguments");
    uint16_t* out = (uint16_t*)host;
    const uint64_t base = synth_base(tensor_id, seed);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
#pragma clang fp contract(off)
        out[i] = host_f2bf(synth_value(base, i, scale, offset));
    }
    return 0;
}

}  // extern "C"
