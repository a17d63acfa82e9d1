// k_gemv.hip — bandwidth-bound skinny GEMM (M <= 8 rows) for the decode step.
//
// Replaces matrix_mul (layers/src/matrix_mul.cu:165-288) at M = 1 / small M,
// where the reference runs 16x16 WMMA tiles with 15 of 16 rows wasted and
// 2-byte loads.  Here (gfx950, wave64):
//   * each wave owns RPW weight rows and streams them along K with 16-byte
//     non-temporal loads (64 lanes x 16 B = 1 KiB per wave-instruction),
//     U chunks in flight per row;
//   * the activation rows live in LDS (optionally produced by a fused RMSNorm
//     prologue — the reference's launch_rms + proj pair in one launch);
//   * fp32 accumulation, wave butterfly reduction, one bf16 rounding;
//   * fused epilogues: bias (Qwen2), residual add (launch_resadd), SwiGLU
//     (launch_act + launch_elem: gate/up row j handled by the same wave), and a
//     greedy arg-max key (logit_decode.cu:15-33 tie rule) for lm_head.
// Grid is persistent-ish: min(tasks/4, CUs * blocks_per_cu) blocks of 4 waves
// that grid-stride over row tasks, so the norm prologue runs once per block.
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

#include <cstdlib>

namespace qie {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct GemvParams {
    const uint16_t* x;
    int64_t ldx;
    const uint16_t* w0;
    const uint16_t* w1;
    const uint16_t* w2;
    const uint16_t* b0;
    const uint16_t* b1;
    const uint16_t* b2;
    int64_t n0, n01;   // rows in seg0, seg0+seg1
    int64_t K, N;      // N = output columns
    uint16_t* y;
    int64_t ldy;
    const uint16_t* norm_w;
    float eps;
    int numerics;
    int M;             // runtime rows (<= MT)
    int xlds;          // 1: x staged in LDS
    unsigned long long* keys;
    int64_t key_col0;
    int64_t n_tasks;
    int dbg;           // skinny kernel timing experiments (QIE_SKINNY_DBG): 1 plain x copy instead of the
                       // fused norm, 2 stop after the prologue, 4 no prologue at all
    // interleaved RoPE in the STORE epilogue (decode QKV, M = 1, REF numerics, no qk-norm):
    // output rows [0, rope_rows) are (q | k) head rows of rope_hd; pair (2j, 2j + 1) of a
    // head is rotated by the fp32 table row of position rope_pos[0] (RoPE.cu:6-22)
    const int32_t* rope_pos;
    const float* rope_cs;
    const float* rope_sn;
    int rope_hd;
    int64_t rope_rows;
    int epre;          // M = 1: the first task's epilogue operands (bias / residual) loaded up front
    int mkdiv;         // x-first fused norm: REF quotient by the FMA-corrected reciprocal (dev A/B)
    int t16;           // skinny kernel, fp8: weights in the 16-row tiled layout (qie_fp8_tile16)
    // F32 epilogue under tensor parallelism (peer backend, M = 1): push = {tag, value} words
    // straight into every rank's tagged exchange slot (push.world > 0) instead of y
    PeerPush push;
};

// REF RMSNorm quotient f / rms: the FMA-corrected product with the reciprocal (Markstein),
// the real division outside [1e-30, 1e30] (and for 0) — see skinny_mfma_kernel's prologue
__device__ __forceinline__ float div_mk(float f, float rms, float inv) {
#pragma clang fp contract(off)
    const float q = f * inv;
    float d = fmaf(fmaf(-q, rms, f), inv, q);
    const float af = fabsf(f);
    if (af != 0.f && (af < 1e-30f || af > 1e30f)) d = f / rms;
    return d;
}

// uniform loads through the scalar cache (constant address space): the RoPE coefficients
// wait on lgkmcnt, not behind the weight stream's in-order vmcnt
template <class T>
__device__ __forceinline__ T sload(const T* p, int64_t i) {
    return ((const __attribute__((address_space(4))) T*)p)[i];
}

__device__ __forceinline__ void fma8(float& acc, const float* xf, u32x4 w) {
    acc = fmaf(xf[0], bf_lo(w.x), acc);
    acc = fmaf(xf[1], bf_hi(w.x), acc);
    acc = fmaf(xf[2], bf_lo(w.y), acc);
    acc = fmaf(xf[3], bf_hi(w.y), acc);
    acc = fmaf(xf[4], bf_lo(w.z), acc);
    acc = fmaf(xf[5], bf_hi(w.z), acc);
    acc = fmaf(xf[6], bf_lo(w.w), acc);
    acc = fmaf(xf[7], bf_hi(w.w), acc);
}

__device__ __forceinline__ void unpack8(u32x4 v, float* f) {
    f[0] = bf_lo(v.x); f[1] = bf_hi(v.x);
    f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
    f[4] = bf_lo(v.z); f[5] = bf_hi(v.z);
    f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
}

// fp8 weights (WT = 1): 16 codes per 16-byte lane load (1024 weights per wave-load),
// decoded with v_cvt_pk_f32_fp8; the power-of-two row scale multiplies the fp32 sum
// once in the epilogue (exact: the same value as summing the dequantised products).
__device__ __forceinline__ const float* fp8_scales(const uint16_t* w, int64_t rows, int64_t K) {
    return reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(w) + rows * K);
}

template <int MT, int RPW, int EPI, int U, int XCH, int WT, int LB = 256>
__global__ __launch_bounds__(LB) void gemv_kernel(GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
    float* red = reinterpret_cast<float*>(smem + (p.xlds ? (size_t)MT * p.K * 2 : 0));
    // wave index made provably wave-uniform: every task / row pointer below derives from
    // it, so the weight rows' buffer resources stay in SGPRs
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int NWv = blockDim.x >> 6;         // waves per block: 4, or 5..9 for the one-block-per-CU grid
    const int64_t TS = (int64_t)blockDim.x * 8;   // x elements per block-wide 16-byte pass
    const int64_t K = p.K;
    constexpr int EB = WT ? 1 : 2;     // bytes per weight
    constexpr int EL = 16 / EB;        // weights per 16-byte lane load
    constexpr int WS = 64 * EL;        // weights per wave-load
    // Weight rows and x are read with buffer loads: one VGPR offset per lane plus a constant
    // per chunk (no 64-bit address per chunk), and a chunk past the row end (K not a multiple
    // of a wave-load) reads zeros from the hardware range check instead of a clamped re-read.
    auto rsrc = [](const void* base, int64_t bytes) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
    };
    constexpr int kNT = 2;   // buffer-load cache policy: nt (weights stream once)

    // ---------------- task -> weight rows / output columns
    auto task_ptrs = [&](int64_t task, const u32x4* (&wr)[RPW]) {
        const uint8_t* w0 = reinterpret_cast<const uint8_t*>(p.w0);
        const uint8_t* w1 = reinterpret_cast<const uint8_t*>(p.w1);
        const uint8_t* w2 = reinterpret_cast<const uint8_t*>(p.w2);
        if constexpr (EPI == QIE_EPI_SWIGLU) {
            constexpr int P2 = RPW / 2;
#pragma unroll
            for (int i = 0; i < P2; i++) {
                int64_t j = task * P2 + i;
                if (j >= p.N) j = p.N - 1;
                wr[i] = reinterpret_cast<const u32x4*>(w0 + j * K * EB);
                wr[P2 + i] = reinterpret_cast<const u32x4*>(w1 + j * K * EB);
            }
        } else {
#pragma unroll
            for (int i = 0; i < RPW; i++) {
                int64_t r = task * RPW + i;
                if (r >= p.N) r = p.N - 1;
                const uint8_t* base;
                if (r < p.n0) base = w0 + r * K * EB;
                else if (r < p.n01) base = w1 + (r - p.n0) * K * EB;
                else base = w2 + (r - p.n01) * K * EB;
                wr[i] = reinterpret_cast<const u32x4*>(base);
            }
        }
    };
    // fp8: the row scale of output column c (segment-resolved like task_ptrs)
    auto row_scale = [&](int64_t c, int i) -> float {
        if constexpr (WT == 0) {
            return 1.f;
        } else if constexpr (EPI == QIE_EPI_SWIGLU) {
            constexpr int P2 = RPW / 2;
            return i < P2 ? fp8_scales(p.w0, p.N, K)[c] : fp8_scales(p.w1, p.N, K)[c];
        } else {
            if (c < p.n0) return fp8_scales(p.w0, p.n0, K)[c];
            if (c < p.n01) return fp8_scales(p.w1, p.n01 - p.n0, K)[c - p.n0];
            return fp8_scales(p.w2, p.N - p.n01, K)[c - p.n01];
        }
    };
    auto task_cols = [&](int64_t task, int64_t (&col)[RPW]) {
        if constexpr (EPI == QIE_EPI_SWIGLU) {
            constexpr int P2 = RPW / 2;
#pragma unroll
            for (int i = 0; i < P2; i++) col[i] = col[P2 + i] = task * P2 + i;
        } else {
#pragma unroll
            for (int i = 0; i < RPW; i++) col[i] = task * RPW + i;
        }
    };
    // Chunk slots past K re-read the row's last 16 B and are skipped by compute_chunk.  A
    // load under a condition (even a per-lane one) is branched around, and at the join
    // the waitcnt pass can no longer count it, so every later wait degrades to vmcnt(0).
    // XCH == 1 (MT = 1, no norm): x is not staged; each lane loads the 16 B of x that its
    // weight chunk multiplies together with that chunk (L1/L2 hits: every wave of the
    // block reads the same row), so no prologue or barrier precedes the weight stream.
    uint4 xg[XCH == 1 ? U : 1];
    // XCH == 3 (MT = 1, fused RMSNorm, K <= 512 U): the 64 lanes of a wave load all of x
    // between them (U 16-B chunks per lane), so every wave reduces the sum of squares itself
    // (wave_sum, no cross-wave exchange); wave w then normalises chunks w, w + NW, ... into
    // LDS — one barrier in all, instead of the x-first prologue's two around a block reduction.
    uint4 xr[XCH == 3 ? U : 1];
    // XCH == 4 (MT = 1, fused RMSNorm, K <= 512 U): as XCH == 3, but every wave also
    // normalises ITS OWN chunks in registers — lane l's x chunk u is exactly the 8 elements
    // its weight chunk u multiplies — so there is no LDS image, no barrier and no LDS read
    // in the weight loop; the norm's divisions are repeated per wave (56 per lane at
    // K = 3,584) while the weight stream is in flight.
    uint4 xq[XCH == 4 ? U : 1];
    // Epilogue operands of the wave's FIRST task (M = 1: bias values of STORE rows, the old
    // residual values of RESIDUAL rows) loaded before its weight stream, so the epilogue of a
    // one-task wave — every small decode GEMV — has no dependent load after the reduction.
    // Unconditional buffer loads (a missing bias reads element 0 of x; the epilogue ignores it).
    constexpr bool EPRE = MT == 1 && (EPI == QIE_EPI_RESIDUAL || EPI == QIE_EPI_STORE);
    uint32_t epre_v[EPRE ? RPW : 1];
    // the loads are issued WITHOUT a branch: a load under a (even uniform) condition makes the
    // waitcnt pass fall back to vmcnt(0) at every later wait, and the weight stream stops
    // pipelining (the first, branched form measured QKV 10.0 -> 10.7, O 6.4 -> 6.9 us)
    constexpr bool EPRE_ON = EPRE && XCH > 0;
    const bool epre_on = EPRE_ON && p.M == 1 && p.epre != 0;   // uniform; p.epre = 0 (dev A/B): reload
    auto epre_issue = [&](int64_t task) {
        if constexpr (EPRE) {
#pragma unroll
            for (int i = 0; i < RPW; i++) {
                int64_t c = task * RPW + i;
                c = c < p.N ? c : p.N - 1;
                if constexpr (EPI == QIE_EPI_RESIDUAL) {
                    const auto ry = rsrc(p.y, p.N * 2);
                    epre_v[i] = __builtin_amdgcn_raw_buffer_load_b16(ry, (int)(c * 2), 0, 0);
                } else {
                    const uint16_t* b = c < p.n0 ? p.b0 : (c < p.n01 ? p.b1 : p.b2);
                    const int64_t bi = c < p.n0 ? c : (c < p.n01 ? c - p.n0 : c - p.n01);
                    const auto rb = rsrc(b ? (const void*)b : (const void*)p.x, b ? (bi + 1) * 2 : 2);
                    epre_v[i] = __builtin_amdgcn_raw_buffer_load_b16(rb, b ? (int)(bi * 2) : 0, 0, 0);
                }
            }
        }
    };
    auto load_chunk = [&](const u32x4* const (&wr)[RPW], int64_t k0, u32x4 (&wv)[U][RPW]) {
        const int voff = (int)(k0 * EB);   // this lane's byte offset in the row (< 2^31)
        const auto rx = rsrc(p.x, K * 2);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if constexpr (XCH == 1) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(k0 * 2), u * WS * 2, 0);
                xg[u] = make_uint4(v.x, v.y, v.z, v.w);
            }
#pragma unroll
            for (int i = 0; i < RPW; i++)   // unconditional loads (a chunk past K reads zeros)
                wv[u][i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(wr[i], K * EB), voff, u * WS * EB, kNT);
        }
    };
    auto x_at = [&](int m, int64_t k) -> uint4 {
        return p.xlds ? *reinterpret_cast<const uint4*>(xs + (int64_t)m * K + k)
                      : (m < p.M ? *reinterpret_cast<const uint4*>(p.x + (int64_t)m * p.ldx + k)
                                 : make_uint4(0, 0, 0, 0));
    };
    auto compute_chunk = [&](int64_t k0, const u32x4 (&wv)[U][RPW], float (&acc)[MT][RPW]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t k = k0 + u * WS;
            if (k < K) {
                if constexpr (WT == 0) {
#pragma unroll
                    for (int m = 0; m < MT; m++) {
                        const uint4 xv = XCH == 1 ? xg[XCH == 1 ? u : 0] : (XCH == 4 ? xq[XCH == 4 ? u : 0] : x_at(m, k));
                        float xf[8];
                        unpack8(u32x4{xv.x, xv.y, xv.z, xv.w}, xf);
#pragma unroll
                        for (int i = 0; i < RPW; i++) fma8(acc[m][i], xf, wv[u][i]);
                    }
                } else {
                    float wf[RPW][16];
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        fp8x4_to_f32(wv[u][i].x, wf[i]);
                        fp8x4_to_f32(wv[u][i].y, wf[i] + 4);
                        fp8x4_to_f32(wv[u][i].z, wf[i] + 8);
                        fp8x4_to_f32(wv[u][i].w, wf[i] + 12);
                    }
#pragma unroll
                    for (int m = 0; m < MT; m++) {
                        const uint4 x0 = x_at(m, k), x1 = x_at(m, k + 8);
                        float xf[16];
                        unpack8(u32x4{x0.x, x0.y, x0.z, x0.w}, xf);
                        unpack8(u32x4{x1.x, x1.y, x1.z, x1.w}, xf + 8);
#pragma unroll
                        for (int i = 0; i < RPW; i++)
#pragma unroll
                            for (int j = 0; j < 16; j++) acc[m][i] = fmaf(xf[j], wf[i][j], acc[m][i]);
                    }
                }
            }
        }
    };

    const int64_t tstride = (int64_t)gridDim.x * NWv;
    const int64_t task0 = (int64_t)blockIdx.x * NWv + wave;
    // RoPE epilogue: the position goes out first (one scalar load), its table row for the
    // first task after the prologue, so neither round trip lands after the weight stream
    constexpr bool ROPE = EPI == QIE_EPI_STORE && RPW % 2 == 0 && MT == 1;
    const bool rope = ROPE && p.rope_rows > 0;
    int32_t rpos = 0;   // loaded right after the first weight issue (an lgkmcnt wait before it would hold the issue)
    const u32x4* wr[RPW];
    u32x4 wv[U][RPW];
    constexpr bool PF = XCH > 0;

    if constexpr (XCH == 1) {
        if constexpr (EPRE_ON) epre_issue(task0 < p.n_tasks ? task0 : p.n_tasks - 1);
        task_ptrs(task0 < p.n_tasks ? task0 : p.n_tasks - 1, wr);
        load_chunk(wr, (int64_t)lane * EL, wv);
    } else if constexpr (XCH == 3) {
        // x chunks first, then the wave's first weight chunks, THEN the norm arithmetic
        // (vmcnt retires in order: the x loads must be the older ones)
        const auto rx = rsrc(p.x, K * 2), rn = rsrc(p.norm_w, K * 2);
#pragma unroll
        for (int u = 0; u < U; u++) {   // a chunk past K reads zeros (range check)
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16, u * 1024, 0);
            xr[u] = make_uint4(a.x, a.y, a.z, a.w);
        }
        // the norm weights of the (at most NWC) chunks this wave normalises, also before the
        // weight stream: a load issued after it could only be waited for behind all of it
        constexpr int NWC = (U + 3) / 4;   // chunks per wave at >= 4 waves per block
        u32x4 nvw[NWC];
#pragma unroll
        for (int c = 0; c < NWC; c++) {
            const int u = wave + c * NWv;   // wave-uniform; past U: a harmless in-range re-read
            nvw[c] = __builtin_amdgcn_raw_buffer_load_b128(rn, lane * 16, (u < U ? u : 0) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (EPRE_ON) epre_issue(task0 < p.n_tasks ? task0 : p.n_tasks - 1);
        task_ptrs(task0 < p.n_tasks ? task0 : p.n_tasks - 1, wr);
        load_chunk(wr, (int64_t)lane * EL, wv);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++)   // opaque: the x math cannot be hoisted above the weight issue
            asm volatile("" : "+v"(xr[u].x), "+v"(xr[u].y), "+v"(xr[u].z), "+v"(xr[u].w));
#pragma unroll
        for (int c = 0; c < NWC; c++) asm volatile("" : "+v"(nvw[c]));
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < U; u++) {
            float f[8];
            unpack8(u32x4{xr[u].x, xr[u].y, xr[u].z, xr[u].w}, f);
#pragma unroll
            for (int j = 0; j < 8; j++) ss += f[j] * f[j];
        }
        ss = wave_sum(ss);
        const float rms = sqrtf((ss / (float)K) + p.eps);
        const float inv = 1.0f / rms;
        const bool hf = p.numerics == QIE_NUMERICS_HF;
        const int nch = (int)((K + WS - 1) / WS);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
        for (int c = 0; c < NWC; c++) {   // static indices into xr / nvw: no scratch
#pragma clang fp contract(off)
            if (u != wave + c * NWv || u >= nch) continue;   // wave-uniform
            float f[8], wf[8];
            unpack8(u32x4{xr[u].x, xr[u].y, xr[u].z, xr[u].w}, f);
            unpack8(nvw[c], wf);
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float y0, y1;
                if (hf) {
                    y0 = wf[2 * j] * rbf(f[2 * j] * inv);
                    y1 = wf[2 * j + 1] * rbf(f[2 * j + 1] * inv);
                } else {
                    y0 = (f[2 * j] / rms) * wf[2 * j];
                    y1 = (f[2 * j + 1] / rms) * wf[2 * j + 1];
                }
                o[j] = pack2(y0, y1);
            }
            const int64_t k = (int64_t)lane * EL + u * WS;
            if (k < K) *reinterpret_cast<uint4*>(xs + k) = make_uint4(o[0], o[1], o[2], o[3]);
        }
        __syncthreads();
    } else if constexpr (XCH == 4) {
        // x and the norm weights first (one 16-B chunk per wave-load slot u, a chunk past K
        // reads zeros), then the first task's weight stream, THEN the norm arithmetic
        const auto rx = rsrc(p.x, K * 2), rn = rsrc(p.norm_w, K * 2);
        u32x4 xa[U], na[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            xa[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16, u * 1024, 0);
            na[u] = __builtin_amdgcn_raw_buffer_load_b128(rn, lane * 16, u * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (EPRE_ON) epre_issue(task0 < p.n_tasks ? task0 : p.n_tasks - 1);
        task_ptrs(task0 < p.n_tasks ? task0 : p.n_tasks - 1, wr);
        load_chunk(wr, (int64_t)lane * EL, wv);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++) asm volatile("" : "+v"(xa[u]), "+v"(na[u]));
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < U; u++) {
            float f[8];
            unpack8(xa[u], f);
#pragma unroll
            for (int j = 0; j < 8; j++) ss += f[j] * f[j];
        }
        ss = wave_sum(ss);
        const float rms = sqrtf((ss / (float)K) + p.eps);
        const float inv = 1.0f / rms;
        const bool hf = p.numerics == QIE_NUMERICS_HF;
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma clang fp contract(off)
            float f[8], wf[8];
            unpack8(xa[u], f);
            unpack8(na[u], wf);
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float y0, y1;
                if (hf) {
                    y0 = wf[2 * j] * rbf(f[2 * j] * inv);
                    y1 = wf[2 * j + 1] * rbf(f[2 * j + 1] * inv);
                } else if (p.mkdiv) {
                    y0 = div_mk(f[2 * j], rms, inv) * wf[2 * j];
                    y1 = div_mk(f[2 * j + 1], rms, inv) * wf[2 * j + 1];
                } else {
                    y0 = (f[2 * j] / rms) * wf[2 * j];
                    y1 = (f[2 * j + 1] / rms) * wf[2 * j + 1];
                }
                o[j] = pack2(y0, y1);
            }
            xq[u] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    } else if constexpr (XCH > 0) {
        // ---------------- x-first prologue (MT = 1, x staged in LDS, K <= 2048 * XCH; the
        // host guarantees it).  Order of issue: this thread's x chunks (+ norm weights),
        // then the first weight chunk of the wave's first task, THEN the x arithmetic — so
        // the weight stream's first HBM round trip overlaps the x round trip instead of
        // following it (vmcnt retires in order: x must be issued first).
        constexpr int NV = XCH <= 5 ? XCH : 1;   // norm weights: fused-norm variants only (XCH <= 5)
        const bool nrm = NV == XCH && p.norm_w != nullptr && !QIE_DBG(p.dbg & 1);   // dev: 1 skips the norm
        uint4 xv[XCH], nv[NV];
#pragma unroll
        for (int c = 0; c < XCH; c++) {
            const int64_t k = (int64_t)tid * 8 + c * TS;
            const int64_t kc = k < K ? k : K - 8;   // clamped: loads stay unconditional
            xv[c] = *reinterpret_cast<const uint4*>(p.x + kc);
            if (c < NV) nv[c] = *reinterpret_cast<const uint4*>((nrm ? p.norm_w : p.x) + kc);
        }
        __builtin_amdgcn_sched_barrier(0);
        // unconditional (a wave without a task re-reads the last row): a load under a
        // branch makes the vmcnt bookkeeping at the join wait for everything
        if constexpr (EPRE_ON) epre_issue(task0 < p.n_tasks ? task0 : p.n_tasks - 1);
        task_ptrs(task0 < p.n_tasks ? task0 : p.n_tasks - 1, wr);
        load_chunk(wr, (int64_t)lane * EL, wv);
        __builtin_amdgcn_sched_barrier(0);
        if (rope) rpos = sload(p.rope_pos, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < XCH; c++) {   // opaque: x math cannot be hoisted above the weight issue
            asm volatile("" : "+v"(xv[c].x), "+v"(xv[c].y), "+v"(xv[c].z), "+v"(xv[c].w));
            if (c < NV) asm volatile("" : "+v"(nv[c].x), "+v"(nv[c].y), "+v"(nv[c].z), "+v"(nv[c].w));
        }
        bool staged = false;
        if constexpr (NV == XCH) if (nrm) {
            staged = true;
            float ss = 0.f;
#pragma unroll
            for (int c = 0; c < XCH; c++) {
                if ((int64_t)tid * 8 + c * TS >= K) continue;
                float f[8];
                unpack8(u32x4{xv[c].x, xv[c].y, xv[c].z, xv[c].w}, f);
#pragma unroll
                for (int j = 0; j < 8; j++) ss += f[j] * f[j];
            }
            ss = wave_sum(ss);
            if (lane == 0) red[wave] = ss;
            __syncthreads();
            ss = 0.f;
            for (int w = 0; w < NWv; w++) ss += red[w];
            const float rms = sqrtf((ss / (float)K) + p.eps);
            const float inv = 1.0f / rms;
            const bool hf = p.numerics == QIE_NUMERICS_HF;
#pragma unroll
            for (int c = 0; c < XCH; c++) {
#pragma clang fp contract(off)
                const int64_t k = (int64_t)tid * 8 + c * TS;
                if (k >= K) continue;
                float f[8], wf[8];
                unpack8(u32x4{xv[c].x, xv[c].y, xv[c].z, xv[c].w}, f);
                unpack8(u32x4{nv[c].x, nv[c].y, nv[c].z, nv[c].w}, wf);
                uint32_t o[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float y0, y1;
                    if (hf) {
                        y0 = wf[2 * j] * rbf(f[2 * j] * inv);
                        y1 = wf[2 * j + 1] * rbf(f[2 * j + 1] * inv);
                    } else if (p.mkdiv) {
                        y0 = div_mk(f[2 * j], rms, inv) * wf[2 * j];
                        y1 = div_mk(f[2 * j + 1], rms, inv) * wf[2 * j + 1];
                    } else {
                        y0 = (f[2 * j] / rms) * wf[2 * j];
                        y1 = (f[2 * j + 1] / rms) * wf[2 * j + 1];
                    }
                    o[j] = pack2(y0, y1);
                }
                *reinterpret_cast<uint4*>(xs + k) = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
        if (!staged) {
#pragma unroll
            for (int c = 0; c < XCH; c++) {
                const int64_t k = (int64_t)tid * 8 + c * TS;
                if (k < K) *reinterpret_cast<uint4*>(xs + k) = xv[c];
            }
        }
        __syncthreads();
    } else if (p.xlds) {
        // ---------------- prologue: activation rows -> LDS (optionally RMS-normed)
        for (int m = 0; m < MT; m++) {
            const uint16_t* xr = p.x + (int64_t)m * p.ldx;
            uint16_t* xo = xs + (int64_t)m * K;
            if (m >= p.M) {
                for (int64_t k = tid * 8; k < K; k += TS)
                    *reinterpret_cast<uint4*>(xo + k) = make_uint4(0, 0, 0, 0);
                continue;
            }
            if (p.norm_w) {
                float ss = 0.f;
                for (int64_t k = tid * 8; k < K; k += TS) {
                    uint4 v = *reinterpret_cast<const uint4*>(xr + k);
                    float f[8];
                    unpack8(u32x4{v.x, v.y, v.z, v.w}, f);
#pragma unroll
                    for (int j = 0; j < 8; j++) ss += f[j] * f[j];
                }
                ss = wave_sum(ss);
                if (lane == 0) red[wave] = ss;
                __syncthreads();
                ss = 0.f;
                for (int w = 0; w < NWv; w++) ss += red[w];
                __syncthreads();
                const float rms = sqrtf((ss / (float)K) + p.eps);
                const float inv = 1.0f / rms;
                const bool hf = p.numerics == QIE_NUMERICS_HF;
                for (int64_t k = tid * 8; k < K; k += TS) {
#pragma clang fp contract(off)
                    uint4 v = *reinterpret_cast<const uint4*>(xr + k);
                    uint4 nw = *reinterpret_cast<const uint4*>(p.norm_w + k);
                    float f[8], wf[8];
                    unpack8(u32x4{v.x, v.y, v.z, v.w}, f);
                    unpack8(u32x4{nw.x, nw.y, nw.z, nw.w}, wf);
                    uint32_t o[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        float y0, y1;
                        if (hf) {
                            y0 = wf[2 * j] * rbf(f[2 * j] * inv);
                            y1 = wf[2 * j + 1] * rbf(f[2 * j + 1] * inv);
                        } else {
                            y0 = (f[2 * j] / rms) * wf[2 * j];
                            y1 = (f[2 * j + 1] / rms) * wf[2 * j + 1];
                        }
                        o[j] = pack2(y0, y1);
                    }
                    *reinterpret_cast<uint4*>(xo + k) = make_uint4(o[0], o[1], o[2], o[3]);
                }
            } else {
                for (int64_t k = tid * 8; k < K; k += TS)
                    *reinterpret_cast<uint4*>(xo + k) = *reinterpret_cast<const uint4*>(xr + k);
            }
        }
        __syncthreads();
    }
    if constexpr (XCH == 0 || XCH == 1 || XCH == 3 || XCH == 4)   // prologues without the early position load
        if (rope) rpos = sload(p.rope_pos, 0);
    float rc[ROPE ? RPW / 2 : 1], rs[ROPE ? RPW / 2 : 1];
    auto rope_coef = [&](int64_t task, float* c_out, float* s_out) {
#pragma unroll
        for (int i = 0; i < (ROPE ? RPW / 2 : 0); i++) {
            const int64_t c = task * RPW + 2 * i;   // STORE: rows of a task are consecutive
            const int64_t j = (int64_t)rpos * (p.rope_hd / 2) + (c % p.rope_hd) / 2;
            const bool ok = c + 1 < p.rope_rows;
            c_out[i] = ok ? sload(p.rope_cs, j) : 1.f;
            s_out[i] = ok ? sload(p.rope_sn, j) : 0.f;
        }
    };
    if (rope) rope_coef(task0 < p.n_tasks ? task0 : 0, rc, rs);

    // Running arg-max key per row (lane 0 of each wave); reduced over the block and
    // published with ONE atomicMax per block after the task loop — an atomic per task
    // serialises ~76k atomics on one address for a 152k-row lm_head (0.9 ms).
    unsigned long long kbest[MT];
#pragma unroll
    for (int m = 0; m < MT; m++) kbest[m] = 0ull;

    // ---------------- main loop over row tasks.  Software-pipelined across tasks: the
    // first weight chunk of a wave's NEXT task is issued before this task's reduction
    // and epilogue (and the first task's before the prologue above), so a wave with one
    // or two tasks — every small decode GEMV — pays one HBM round trip, not three.
    for (int64_t task = task0; task < p.n_tasks; task += tstride) {
        int64_t col[RPW];
        task_cols(task, col);
        if constexpr (!PF) {
            task_ptrs(task, wr);
            load_chunk(wr, (int64_t)lane * EL, wv);
        }
        float acc[MT][RPW];
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int i = 0; i < RPW; i++) acc[m][i] = 0.f;
        compute_chunk((int64_t)lane * EL, wv, acc);
        for (int64_t k0 = (int64_t)lane * EL + WS * U; k0 < K; k0 += WS * U) {
            load_chunk(wr, k0, wv);
            compute_chunk(k0, wv, acc);
        }
        if (PF && task + tstride < p.n_tasks) {
            task_ptrs(task + tstride, wr);
            load_chunk(wr, (int64_t)lane * EL, wv);
        }
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int i = 0; i < RPW; i++) acc[m][i] = wave_sum(acc[m][i]);
        if constexpr (WT != 0) {   // fp8: the power-of-two row scale, once per output
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < RPW; i++) {
                    const float sc = row_scale(col[i] < p.N ? col[i] : p.N - 1, i);
#pragma unroll
                    for (int m = 0; m < MT; m++) acc[m][i] *= sc;
                }
            }
        }

        // ---------------- epilogue (lane 0 writes; outputs are tiny)
        if (lane == 0) {
#pragma clang fp contract(off)
#pragma unroll
            for (int m = 0; m < MT; m++) {
                if (m >= p.M) continue;
                uint16_t* yr = p.y + (int64_t)m * p.ldy;
                if constexpr (EPI == QIE_EPI_SWIGLU) {
                    constexpr int P2 = RPW / 2;
#pragma unroll
                    for (int i = 0; i < P2; i++) {
                        if (col[i] >= p.N) continue;
                        float g = rbf(acc[m][i]);
                        float u = rbf(acc[m][P2 + i]);
                        float a = rbf(g * (1.0f / (1.0f + expf(-g))));
                        yr[col[i]] = f2bf(u * a);
                    }
                } else if constexpr (EPI == QIE_EPI_F32) {
                    if (p.push.world > 0) {
                        // the row-parallel exchange's send, issued as each row finishes
                        // (comm.hip peer_tag_kernel<true> waits for and reduces it)
                        const unsigned e = __hip_atomic_load(p.push.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                        for (int i = 0; i < RPW; i++) {
                            if (col[i] >= p.N) continue;
                            const uint64_t w = (uint64_t)(e + 1) | ((uint64_t)__float_as_uint(acc[m][i]) << 32);
                            const int64_t at = (int64_t)m * p.ldy + col[i];
#pragma unroll
                            for (int q = 0; q < kPeerTagMaxWorld; q++)
                                if (q < p.push.world)
                                    __hip_atomic_store(peer_tag_slot(p.push.tb[q], e, p.push.rank) + at, w,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                    } else {
                        float* yf = reinterpret_cast<float*>(p.y) + (int64_t)m * p.ldy;
#pragma unroll
                        for (int i = 0; i < RPW; i++)
                            if (col[i] < p.N) yf[col[i]] = acc[m][i];
                    }
                } else if constexpr (EPI == QIE_EPI_RESIDUAL) {
                    const bool pre = epre_on && task == task0;
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        if (col[i] >= p.N) continue;
                        const float old = pre ? bf2f(epre_v[EPRE ? i : 0]) : bf2f(yr[col[i]]);
                        yr[col[i]] = f2bf(old + rbf(acc[m][i]));
                    }
                } else {
                    unsigned long long best = kbest[m];
                    float vv[RPW];
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        const int64_t c = col[i] < p.N ? col[i] : p.N - 1;
                        float v = acc[m][i];
                        const uint16_t* b = c < p.n0 ? p.b0 : (c < p.n01 ? p.b1 : p.b2);
                        if (QIE_DBG(p.dbg & 2)) {   // dev: 2 skips the bias
                        } else if (epre_on && task == task0) {
                            if (b) v = v + bf2f(epre_v[EPRE ? i : 0]);
                        } else if (b) {
                            int64_t bi = c < p.n0 ? c : (c < p.n01 ? c - p.n0 : c - p.n01);
                            v = v + bf2f(b[bi]);
                        }
                        vv[i] = rbf(v);   // the projection's bf16 output
                    }
                    if constexpr (ROPE) {
                        if (rope) {   // uniform: (2j, 2j + 1) pairs of q / k head rows
                            float tc[RPW / 2], ts[RPW / 2];
                            if (task != task0) rope_coef(task, tc, ts);
#pragma unroll
                            for (int i = 0; i < RPW / 2; i++) {
                                const int64_t c = col[2 * i];
                                if (c + 1 >= p.rope_rows || c + 1 >= p.N) continue;
                                const float cs = task == task0 ? rc[i] : tc[i];
                                const float sn = task == task0 ? rs[i] : ts[i];
                                const float x0 = vv[2 * i], x1 = vv[2 * i + 1];
                                vv[2 * i] = x0 * cs - x1 * sn;
                                vv[2 * i + 1] = x1 * cs + x0 * sn;
                            }
                        }
                    }
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        const int64_t c = col[i];
                        if (c >= p.N) continue;
                        uint16_t o = f2bf(vv[i]);
                        yr[c] = o;
                        if (p.keys) {
                            unsigned long long kk = sel_key(bf2f(o), (uint32_t)(c + p.key_col0));
                            best = kk > best ? kk : best;
                        }
                    }
                    kbest[m] = best;
                }
            }
        }
    }
    if constexpr (EPI == QIE_EPI_STORE) {
        if (p.keys) {
            __shared__ unsigned long long kb_s[16][MT];
            if (lane == 0) {
#pragma unroll
                for (int m = 0; m < MT; m++) kb_s[wave][m] = kbest[m];
            }
            __syncthreads();
            if (tid < MT && tid < p.M) {
                unsigned long long b = kb_s[0][tid];
#pragma unroll
                for (int w = 1; w < NWv; w++) b = kb_s[w][tid] > b ? kb_s[w][tid] : b;
                if (b) atomicMax(p.keys + tid, b);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Skinny MFMA GEMM for 2 <= M <= 16 (batched decode, short prefills): the M activation
// rows are the 16 rows of v_mfma_f32_16x16x32_bf16's A operand (rows >= M compute
// garbage that is never stored), a block owns 16 output columns (16 weight rows; 16
// gate + 16 up for SwiGLU) and its 4 waves split K, so the weights stream exactly once
// as B fragments (16 B per lane per MFMA step, one weight row per lane column) and the
// per-element VALU work of the GEMV (M FMAs per weight) moves to the matrix cores.  fp8
// weights: a 16-B load holds 16 codes = two k-steps; decoded to bf16 (exact) for the
// bf16 MFMA, the row scale applied to the fp32 result.  Partial C tiles of the 4 waves
// are summed in LDS, then the epilogue (bias / arg-max keys / residual / SwiGLU / f32).
// Persistent over column tiles (grid <= 4 blocks per CU) so arg-max keys merge per block.
template <int EPI, int WT, int XL, int NW, int UO = 0>
__global__ __launch_bounds__(NW * 64) void skinny_mfma_kernel(GemvParams p) {
#pragma clang fp contract(off)
    constexpr int NB = EPI == QIE_EPI_SWIGLU ? 2 : 1;   // B tiles per block (gate, up)
    // A unit = 64 k of each of the tile's 16 weight rows: a lane loads 32 contiguous bytes
    // of its row (bf16: two 16-B vectors, two MFMA k-steps; fp8: one 16-B vector of 16
    // codes), so one unit reads whole 128-B lines per row (bf16; fp8 64 B) instead of the
    // 64-B half lines of a 32-k unit.
    constexpr int KSTEP = 64;
    constexpr int WV = WT ? 1 : 2;                        // 16-B weight vectors per lane per unit
    // units per step (UO: sized to the wave's K range, so no step slot is a dead unit)
    constexpr int U = UO ? UO : (WT ? ((XL && NB == 1) ? 8 : 4) : ((XL && NB == 1) ? 4 : 2));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t K = p.K;
    const int M = p.M;
    // [M][K + 8]: the 16-B row pad puts the 16 A rows of an MFMA fragment read on
    // distinct LDS banks (an unpadded 7168-B row stride maps every row to one bank)
    const int64_t KP = K + 8;
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
    float* red = reinterpret_cast<float*>(smem + (XL ? (size_t)M * KP * 2 : 0));            // [NW - 1][NB][256]
    __shared__ unsigned long long kb_s[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fr = lane & 15, g = lane >> 4;
    const int arow = fr < M ? fr : M - 1;   // A row of this lane (rows >= M: garbage, never stored)

    auto xa = [&](int64_t k) -> uint4 {   // 8 activations of this lane's A row at k
        return XL ? *reinterpret_cast<const uint4*>(xs + (int64_t)arow * KP + k)
                  : *reinterpret_cast<const uint4*>(p.x + (int64_t)arow * p.ldx + k);
    };

    // segment pointers as laundered byte offsets from one base (see issue()): the
    // result stays a global-address-space pointer derived from that base
    const uint8_t* const wbase = reinterpret_cast<const uint8_t*>(p.w0);
    const uint64_t dw1 = launder_u64((uint64_t)p.w1 - (uint64_t)p.w0);
    const uint64_t dw2 = launder_u64((uint64_t)p.w2 - (uint64_t)p.w0);
    const uint8_t* const bbase = reinterpret_cast<const uint8_t*>(p.x);
    auto boff = [&](const uint16_t* b) { return launder_u64(b ? (uint64_t)b - (uint64_t)p.x : 0ull); };
    const uint64_t db0 = boff(p.b0), db1 = boff(p.b1), db2 = boff(p.b2);
    const uint64_t hb0 = launder_u64(p.b0 ? ~0ull : 0ull), hb1 = launder_u64(p.b1 ? ~0ull : 0ull),
                   hb2 = launder_u64(p.b2 ? ~0ull : 0ull);   // segment has a bias (all-ones mask)
    // this wave's K range, in 16-byte load units; a tile is NBAT steps of U units
    const int64_t units = K / KSTEP;
    const int64_t uw = (units + NW - 1) / NW;
    const int64_t ub = wave * uw, ue = ub + uw < units ? ub + uw : units;
    const int64_t nbat = (uw + U - 1) / U;
    const int64_t n_tiles = (p.N + 15) / 16;
    if ((int64_t)blockIdx.x >= n_tiles) return;   // block-uniform, before any barrier
    const int64_t my_tiles = (n_tiles - 1 - blockIdx.x) / gridDim.x + 1;
    const int64_t S = my_tiles * nbat;            // steps of this block (same for every wave)
    unsigned long long kbest[4] = {0ull, 0ull, 0ull, 0ull};   // rows 4 g + r

    // One step = U units of every B tile of one column tile, plus that tile's epilogue
    // operands (row scales, bias / residual values), all loaded unconditionally so no
    // global load sits under a branch: the steps form one stream per wave, double-
    // buffered in registers, so the next step's loads (next tile included) are in
    // flight while this step's MFMAs, the cross-wave reduction and the epilogue run.
    constexpr int AW = KSTEP / 32;   // 16-B A fragments per unit (8 k each, from k KSTEP/4 * g)
    constexpr int EB = WT ? 1 : 2;
    struct Step {
        u32x4 wv[U][NB][WV];
        uint4 av[XL ? 1 : U][AW];
        float wsc[NB];
        float ep[4];       // residual values (rows 4 g + r) or the bias (ep[0])
        int64_t u0, tile;
        bool last;         // last step of its tile
    };
    auto issue = [&](Step& st, int64_t s) {
        s = s < S ? s : S - 1;
        const int32_t tl = (int32_t)s / (int32_t)nbat, j = (int32_t)s - tl * (int32_t)nbat;   // < 2^31 steps
        st.tile = blockIdx.x + tl * gridDim.x;
        st.u0 = ub + j * U;
        st.last = j == nbat - 1;
        const int64_t n = st.tile * 16 + fr;
        const int64_t nc = n < p.N ? n : p.N - 1;
        const uint8_t* wrow[NB];
        const uint8_t* wseg[NB];   // segment bases (the 16-row tiled fp8 layout)
        const float* scp[NB];
        int64_t r = nc;    // row within the column's segment
        if constexpr (NB == 2) {
            wseg[0] = wbase;
            wseg[1] = wbase + dw1;
            wrow[0] = wbase + nc * K * EB;
            wrow[1] = wbase + dw1 + nc * K * EB;
            scp[0] = reinterpret_cast<const float*>(wbase + p.N * K) + nc;
            scp[1] = reinterpret_cast<const float*>(wbase + dw1 + p.N * K) + nc;
        } else {
            // segment resolved by integer selects on laundered (register) pointers: a
            // select between two kernel-argument loads would become a per-lane load
            const bool s0 = nc < p.n0, s1 = !s0 && nc < p.n01;
            r = s0 ? nc : (s1 ? nc - p.n0 : nc - p.n01);
            const uint64_t m0 = 0ull - (uint64_t)s0, m1 = 0ull - (uint64_t)s1, m2 = ~(m0 | m1);
            const uint8_t* wb = wbase + ((dw1 & m1) | (dw2 & m2));
            (void)m0;
            const int64_t rows = s0 ? p.n0 : (s1 ? p.n01 - p.n0 : p.N - p.n01);
            wseg[0] = wb;
            wrow[0] = wb + r * K * EB;
            scp[0] = reinterpret_cast<const float*>(wb + rows * K) + r;
        }
        if constexpr (WT != 0) {
#pragma unroll
            for (int b = 0; b < NB; b++) st.wsc[b] = *scp[b];
        }
        if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int i = 4 * g + rr < M ? 4 * g + rr : M - 1;
                st.ep[rr] = bf2f(p.y[(int64_t)i * p.ldy + nc]);
            }
        } else if constexpr (EPI == QIE_EPI_STORE) {
            // bias: always loaded (a missing segment bias reads x[0] and is multiplied by 0)
            const bool s0 = nc < p.n0, s1 = !s0 && nc < p.n01;
            const uint64_t m0 = 0ull - (uint64_t)s0, m1 = 0ull - (uint64_t)s1, m2 = ~(m0 | m1);
            const uint8_t* bb = bbase + ((db0 & m0) | (db1 & m1) | (db2 & m2));
            const uint64_t hb = (hb0 & m0) | (hb1 & m1) | (hb2 & m2);
            const uint16_t v = *(reinterpret_cast<const uint16_t*>(bb) + (r & (int64_t)hb));
            st.ep[0] = __uint_as_float((uint32_t)hb & __float_as_uint(bf2f(v)));
        }
        // fp8: lane (fr, g)'s 16 codes of unit uu — plain rows: bytes uu * 64 + 16 g of its row;
        // 16-row tiled (p.t16): bytes (fr + 16 g) * 16 of the unit's 1-KiB block, so one load
        // instruction reads 8 whole lines instead of 16 rows x 64 B (tiles start at segment
        // starts; a clamped row past N stays inside its segment's last tile)
        const uint8_t* lb[NB];
        int64_t ls = KSTEP * EB;
        if constexpr (WT != 0) {
#pragma unroll
            for (int b = 0; b < NB; b++)
                lb[b] = p.t16 ? wseg[b] + (r >> 4) * 16 * K + ((r & 15) + 16 * g) * 16 : wrow[b] + 16 * g;
            ls = p.t16 ? 1024 : KSTEP;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t uu = st.u0 + u < ue ? st.u0 + u : ue - 1;
#pragma unroll
            for (int b = 0; b < NB; b++)   // bytes [uu * KSTEP * EB + 16 WV g, +16 WV) of the row
#pragma unroll
                for (int h = 0; h < WV; h++) {
                    if constexpr (WT != 0)
                        st.wv[u][b][h] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(lb[b] + uu * ls));
                    else
                        st.wv[u][b][h] =
                            __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow[b]) + uu * (4 * WV) + WV * g + h);
                }
            if constexpr (!XL) {
                const int64_t kk = uu * KSTEP + (KSTEP / 4) * g;
#pragma unroll
                for (int h = 0; h < AW; h++) st.av[u][h] = xa(kk + 8 * h);
            }
        }
    };
    f32x4_t acc[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) acc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // full: every unit of the step is inside this wave's K range (all but a range's last
    // step), so no per-unit masking; otherwise dead units multiply a zero A fragment
    auto compute = [&](const Step& st, bool full) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool live = full || st.u0 + u < ue;
            const int64_t uu = live ? st.u0 + u : ue - 1;
            const int64_t kk = uu * KSTEP + (KSTEP / 4) * g;
            uint4 ar[AW];
#pragma unroll
            for (int h = 0; h < AW; h++) {
                const uint4 v = XL ? xa(kk + 8 * h) : st.av[XL ? 0 : u][h];
                ar[h] = live ? v : make_uint4(0, 0, 0, 0);
            }
            if constexpr (WT == 0) {
                const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, ar[0]);
                const bf16x8_t a1 = __builtin_bit_cast(bf16x8_t, ar[1]);
#pragma unroll
                for (int b = 0; b < NB; b++) {
                    acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, __builtin_bit_cast(bf16x8_t, st.wv[u][b][0]),
                                                                     acc[b], 0, 0, 0);
                    acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, __builtin_bit_cast(bf16x8_t, st.wv[u][b][1]),
                                                                     acc[b], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int h = 0; h < WV; h++) {   // 16 codes: A fragments 2h (codes 0..7), 2h + 1 (8..15)
                    const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, ar[2 * h]);
                    const bf16x8_t a1 = __builtin_bit_cast(bf16x8_t, ar[2 * h + 1]);
#pragma unroll
                    for (int b = 0; b < NB; b++) {
                        const uint2 c0 = fp8x4_to_bf16x4(st.wv[u][b][h].x), c1 = fp8x4_to_bf16x4(st.wv[u][b][h].y);
                        const uint2 c2 = fp8x4_to_bf16x4(st.wv[u][b][h].z), c3 = fp8x4_to_bf16x4(st.wv[u][b][h].w);
                        const uint4 lo = make_uint4(c0.x, c0.y, c1.x, c1.y);
                        const uint4 hi = make_uint4(c2.x, c2.y, c3.x, c3.y);
                        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, __builtin_bit_cast(bf16x8_t, lo), acc[b],
                                                                         0, 0, 0);
                        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, __builtin_bit_cast(bf16x8_t, hi), acc[b],
                                                                         0, 0, 0);
                    }
                }
            }
        }
    };
    // ---- end of a tile: sum the 4 waves' partial tiles (C map: col = fr, rows 4 g + r),
    // epilogue by wave 0.  The barriers wait on LDS only (no vmcnt), so the prefetched
    // next step stays in flight.
    auto tile_end = [&](const Step& st) {
        // waves 1.. publish (wave 0 keeps its partial in registers: NW - 1 tiles of LDS,
        // which keeps config 4's staged gate/up launch within 64 KiB of dynamic LDS)
        if (wave > 0) {
#pragma unroll
            for (int b = 0; b < NB; b++)
                *reinterpret_cast<float4*>(&red[((wave - 1) * NB + b) * 256 + lane * 4]) =
                    make_float4(acc[b][0], acc[b][1], acc[b][2], acc[b][3]);
        }
        __syncthreads();
        if (wave == 0) {
            const int64_t n = st.tile * 16 + fr;
            float c[NB][4];
#pragma unroll
            for (int b = 0; b < NB; b++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                {
                    float t = acc[b][r];   // same order as before: wave 0, then 1 .. NW - 1
#pragma unroll
                    for (int w = 1; w < NW; w++) t += red[((w - 1) * NB + b) * 256 + lane * 4 + r];
                    c[b][r] = t;
                }
            if constexpr (WT != 0) {
#pragma unroll
                for (int b = 0; b < NB; b++)
#pragma unroll
                    for (int r = 0; r < 4; r++) c[b][r] *= st.wsc[b];
            }
            if (n < p.N) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int i = 4 * g + r;
                    if (i >= M) continue;
                    uint16_t* yr = p.y + (int64_t)i * p.ldy;
                    if constexpr (EPI == QIE_EPI_SWIGLU) {
                        const float gg = rbf(c[0][r]);
                        const float uu = rbf(c[1][r]);
                        const float av = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                        yr[n] = f2bf(uu * av);
                    } else if constexpr (EPI == QIE_EPI_RESIDUAL) {
                        yr[n] = f2bf(st.ep[r] + rbf(c[0][r]));
                    } else if constexpr (EPI == QIE_EPI_F32) {
                        reinterpret_cast<float*>(p.y)[(int64_t)i * p.ldy + n] = c[0][r];
                    } else {
                        const uint16_t o = f2bf(c[0][r] + st.ep[0]);
                        yr[n] = o;
                        if (p.keys) {
                            const unsigned long long kk = sel_key(bf2f(o), (uint32_t)(n + p.key_col0));
                            kbest[r] = kk > kbest[r] ? kk : kbest[r];
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int b = 0; b < NB; b++) acc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        __syncthreads();   // red[] reused by the next tile
    };

    // steady state issues unconditionally (a load under a branch costs a vmcnt(0) at the
    // join); the last one or two steps are peeled so nothing past step S - 1 is fetched
    Step sa, sb;
    issue(sa, 0);
    // ---------------- prologue: the M activation rows -> LDS (optionally RMS-normed).  It runs
    // AFTER the first step's weight loads are issued (weights do not depend on x), so the
    // weight stream's first HBM round trip overlaps the prologue's loads and reductions.
    if (XL && !QIE_DBG(p.dbg & 4)) {
        if (p.norm_w && !QIE_DBG(p.dbg & 1)) {
            // pass 1: every row's sum of squares at once (loads of all rows in flight,
            // clamped rows past M), ONE exchange — not a barrier pair per row
            float ss[16];
#pragma unroll
            for (int m = 0; m < 16; m++) ss[m] = 0.f;
            for (int64_t k = tid * 8; k < K; k += NW * 512) {
                uint4 v[16];
#pragma unroll
                for (int m = 0; m < 16; m++)
                    v[m] = *reinterpret_cast<const uint4*>(p.x + (int64_t)(m < M ? m : M - 1) * p.ldx + k);
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    if (m >= M) continue;   // uniform, ALU only (the loads are above)
                    float f[8];
                    unpack8(u32x4{v[m].x, v[m].y, v[m].z, v[m].w}, f);
#pragma unroll
                    for (int j = 0; j < 8; j++) ss[m] += f[j] * f[j];
                }
            }
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m >= M) continue;
                const float t = wave_sum(ss[m]);
                if (lane == 0) red[wave * 16 + m] = t;
            }
            __syncthreads();
            const bool hf = p.numerics == QIE_NUMERICS_HF;
            float rms[16], inv[16];
#pragma unroll
            for (int m = 0; m < 16; m++) {
                const int mm = m < M ? m : 0;
                float sm = red[mm];
#pragma unroll
                for (int w = 1; w < NW; w++) sm += red[16 * w + mm];
                rms[m] = sqrtf((sm / (float)K) + p.eps);
                inv[m] = 1.0f / rms[m];
            }
            // pass 2: all rows of a chunk at once (loads unconditional and clamped; the
            // per-row math under uniform branches).  REF's f / rms uses the FMA-corrected
            // quotient (Markstein): correctly rounded, i.e. equal to the division, for
            // normal operands — |f| outside [1e-30, 1e30] takes the real division.
            for (int64_t k = tid * 8; k < K; k += NW * 512) {
                const uint4 nw = *reinterpret_cast<const uint4*>(p.norm_w + k);
                uint4 v[16];
#pragma unroll
                for (int m = 0; m < 16; m++)
                    v[m] = *reinterpret_cast<const uint4*>(p.x + (int64_t)(m < M ? m : M - 1) * p.ldx + k);
                float wf[8];
                unpack8(u32x4{nw.x, nw.y, nw.z, nw.w}, wf);
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    if (m >= M) continue;
                    float f[8];
                    unpack8(u32x4{v[m].x, v[m].y, v[m].z, v[m].w}, f);
                    uint32_t o[4];
                    if (hf) {
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            o[j] = pack2(wf[2 * j] * rbf(f[2 * j] * inv[m]), wf[2 * j + 1] * rbf(f[2 * j + 1] * inv[m]));
                    } else {
                        float y[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const float q = f[j] * inv[m];
                            float d = fmaf(fmaf(-q, rms[m], f[j]), inv[m], q);
                            const float af = fabsf(f[j]);
                            if (af != 0.f && (af < 1e-30f || af > 1e30f)) d = f[j] / rms[m];
                            y[j] = d * wf[j];
                        }
#pragma unroll
                        for (int j = 0; j < 4; j++) o[j] = pack2(y[2 * j], y[2 * j + 1]);
                    }
                    *reinterpret_cast<uint4*>(xs + (int64_t)m * KP + k) = make_uint4(o[0], o[1], o[2], o[3]);
                }
            }
        } else {
            for (int m = 0; m < M; m++)
                for (int64_t k = tid * 8; k < K; k += NW * 512)
                    *reinterpret_cast<uint4*>(xs + (int64_t)m * KP + k) =
                        *reinterpret_cast<const uint4*>(p.x + (int64_t)m * p.ldx + k);
        }
        __syncthreads();
    }
    if (QIE_DBG(p.dbg & 2)) {
        if (tid == 0 && p.dbg == 0x7fffffff) p.y[0] = xs[0];
        return;
    }
    auto run = [&](const Step& st) {   // the full/tail choice is wave-uniform
        if (st.u0 + U <= ue) compute(st, true);
        else compute(st, false);
    };
    int64_t s = 0;
    for (; s + 2 < S; s += 2) {
        issue(sb, s + 1);
        run(sa);
        if (sa.last) tile_end(sa);
        issue(sa, s + 2);
        run(sb);
        if (sb.last) tile_end(sb);
    }
    if (S - s == 2) {
        issue(sb, s + 1);
        run(sa);
        if (sa.last) tile_end(sa);
        run(sb);
        tile_end(sb);
    } else {
        run(sa);
        tile_end(sa);
    }
    if constexpr (EPI == QIE_EPI_STORE) {
        if (p.keys && wave == 0) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                unsigned long long v = kbest[r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {   // max over the 16 columns of row 4 g + r
                    const unsigned long long t = __shfl_xor(v, o, 64);
                    v = t > v ? t : v;
                }
                if (fr == 0 && 4 * g + r < M && v) atomicMax(p.keys + 4 * g + r, v);
            }
        }
    }
}

// block size bound of the one-block-per-CU GEMV variant (9 waves: Qwen2-7B QKV; O / down use 7)
constexpr int kGemvBalancedThreads = 576;

static int env_int_gemv(const char* name, int dflt) { return dev_env(name, dflt); }

// UO: chunks per row in flight when K needs fewer than the default 8 wave-loads per row
// (0 = default).  A slot past K re-reads the row's last 16 B, so at K = 896 (Qwen2-0.5B)
// the default issued 8 loads per row of which 6 were duplicates.
template <int MT, int RPW, int EPI, int XCH, int WT, int UO = 0>
static int launch_gemv_t(const GemvParams& p, hipStream_t st, int blocks_per_cu) {
    constexpr int U = UO ? UO : ((RPW >= 4) ? 4 : 8);
    const void* fn = (const void*)gemv_kernel<MT, RPW, EPI, U, XCH, WT>;
    const size_t shm = (p.xlds ? (size_t)MT * p.K * 2 : 0) + 64;
    if (shm > 65536) {
        static bool raised = false;   // per instantiation
        if (!raised) {
            QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            raised = true;
        }
    }
    const int64_t n_blocks_needed = (p.n_tasks + 3) / 4;
    int64_t cap = (int64_t)device_cu_count() * blocks_per_cu;
    int64_t grid64 = std::max<int64_t>(1, std::min(n_blocks_needed, cap));
    if (blocks_per_cu == -2) {
        // Full-residency grid-stride grid (the SwiGLU default): every CU holds the same number
        // of blocks for the whole launch.  The balanced grid below gives every WAVE the same
        // task count but leaves CUs with 3 and 4 blocks (948 blocks at 4 per CU for Qwen2-7B
        // gate/up): in-graph gate/up 43.0 -> 42.2 us, 358.9 -> 361.5 tok/s (same box, A/B)
        static size_t cached_shm2 = 0;
        static int cached_nb2 = 0;
        int nb = cached_shm2 == shm ? cached_nb2 : 0;
        if (nb == 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, shm) != hipSuccess || nb < 1) nb = 2;
            cached_shm2 = shm;
            cached_nb2 = nb;
        }
        grid64 = std::max<int64_t>(1, std::min(n_blocks_needed, (int64_t)device_cu_count() * nb));
    } else if (blocks_per_cu <= 0) {
        // Balanced persistent grid (default): the grid is what fits on the chip at once, and
        // the task count per wave is made (nearly) equal — e.g. gate/up (18,944 tasks) on
        // 768 resident blocks: 7 rounds over 677 blocks instead of 4.6 rounds over 1024
        // blocks, whose last 0.6 round ran the chip at 60 % of its waves.
        static size_t cached_shm = 0;   // per instantiation: occupancy depends on LDS bytes
        static int cached_nb = 0;
        int nb = cached_shm == shm ? cached_nb : 0;
        if (nb == 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, shm) != hipSuccess || nb < 1) nb = 2;
            cached_shm = shm;
            cached_nb = nb;
        }
        cap = (int64_t)device_cu_count() * nb;
        const int64_t rounds = (p.n_tasks + 4 * cap - 1) / (4 * cap);
        grid64 = std::max<int64_t>(1, (p.n_tasks + 4 * rounds - 1) / (4 * rounds));
    }
    // One block per CU for mid-sized GEMVs (4..16 row tasks per CU: Qwen2-7B QKV 2,304, O and
    // down 1,792): 448 four-wave blocks on 256 CUs left 64 CUs with half the waves, and the
    // whole launch waited for the doubly loaded CUs.  Block = ceil(tasks / CUs) waves, so every
    // CU streams the same rows.  (SwiGLU and lm_head have > 9 tasks per CU: grid-stride.)
    int threads = 256;
    const int64_t cus = device_cu_count();
    // one row per wave: up to 16 waves per block (Qwen2-7B O / down: 14 one-row waves per CU)
    constexpr int LBB = RPW == 1 ? 1024 : kGemvBalancedThreads;
    if (MT == 1 && WT == 0 && EPI != QIE_EPI_SWIGLU && blocks_per_cu < 0 && p.n_tasks > 4 * cus &&
        p.n_tasks <= (LBB / 64) * cus &&
        env_int_gemv("QIE_GEMV_BALANCED", 1) != 0) {
        const int64_t nw = (p.n_tasks + cus - 1) / cus;
        threads = (int)(64 * nw);
        grid64 = (p.n_tasks + nw - 1) / nw;
    }
    const unsigned grid = (unsigned)grid64;
    if (threads > 256) {
        if constexpr (MT == 1 && WT == 0 && EPI != QIE_EPI_SWIGLU) {
            const void* fb = (const void*)gemv_kernel<MT, RPW, EPI, U, XCH, WT, LBB>;
            if (shm > 65536) {
                static bool raised_b = false;
                if (!raised_b) {
                    QIE_HIP(hipFuncSetAttribute(fb, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                    raised_b = true;
                }
            }
            hipLaunchKernelGGL((gemv_kernel<MT, RPW, EPI, U, XCH, WT, LBB>), dim3(grid), dim3(threads), shm, st, p);
            QIE_LAUNCH_CHECK();
            return 0;
        }
    }
    hipLaunchKernelGGL((gemv_kernel<MT, RPW, EPI, U, XCH, WT>), dim3(grid), dim3(threads), shm, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

template <int MT, int XCH, int WT = 0, int UO = 0>
static int launch_gemv_m(const GemvParams& p, int rpw, int epi, hipStream_t st, int bpc) {
    if constexpr (MT == 1 && XCH == 1 && WT == 0) {   // one row per wave (O / down, x beside the weights)
        if (rpw == 1 && epi == QIE_EPI_RESIDUAL) return launch_gemv_t<1, 1, QIE_EPI_RESIDUAL, 1, 0, UO>(p, st, bpc);
        if (rpw == 1 && epi == QIE_EPI_STORE) return launch_gemv_t<1, 1, QIE_EPI_STORE, 1, 0, UO>(p, st, bpc);
    }
    if (epi == QIE_EPI_SWIGLU) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_SWIGLU, XCH, WT, UO>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_SWIGLU, XCH, WT, UO>(p, st, bpc);
    } else if (epi == QIE_EPI_RESIDUAL) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_RESIDUAL, XCH, WT, UO>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_RESIDUAL, XCH, WT, UO>(p, st, bpc);
    } else if (epi == QIE_EPI_F32) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_F32, XCH, WT, UO>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_F32, XCH, WT, UO>(p, st, bpc);
    }
    return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_STORE, XCH, WT, UO>(p, st, bpc)
                    : launch_gemv_t<MT, 2, QIE_EPI_STORE, XCH, WT, UO>(p, st, bpc);
}
// x-first prologue variants (MT = 1 only): XCH 2048-element x chunks per thread
static int launch_gemv_1(const GemvParams& p, int rpw, int epi, hipStream_t st, int bpc, int xch) {
    // Chunks in flight per row sized to K (bf16 wave-loads per row n), so no load slot
    // re-reads the row's tail: n <= 2 (Qwen2-0.5B, K = 896): 2 instead of 8 slots, 6 of
    // them duplicates — lm_head 72.1 -> 47.4 us, gate/up 8.4 -> 6.3, decode 1,283 -> 1,471
    // tok/s; n = 7 (Qwen2-7B, K = 3,584): 7 instead of 8 — gate/up 44.2 -> 42.9, QKV
    // 9.67 -> 9.41 us, 349 -> 354 tok/s, but lm_head 166 -> 175 us (25 row tasks per wave:
    // there the 8th slot's duplicate costs less than the bytes in flight it drops), so the
    // vocabulary projection keeps 8; n = 10 (Qwen3-14B, K = 5,120): 5 per pass, two passes.
    const int64_t n = (p.K + 511) / 512;   // bf16 wave-loads per row
    const bool vocab = p.n_tasks * rpw >= 65536;
    const int64_t ub = (n + (n + 7) / 8 - 1) / ((n + 7) / 8);   // balanced slots per pass (<= 8)
    if (xch == 4) {   // fused norm, normalised x in every wave's registers
        if (n <= 2) return launch_gemv_m<1, 4, 0, 2>(p, rpw, epi, st, bpc);
        if (n == 7 && !vocab) return launch_gemv_m<1, 4, 0, 7>(p, rpw, epi, st, bpc);
        return launch_gemv_m<1, 4, 0, 8>(p, rpw, epi, st, bpc);
    }
    if (xch == 3) {   // fused norm, x in registers: one batch of wave-loads covers a row
        if (n <= 2) return launch_gemv_m<1, 3, 0, 2>(p, rpw, epi, st, bpc);
        if (n == 7 && !vocab) return launch_gemv_m<1, 3, 0, 7>(p, rpw, epi, st, bpc);
        return launch_gemv_m<1, 3, 0, 8>(p, rpw, epi, st, bpc);
    }
    if (xch == 2 && n <= 2) return launch_gemv_m<1, 2, 0, 2>(p, rpw, epi, st, bpc);
    if (xch == 2 && n == 7 && !vocab) return launch_gemv_m<1, 2, 0, 7>(p, rpw, epi, st, bpc);
    if (xch == 5 && (n == 9 || n == 10) && !vocab) return launch_gemv_m<1, 5, 0, 5>(p, rpw, epi, st, bpc);
    // K <= 20,480 without a norm (Qwen3-14B O at K = 5,120: 2 x 5; down at K = 17,408: 5 x 7)
    if (xch == 10 && ub == 5 && !vocab) return launch_gemv_m<1, 10, 0, 5>(p, rpw, epi, st, bpc);
    if (xch == 10 && ub == 7 && !vocab) return launch_gemv_m<1, 10, 0, 7>(p, rpw, epi, st, bpc);
    if (xch == 1 && n == 7) return launch_gemv_m<1, 1, 0, 7>(p, rpw, epi, st, bpc);
    if (xch == 1) return launch_gemv_m<1, 1>(p, rpw, epi, st, bpc);
    if (xch == 2) return launch_gemv_m<1, 2>(p, rpw, epi, st, bpc);
    if (xch == 5) return launch_gemv_m<1, 5>(p, rpw, epi, st, bpc);
    if (xch == 10) return launch_gemv_m<1, 10>(p, rpw, epi, st, bpc);
    return launch_gemv_m<1, 0>(p, rpw, epi, st, bpc);
}

int gemm(const qie_linear_args* a, hipStream_t st);

static int env_int(const char* name, int dflt) { return dev_env(name, dflt); }

constexpr size_t kGemvLdsCap = 96 * 1024;
constexpr size_t kSkinnyLdsCap = 120 * 1024;

template <int EPI, int WT, int XL, int NW, int UO = 0>
static int launch_skinny_x(const GemvParams& p, hipStream_t st) {
    constexpr int NB = EPI == QIE_EPI_SWIGLU ? 2 : 1;
    const void* fn = (const void*)skinny_mfma_kernel<EPI, WT, XL, NW, UO>;
    // reduction tiles: NW - 1 partial C tiles per B tile (>= 64 floats for the norm prologue)
    const size_t shm = (p.xlds ? (size_t)p.M * (p.K + 8) * 2 : 0) + (size_t)std::max(NW - 1, 1) * NB * 256 * 4;
    if (shm > 65536) {
        static bool raised = false;
        if (!raised) {
            QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            raised = true;
        }
    }
    const int64_t n_tiles = (p.N + 15) / 16;
    // as many blocks as are resident at once (LDS-limited when the M rows are staged)
    static size_t cached_shm = 0;
    static int cached_nb = 0;
    if (cached_shm != shm || cached_nb == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, NW * 64, shm) != hipSuccess || nb < 1) nb = 1;
        cached_shm = shm;
        cached_nb = nb;
    }
    // dev A/B: blocks per CU (0: all resident — config 4's tiled lm_head 100.1 µs; caps 1 / 2 / 3 / 6
    // measured 101.9 / 100.5 / 111.0 / 127.7)
    const int cap = dev_env("QIE_SKINNY_BPC", 0);
    const unsigned grid = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>(n_tiles, (int64_t)device_cu_count() * (cap > 0 ? cap : cached_nb)));
    hipLaunchKernelGGL((skinny_mfma_kernel<EPI, WT, XL, NW, UO>), dim3(grid), dim3(NW * 64), shm, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}
// 4 waves per block: 8 (2,304 waves for Qwen2-7B QKV) measured 1-9 % slower at config 4,
// 16 spills (128 VGPRs at 1,024 threads)
template <int EPI, int WT>
static int launch_skinny_t(const GemvParams& p, hipStream_t st) {
    if constexpr (WT == 1) {
        // fp8: 7 units per step where a wave's K range is 7 or 14 units (Qwen2-7B, K = 3,584:
        // 2 steps of 7 instead of 4 of 4 / 2 of 8 with two dead units).  Config 4 (fp8, B = 8):
        // gate/up 36.2 -> 35.2, O 8.4 -> 7.45, lm_head 129 -> 122 us, 2,509 -> 2,535 tok/s
        const int64_t uw = (p.K / 64 + 3) / 4;
        if (uw == 7 || uw == 14)
            return p.xlds ? launch_skinny_x<EPI, WT, 1, 4, 7>(p, st) : launch_skinny_x<EPI, WT, 0, 4, 7>(p, st);
    }
    return p.xlds ? launch_skinny_x<EPI, WT, 1, 4>(p, st) : launch_skinny_x<EPI, WT, 0, 4>(p, st);
}

static int launch_skinny(const GemvParams& p, int epi, bool fp8w, hipStream_t st) {
    if (fp8w) {
        if (epi == QIE_EPI_SWIGLU) return launch_skinny_t<QIE_EPI_SWIGLU, 1>(p, st);
        if (epi == QIE_EPI_RESIDUAL) return launch_skinny_t<QIE_EPI_RESIDUAL, 1>(p, st);
        if (epi == QIE_EPI_F32) return launch_skinny_t<QIE_EPI_F32, 1>(p, st);
        return launch_skinny_t<QIE_EPI_STORE, 1>(p, st);
    }
    if (epi == QIE_EPI_SWIGLU) return launch_skinny_t<QIE_EPI_SWIGLU, 0>(p, st);
    if (epi == QIE_EPI_RESIDUAL) return launch_skinny_t<QIE_EPI_RESIDUAL, 0>(p, st);
    if (epi == QIE_EPI_F32) return launch_skinny_t<QIE_EPI_F32, 0>(p, st);
    return launch_skinny_t<QIE_EPI_STORE, 0>(p, st);
}
static bool K_fits(int64_t K, int xch) { return K <= 2048 * (int64_t)xch && K % 8 == 0; }

// RoPE for the next gemv() call only (gemv_rope); thread-local: engines on other host
// threads (tensor-parallel ranks) enqueue concurrently
struct RopeArgs {
    const int32_t* pos = nullptr;
    const float* cs = nullptr;
    const float* sn = nullptr;
    int hd = 0;
    int64_t rows = 0;
};
static thread_local RopeArgs g_rope;
static thread_local const PeerPush* g_push = nullptr;
static thread_local bool g_push_taken = false;
void set_gemv_push(const PeerPush* pp) {
    g_push = pp;
    g_push_taken = false;
}
bool gemv_push_taken() { return g_push_taken; }

int gemv(const qie_linear_args* a, hipStream_t st);

// Decode QKV projection (M = 1, REF numerics, no qk-norm) with the interleaved RoPE of its q
// and k rows fused into the STORE epilogue (RoPE.cu:6-22 on the projection's bf16 output):
// the decode attention then takes q / k as they are (qie_attention_decode, QIE_ATTN_PREROPED).
int gemv_rope(const qie_linear_args* a, const int32_t* pos, const float* cs, const float* sn, int hd,
              int64_t rows, hipStream_t st) {
    QIE_REQUIRE(a->M == 1 && a->epilogue == QIE_EPI_STORE && rows % 2 == 0 && hd % 2 == 0 && pos && cs && sn,
                "gemv_rope: M = 1 STORE projections only");
    g_rope = RopeArgs{pos, cs, sn, hd, rows};
    const int rc = gemv(a, st);
    g_rope = RopeArgs{};
    return rc;
}

bool dec8_applies(const qie_linear_args* a);
int dec8_linear(const qie_linear_args* a, hipStream_t st, bool* done);

int gemv(const qie_linear_args* a, hipStream_t st) {
    // fp8 weights, 2..16 rows, K a whole number of per-wave slices (or split-K): k_decode_fp8.hip
    if (dec8_applies(a)) {
        bool done = false;
        const int rc = dec8_linear(a, st, &done);
        if (done) return rc;
    }
    GemvParams p;
    p.x = (const uint16_t*)a->x;
    p.ldx = a->ldx;
    p.w0 = (const uint16_t*)a->w[0];
    p.w1 = (const uint16_t*)a->w[1];
    p.w2 = (const uint16_t*)a->w[2];
    p.b0 = (const uint16_t*)a->bias[0];
    p.b1 = (const uint16_t*)a->bias[1];
    p.b2 = (const uint16_t*)a->bias[2];
    p.n0 = a->seg_rows[0];
    p.n01 = a->seg_rows[0] + a->seg_rows[1];
    p.K = a->K;
    p.N = a->N;
    p.y = (uint16_t*)a->y;
    p.ldy = a->ldy;
    p.norm_w = (const uint16_t*)a->norm_w;
    p.eps = a->norm_eps;
    p.numerics = a->numerics;
    p.M = (int)a->M;
    p.keys = (unsigned long long*)a->argmax_keys;
    p.key_col0 = a->key_col0;
    p.dbg = 0;
    p.rope_pos = g_rope.pos;
    p.rope_cs = g_rope.cs;
    p.rope_sn = g_rope.sn;
    p.rope_hd = g_rope.hd;
    p.rope_rows = g_rope.rows;
    p.epre = env_int("QIE_GEMV_EPRE", 1);
    p.mkdiv = env_int("QIE_GEMV_MKDIV", 0);
    // 16-row tiled fp8 weights the batched-decode kernel did not take (the vocabulary
    // projection): the skinny kernel reads them, at any 1 <= M <= 16 (qie_linear checked the shape)
    p.t16 = (a->flags & QIE_LINEAR_FP8_T16) ? 1 : 0;
    p.push = PeerPush{};
    g_push_taken = false;
    if ((a->M >= 2 || p.t16) && a->M <= 16 && (p.t16 || env_int("QIE_SKINNY_MFMA", 1) != 0)) {
        const bool fp8w = (a->flags & QIE_LINEAR_FP8) != 0;
        const int kstep = 64;
        const bool lds_ok = (size_t)a->M * (a->K + 8) * 2 <= kSkinnyLdsCap;
        QIE_REQUIRE(!p.t16 || (fp8w && a->K % kstep == 0 && (lds_ok || !a->norm_w)),
                    "qie_linear: tiled fp8 weights: the skinny kernel cannot take M=%lld K=%lld", (long long)a->M,
                    (long long)a->K);
        if (a->K % kstep == 0 && (lds_ok || !a->norm_w)) {
            p.M = (int)a->M;
            // Stage the M rows in LDS only when the norm is fused (it needs them) or a block
            // serves several column tiles (gate/up, lm_head: the copy is amortised); with
            // about one tile per CU (QKV, O, down) each wave loads its A fragments from L2
            // with its weight steps instead of a 57-KB copy + barrier per block (config 4,
            // fp8: O 9.7 -> 7.8 us, down 26.4 -> 24.6; bf16 O 11.6 -> 10.1, QKV 16.5 -> 15.3)
            const int64_t n_tiles = (a->N + 15) / 16;
            p.xlds = lds_ok && (a->norm_w || n_tiles > 2 * (int64_t)device_cu_count()) ? 1 : 0;
            // Without a fused norm the staged copy is only an optimisation: keep the launch's
            // dynamic LDS within the default 64 KiB (no raised kernel attribute).  r02's config-4
            // gate/up node (8 rows x 3,592 + two 4-KiB reduction tiles per wave = 65,664 B) was
            // the one decode-graph node above it, and rocprofv3's kernel trace crashed on that
            // graph only; with NW - 1 reduction tiles it is 63,616 B and stays staged.
            const size_t staged = (size_t)a->M * (a->K + 8) * 2 + (a->epilogue == QIE_EPI_SWIGLU ? 2 : 1) * 3072;
            if (p.xlds && !a->norm_w && staged > 65536 && env_int("QIE_SKINNY_LDS64", 1) != 0) p.xlds = 0;
            const int fx = env_int("QIE_SKINNY_XL", -1);
            if (fx >= 0) p.xlds = fx && lds_ok ? 1 : 0;
            p.dbg = env_int("QIE_SKINNY_DBG", 0);
            return launch_skinny(p, a->epilogue, fp8w, st);
        }
    }
    if (a->M > 8) return gemm(a, st);   // 9..16 rows the skinny kernel could not take
    if (g_push && a->M == 1 && a->epilogue == QIE_EPI_F32) {   // every M = 1 launch below is gemv_kernel
        p.push = *g_push;
        g_push_taken = true;
    }
    p.dbg = a->M == 1 ? env_int("QIE_GEMV_DBG", 0) : 0;   // dev timing experiments (1 no norm, 2 no bias)
    const int MT = a->M <= 1 ? 1 : a->M <= 2 ? 2 : a->M <= 4 ? 4 : 8;
    p.xlds = ((size_t)MT * a->K * 2 <= kGemvLdsCap) ? 1 : 0;
    QIE_REQUIRE(p.xlds || !p.norm_w,
                "qie_linear: fused RMSNorm needs M*K*2 <= %zu bytes (M=%lld K=%lld)", kGemvLdsCap,
                (long long)a->M, (long long)a->K);
    // Rows per wave: 4 while the grid still has >= 2 waves per SIMD of work.
    const int cus = device_cu_count();
    const int64_t rows = a->epilogue == QIE_EPI_SWIGLU ? 2 * a->N : a->N;
    // Rows per wave: 2 (measured faster than 4 for every Qwen2-7B decode GEMV on
    // MI355X: down 23.7 vs 28.0 us, qkv 9.7 vs 10.9, o 6.6 vs 7.7, gate/up 42.9 vs 43.8).
    int rpw = env_int("QIE_GEMV_RPW", 2);
    // (dev A/B) vocabulary rows: 4 rows per wave measured 165.9 vs 164.8 µs at Qwen2-7B,
    // 53.4 vs 48.7 at Qwen2-0.5B
    if (MT == 1 && rows >= 65536) rpw = env_int("QIE_GEMV_RPW_LM", rpw);
    if (rpw != 2 && rpw != 4) rpw = 2;
    p.n_tasks = (rows + rpw - 1) / rpw;
    // Grid (QIE_GEMV_BLOCKS_PER_CU): default (auto) = one block per CU with ceil(tasks / CUs)
    // waves where 4..9 tasks per CU (Qwen2-7B QKV, O, down), else the occupancy-balanced
    // persistent grid (lm_head 169 vs 183 us, gate/up 43.1 vs 43.5 against a cap of 8 blocks
    // per CU); 0 = always the occupancy grid; N > 0 = cap of N blocks per CU.
    int bpc = env_int("QIE_GEMV_BLOCKS_PER_CU", -1);
    // x-first prologue + cross-task weight prefetch (QIE_GEMV_XFIRST, MT = 1).  A first
    // attempt that issued the weights BEFORE x was slower everywhere (qkv 11.4 vs 9.4 us):
    // x then queued behind the weights in the in-order vmcnt.
    if (a->flags & QIE_LINEAR_FP8) {
        QIE_REQUIRE(a->K % 16 == 0, "qie_linear: fp8 weights need K %% 16 == 0 (K=%lld)", (long long)a->K);
        switch (MT) {
            case 1: return launch_gemv_m<1, 0, 1>(p, rpw, a->epilogue, st, bpc);
            case 2: return launch_gemv_m<2, 0, 1>(p, rpw, a->epilogue, st, bpc);
            case 4: return launch_gemv_m<4, 0, 1>(p, rpw, a->epilogue, st, bpc);
            default: return launch_gemv_m<8, 0, 1>(p, rpw, a->epilogue, st, bpc);
        }
    }
    int xch = 0;
    // The x-first variants with a fused RMSNorm are XCH 2 and 5 (the norm weights ride along
    // with x); XCH 10 (down, K = 18,944) stages x only — a fused norm there would be dropped,
    // so a normed K > 10,240 takes the generic prologue.
    if (MT == 1 && p.xlds && p.M == 1 && env_int("QIE_GEMV_XFIRST", 1) != 0) {
        if (p.norm_w) xch = K_fits(a->K, 2) ? 2 : (K_fits(a->K, 5) ? 5 : 0);
        else xch = K_fits(a->K, 2) ? 2 : (K_fits(a->K, 10) ? 10 : 0);
    }
    // Fused norm with a per-wave sum of squares (XCH 3) where one batch of <= 8 wave-loads
    // covers a row (K <= 4,096, K % 8 == 0: Qwen2-7B QKV / gate/up / lm_head at K = 3,584,
    // Qwen2-0.5B at 896): no block reduction, one barrier before the weight stream.
    // Measured (tools/ubench.py, Qwen2-7B): lm_head 175.3 -> 167.4 us; QKV (9.14 vs 9.67) and
    // gate/up (42.7 vs 43.8) are faster with the x-first prologue's one-chunk-per-thread x
    // loads, so only the vocabulary projection takes it.
    const bool vocab_rows = rows >= 65536;
    if (MT == 1 && p.M == 1 && p.norm_w && a->K % 8 == 0 && a->K <= 4096 &&
        env_int("QIE_GEMV_XREG", vocab_rows ? 1 : 0) != 0) {
        xch = 3;
    }
    // Normalised x in every wave's registers (XCH 4): no LDS image, no barrier.  Default for
    // gate/up (5 row tasks per wave reuse it): 361.5 -> 362.7 tok/s at Qwen2-7B; the QKV
    // projection (one task per wave) pays the per-wave divisions on its critical path:
    // 9.98 -> 14.6 us (dev knobs QIE_GEMV_XREG4 / _LM / _SW)
    if (MT == 1 && p.M == 1 && p.norm_w && a->K % 8 == 0 && a->K <= 4096 &&
        env_int(a->epilogue == QIE_EPI_SWIGLU ? "QIE_GEMV_XREG4_SW" : (vocab_rows ? "QIE_GEMV_XREG4_LM" : "QIE_GEMV_XREG4"),
                a->epilogue == QIE_EPI_SWIGLU ? 1 : 0) != 0) {
        xch = 4;
        p.xlds = 0;
    }
    // gate/up grid: full residency, grid-stride (-2, launch_gemv_t); QIE_GEMV_SWIGLU_BPC = N > 0
    // caps N blocks per CU, -1 the balanced grid (dev A/B)
    //
    // Round 5, grid caps measured per shape (same box, interleaved, in the graph: tools/ab_decode.py;
    // outputs bit-identical — the grid only changes which wave takes which row task):
    //  * gate/up, Qwen2-7B (K 3,584, 74 row tasks per CU; 198 VGPRs, 2 resident blocks per CU):
    //    6 blocks per CU 42.7 -> 41.3 µs, 361.8 -> 366.7 tok/s — a sharp optimum (5: 357.4,
    //    8: 358.1, 10: 343.2; the full-residency grid, 2 per CU, 361.8);
    //  * gate/up, Qwen2-0.5B (K 896, 19 tasks per CU; 62 VGPRs): 3 per CU 6.48 -> 5.22 µs,
    //    1,484 -> 1,542 tok/s (2: 1,543, 4: 1,511, 5: 1,483);
    //  * lm_head (vocabulary rows, occupancy-balanced grid otherwise): K 896 5 per CU
    //    53.4 -> 48.8 µs; K 3,584 2 per CU 167.3 -> 164.7 µs.
    // Shapes outside those ranges keep the former grids (unmeasured there).
    if (a->epilogue == QIE_EPI_SWIGLU && MT == 1 && bpc < 0) {
        const int64_t tpc = p.n_tasks / cus;
        int dflt = -2;
        if (a->K <= 1024 && tpc <= 32) dflt = 3;
        else if (a->K >= 3072 && a->K <= 4096 && tpc >= 64 && tpc <= 96) dflt = 6;
        bpc = env_int("QIE_GEMV_SWIGLU_BPC", dflt);
    }
    if (vocab_rows && MT == 1 && bpc < 0)
        bpc = env_int("QIE_GEMV_LM_BPC", a->K <= 1024 ? 5 : (a->K <= 4096 ? 2 : -1));
    // The normed STORE projection (QKV), Qwen2-7B (K 3,584, 9 row tasks per CU): 2 blocks of 4
    // waves per CU instead of one 9-wave block, 9.77 -> 9.26 µs, 367.4 -> 369.4 tok/s (1: 357.2,
    // 3: 364.8, 4: 364.8).  The fused norm's sum of squares is then reduced over 256 threads
    // instead of 576 (another fp32 order of the same sum; the parity tests bound it).
    // Qwen2-0.5B's QKV: equal at 1-3 per CU, kept.
    // (dev A/B) residual projections (O, down): caps 3 / 5 / 6 / 8 per CU all ran Qwen2-7B at
    // 363.4-363.5 vs 369.6 tok/s on their one-block-per-CU layout; 0.5B equal

    if (MT == 1 && a->epilogue == QIE_EPI_RESIDUAL && bpc < 0) bpc = env_int("QIE_GEMV_RES_BPC", -1);
    if (!vocab_rows && MT == 1 && p.norm_w && a->epilogue == QIE_EPI_STORE && bpc < 0) {
        const int64_t tpc = p.n_tasks / cus;
        bpc = env_int("QIE_GEMV_QKV_BPC", a->K >= 3072 && a->K <= 4096 && tpc >= 6 && tpc <= 12 ? 2 : -1);
    }
    // Batch-1 GEMVs without a fused norm on the one-block-per-CU grid (one row task per
    // wave: Qwen2-7B O, down) read x from L2 beside each weight chunk (XCH = 1) instead of
    // staging it in LDS behind a barrier: Qwen2-7B decode 355 -> 358 tok/s (two A/B rounds),
    // in-graph down 24.5 -> 23.5 us, O 7.3 -> 7.05.  Where a wave walks several row tasks
    // (Qwen3-14B O / down, 10 per CU; Qwen2-0.5B) x would be re-read per task: O 13.1 ->
    // 16.5, down 32.9 -> 39.7 us at 14B, so those keep the staged copy.
    // (the condition is launch_gemv_t's one-block-per-CU grid)
    if (MT == 1 && p.M == 1 && !p.norm_w && !(a->flags & QIE_LINEAR_FP8) && a->epilogue != QIE_EPI_SWIGLU &&
        a->K % 8 == 0 && bpc < 0 && p.n_tasks > 4 * (int64_t)cus &&
        p.n_tasks <= (kGemvBalancedThreads / 64) * (int64_t)cus && env_int_gemv("QIE_GEMV_BALANCED", 1) != 0) {
        xch = 1;
        p.xlds = 0;
        // one row per wave, up to 16 waves per CU, where x is short (each wave re-reads all of x
        // from L2): Qwen2-7B O 6.68 -> 6.45 us; down (x 37.9 KB, K = 18,944) doubled its L2
        // traffic for x that way (23.3 -> 25.1 us), so it keeps two rows per wave
        if ((a->epilogue == QIE_EPI_RESIDUAL || a->epilogue == QIE_EPI_STORE) && rows <= 16 * (int64_t)cus &&
            a->K <= 4096 && env_int("QIE_GEMV_RPW1", 1) != 0) {
            rpw = 1;
            p.n_tasks = rows;
        }
    }
    QIE_REQUIRE(!(xch == 10 && p.norm_w), "qie_linear: internal: fused norm routed to a variant without one");
    switch (MT) {
        case 1: return launch_gemv_1(p, rpw, a->epilogue, st, bpc, xch);
        case 2: return launch_gemv_m<2, 0>(p, rpw, a->epilogue, st, bpc);
        case 4: return launch_gemv_m<4, 0>(p, rpw, a->epilogue, st, bpc);
        default: return launch_gemv_m<8, 0>(p, rpw, a->epilogue, st, bpc);
    }
}

}  // namespace qie
