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
};

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

template <int MT, int RPW, int EPI, int U, int XCH, int WT>
__global__ __launch_bounds__(256) void gemv_kernel(GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
    float* red = reinterpret_cast<float*>(smem + (p.xlds ? (size_t)MT * p.K * 2 : 0));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t K = p.K;
    constexpr int EB = WT ? 1 : 2;     // bytes per weight
    constexpr int EL = 16 / EB;        // weights per 16-byte lane load
    constexpr int WS = 64 * EL;        // weights per wave-load

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
    auto load_chunk = [&](const u32x4* const (&wr)[RPW], int64_t k0, u32x4 (&wv)[U][RPW]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t k = k0 + u * WS;
#pragma unroll
            for (int i = 0; i < RPW; i++)   // unconditional (clamped) loads: see below
                wv[u][i] = __builtin_nontemporal_load(wr[i] + ((k < K ? k : K - EL) / EL));
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
                        const uint4 xv = x_at(m, k);
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

    const int64_t tstride = (int64_t)gridDim.x * 4;
    const int64_t task0 = (int64_t)blockIdx.x * 4 + wave;
    const u32x4* wr[RPW];
    u32x4 wv[U][RPW];
    constexpr bool PF = XCH > 0;

    if constexpr (XCH > 0) {
        // ---------------- x-first prologue (MT = 1, x staged in LDS, K <= 2048 * XCH; the
        // host guarantees it).  Order of issue: this thread's x chunks (+ norm weights),
        // then the first weight chunk of the wave's first task, THEN the x arithmetic — so
        // the weight stream's first HBM round trip overlaps the x round trip instead of
        // following it (vmcnt retires in order: x must be issued first).
        constexpr int NV = XCH <= 2 ? XCH : 1;   // norm weights: fused-norm variants only (XCH <= 2)
        const bool nrm = NV == XCH && p.norm_w != nullptr;
        uint4 xv[XCH], nv[NV];
#pragma unroll
        for (int c = 0; c < XCH; c++) {
            const int64_t k = (int64_t)tid * 8 + c * 2048;
            const int64_t kc = k < K ? k : K - 8;   // clamped: loads stay unconditional
            xv[c] = *reinterpret_cast<const uint4*>(p.x + kc);
            if (c < NV) nv[c] = *reinterpret_cast<const uint4*>((nrm ? p.norm_w : p.x) + kc);
        }
        __builtin_amdgcn_sched_barrier(0);
        // unconditional (a wave without a task re-reads the last row): a load under a
        // branch makes the vmcnt bookkeeping at the join wait for everything
        task_ptrs(task0 < p.n_tasks ? task0 : p.n_tasks - 1, wr);
        load_chunk(wr, (int64_t)lane * EL, wv);
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
                if ((int64_t)tid * 8 + c * 2048 >= K) continue;
                float f[8];
                unpack8(u32x4{xv[c].x, xv[c].y, xv[c].z, xv[c].w}, f);
#pragma unroll
                for (int j = 0; j < 8; j++) ss += f[j] * f[j];
            }
            ss = wave_sum(ss);
            if (lane == 0) red[wave] = ss;
            __syncthreads();
            ss = red[0] + red[1] + red[2] + red[3];
            const float rms = sqrtf((ss / (float)K) + p.eps);
            const float inv = 1.0f / rms;
            const bool hf = p.numerics == QIE_NUMERICS_HF;
#pragma unroll
            for (int c = 0; c < XCH; c++) {
#pragma clang fp contract(off)
                const int64_t k = (int64_t)tid * 8 + c * 2048;
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
                const int64_t k = (int64_t)tid * 8 + c * 2048;
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
                for (int64_t k = tid * 8; k < K; k += 2048)
                    *reinterpret_cast<uint4*>(xo + k) = make_uint4(0, 0, 0, 0);
                continue;
            }
            if (p.norm_w) {
                float ss = 0.f;
                for (int64_t k = tid * 8; k < K; k += 2048) {
                    uint4 v = *reinterpret_cast<const uint4*>(xr + k);
                    float f[8];
                    unpack8(u32x4{v.x, v.y, v.z, v.w}, f);
#pragma unroll
                    for (int j = 0; j < 8; j++) ss += f[j] * f[j];
                }
                ss = wave_sum(ss);
                if (lane == 0) red[wave] = ss;
                __syncthreads();
                ss = red[0] + red[1] + red[2] + red[3];
                __syncthreads();
                const float rms = sqrtf((ss / (float)K) + p.eps);
                const float inv = 1.0f / rms;
                const bool hf = p.numerics == QIE_NUMERICS_HF;
                for (int64_t k = tid * 8; k < K; k += 2048) {
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
                for (int64_t k = tid * 8; k < K; k += 2048)
                    *reinterpret_cast<uint4*>(xo + k) = *reinterpret_cast<const uint4*>(xr + k);
            }
        }
        __syncthreads();
    }

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
                    float* yf = reinterpret_cast<float*>(p.y) + (int64_t)m * p.ldy;
#pragma unroll
                    for (int i = 0; i < RPW; i++)
                        if (col[i] < p.N) yf[col[i]] = acc[m][i];
                } else if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        if (col[i] >= p.N) continue;
                        yr[col[i]] = f2bf(bf2f(yr[col[i]]) + rbf(acc[m][i]));
                    }
                } else {
                    unsigned long long best = kbest[m];
#pragma unroll
                    for (int i = 0; i < RPW; i++) {
                        const int64_t c = col[i];
                        if (c >= p.N) continue;
                        float v = acc[m][i];
                        const uint16_t* b = c < p.n0 ? p.b0 : (c < p.n01 ? p.b1 : p.b2);
                        if (b) {
                            int64_t bi = c < p.n0 ? c : (c < p.n01 ? c - p.n0 : c - p.n01);
                            v = v + bf2f(b[bi]);
                        }
                        uint16_t o = f2bf(v);
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
            __shared__ unsigned long long kb_s[4][MT];
            if (lane == 0) {
#pragma unroll
                for (int m = 0; m < MT; m++) kb_s[wave][m] = kbest[m];
            }
            __syncthreads();
            if (tid < MT && tid < p.M) {
                unsigned long long b = kb_s[0][tid];
#pragma unroll
                for (int w = 1; w < 4; w++) b = kb_s[w][tid] > b ? kb_s[w][tid] : b;
                if (b) atomicMax(p.keys + tid, b);
            }
        }
    }
}

template <int MT, int RPW, int EPI, int XCH, int WT>
static int launch_gemv_t(const GemvParams& p, hipStream_t st, int blocks_per_cu) {
    constexpr int U = (RPW >= 4) ? 4 : 8;
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
    if (blocks_per_cu <= 0) {
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
    const unsigned grid = (unsigned)grid64;
    hipLaunchKernelGGL((gemv_kernel<MT, RPW, EPI, U, XCH, WT>), dim3(grid), dim3(256), shm, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

template <int MT, int XCH, int WT = 0>
static int launch_gemv_m(const GemvParams& p, int rpw, int epi, hipStream_t st, int bpc) {
    if (epi == QIE_EPI_SWIGLU) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_SWIGLU, XCH, WT>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_SWIGLU, XCH, WT>(p, st, bpc);
    } else if (epi == QIE_EPI_RESIDUAL) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_RESIDUAL, XCH, WT>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_RESIDUAL, XCH, WT>(p, st, bpc);
    } else if (epi == QIE_EPI_F32) {
        return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_F32, XCH, WT>(p, st, bpc)
                        : launch_gemv_t<MT, 2, QIE_EPI_F32, XCH, WT>(p, st, bpc);
    }
    return rpw >= 4 ? launch_gemv_t<MT, 4, QIE_EPI_STORE, XCH, WT>(p, st, bpc)
                    : launch_gemv_t<MT, 2, QIE_EPI_STORE, XCH, WT>(p, st, bpc);
}
// x-first prologue variants (MT = 1 only): XCH 2048-element x chunks per thread
static int launch_gemv_1(const GemvParams& p, int rpw, int epi, hipStream_t st, int bpc, int xch) {
    if (xch == 2) return launch_gemv_m<1, 2>(p, rpw, epi, st, bpc);
    if (xch == 10) return launch_gemv_m<1, 10>(p, rpw, epi, st, bpc);
    return launch_gemv_m<1, 0>(p, rpw, epi, st, bpc);
}

static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}

constexpr size_t kGemvLdsCap = 96 * 1024;
static bool K_fits(int64_t K, int xch) { return K <= 2048 * (int64_t)xch && K % 8 == 0; }

int gemv(const qie_linear_args* a, hipStream_t st) {
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
    if (rpw != 2 && rpw != 4) rpw = 2;
    (void)cus;
    p.n_tasks = (rows + rpw - 1) / rpw;
    // blocks per CU cap of the grid (8: measured best for every Qwen2-7B decode GEMV but lm_head);
    // 0 = the occupancy-balanced persistent grid (QIE_GEMV_BLOCKS_PER_CU=0)
    const int bpc = std::max(0, env_int("QIE_GEMV_BLOCKS_PER_CU", 8));
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
    if (MT == 1 && p.xlds && p.M == 1 && env_int("QIE_GEMV_XFIRST", 1) != 0)
        xch = K_fits(a->K, 2) ? 2 : (K_fits(a->K, 10) ? 10 : 0);
    switch (MT) {
        case 1: return launch_gemv_1(p, rpw, a->epilogue, st, bpc, xch);
        case 2: return launch_gemv_m<2, 0>(p, rpw, a->epilogue, st, bpc);
        case 4: return launch_gemv_m<4, 0>(p, rpw, a->epilogue, st, bpc);
        default: return launch_gemv_m<8, 0>(p, rpw, a->epilogue, st, bpc);
    }
}

}  // namespace qie
