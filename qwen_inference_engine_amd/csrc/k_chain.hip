// k_chain.hip — batch-1 decode: the weight-streaming part of a layer as ONE persistent
// launch.
//
// Per decode layer the reference runs o_proj, resadd, rms, up, gate, act, elem, down,
// resadd, then the next layer's rms, q, k, v projections (qwen_main.cu:305-360, 271-296)
// — here four dependent GEMV phases in one launch of one workgroup per CU:
//
//   O : x[r]  = bf16(x[r] + bf16(W_o[r] . att))                 (row-parallel over H)
//   G : h[j]  = bf16(bf16(up_j . n) * bf16(silu(bf16(gate_j . n)))),  n = rms(x) * w_ffn
//   D : x[r]  = bf16(x[r] + bf16(W_down[r] . h))
//   Q : qkv[c] = bf16(W_qkv[c] . rms(x) * w_attn + b[c])          (the NEXT layer's QKV)
//
// Every phase depends on ALL outputs of the one before (a chip-wide seam), but not its
// WEIGHTS: each wave issues the first weight chunks of its next phase BEFORE it waits
// for the seam, so the HBM stream keeps running across the hand-off instead of
// restarting at every kernel boundary (cdna_hip_programming.md §5.6: one launch won on
// weight-streaming batch-1 decode chains).  The attention stays its own launch.
//
// Hand-off (cdna_hip_programming.md §6 Guideline 16, the sc1 form): every store of the
// handed-off vectors (x rows, h) is an agent-scope store (sc1, write-through), drained
// (s_waitcnt vmcnt(0)) and barriered before one lane adds 1 to each of 8 replicas of the
// phase counter (64 B apart); consumers poll the replica of their blockIdx % 8 and read the
// vectors with agent-scope loads.  Spins are bounded (give-up flag, checked by the host).
// The last workgroup to finish zeroes the counters for the next launch.
//
// Work split: rows are handed out in PAIRS (two adjacent outputs = one 32-bit sc1 store),
// pair p of a phase with P pairs to workgroup p * 256 / P's block — a contiguous slice
// per CU — and within the workgroup round-robin over its 8 waves.  Per-row arithmetic is
// the GEMV's (k_gemv.hip): lane l of a wave accumulates elements 8 l + 512 u in fp32 with
// FMAs, then a DPP/permlane butterfly, one bf16 rounding.
#include "qie_common.hpp"
#include "k_chain.hpp"
#include "../../include/qie/qie_ops.h"

namespace qie {

typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));

constexpr int kChainWaves = 8;                   // 512 threads, one workgroup per CU
constexpr int kChainU2 = 8;                      // 512-element chunks in flight per row, 2-row tasks
constexpr int kChainU4 = 4;                      //   and 4-row (gate/up) tasks: 16 KB per wave either way
constexpr int kChainCtrStride = 16;              // 64 B between counter replicas
constexpr int kChainPhases = 4;
constexpr int kChainCtrWords = kChainPhases * 8 * kChainCtrStride + 64;   // + fin, err
constexpr int kChainFin = kChainPhases * 8 * kChainCtrStride;
constexpr int kChainErr = kChainFin + 16;

// agent-scope (sc1) 32-bit store / 128-bit-as-2x64 load of handed-off data
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld_sc1_16(const uint16_t* p) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

// Pair tasks are dealt round-robin over every wave of the grid (pair p to workgroup
// p % G, wave (p / G) % 8): the 2048 waves stream 2048 neighbouring row pairs at any
// moment, spread over all HBM channels.  (Contiguous per-CU slices, every CU at the same
// offset of its own slice, ran the gate/up phase 10 % slower with a 5 us spread across
// XCDs.)
__device__ __forceinline__ int64_t chain_first(int wave) { return blockIdx.x + (int64_t)gridDim.x * wave; }
__device__ __forceinline__ int64_t chain_step() { return (int64_t)gridDim.x * 8; }

// seam: publish (after this workgroup's last store of the phase) / wait for all
__device__ __forceinline__ void chain_signal(unsigned* ctr, int phase) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x < 8)
        __hip_atomic_fetch_add(&ctr[(phase * 8 + threadIdx.x) * kChainCtrStride], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}
// The poll runs on the LAST wave, which issues no prefetch loads: vmcnt retires a wave's
// loads in order, so a poll from a wave with 16 KB of weights in flight returns only after
// they do (measured: ~5 us seams with the poll on wave 0).
constexpr int kChainPoller = 0;
__device__ __forceinline__ void chain_wait(unsigned* ctr, int phase) {
    if (threadIdx.x == 64 * kChainPoller) {
        const unsigned* rep = &ctr[(phase * 8 + (blockIdx.x & 7)) * kChainCtrStride];
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {   // 20 ms at 100 MHz: give up
                __hip_atomic_store(&ctr[kChainErr], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

// One task = R weight rows (all of length K) dotted with the vector in LDS.
// wr[i]: row pointers; chunks of 512 elements, U in flight.
template <int R>
struct RowTask {
    const cu32x4* wr[R];
};

template <int R, int U>
__device__ __forceinline__ void chain_load(const RowTask<R>& t, int64_t K, int64_t k0, cu32x4 (&wv)[U][R]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t k = k0 + u * 512 + lane * 8;
        const int64_t kc = (k < K ? k : K - 8) / 8;   // clamped: loads stay unconditional
#pragma unroll
        for (int i = 0; i < R; i++) wv[u][i] = __builtin_nontemporal_load(t.wr[i] + kc);
    }
}

template <int R, int U>
__device__ __forceinline__ void chain_fma(const uint16_t* xs, int64_t K, int64_t k0, const cu32x4 (&wv)[U][R],
                                          float (&acc)[R]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t k = k0 + u * 512 + lane * 8;
        if (k < K) {
            const uint4 xv = *reinterpret_cast<const uint4*>(xs + k);
            const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w};
            float xf[8];
#pragma unroll
            for (int j = 0; j < 4; j++) { xf[2 * j] = bf_lo(xw[j]); xf[2 * j + 1] = bf_hi(xw[j]); }
#pragma unroll
            for (int i = 0; i < R; i++) {
                const uint32_t w4[4] = {wv[u][i].x, wv[u][i].y, wv[u][i].z, wv[u][i].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[i] = fmaf(xf[2 * j], bf_lo(w4[j]), acc[i]);
                    acc[i] = fmaf(xf[2 * j + 1], bf_hi(w4[j]), acc[i]);
                }
            }
        }
    }
}

// Runs this wave's tasks of one phase.  `first` holds the first U chunks of the wave's
// first task (issued before the seam); each task's first chunks of the NEXT task are
// issued before this task's reduction and epilogue.  make(task, RowTask&) resolves the
// rows; done(task, acc[R]) runs on every lane with the wave-reduced sums.
template <int R, int U, class Make, class Done>
__device__ __forceinline__ void chain_phase(const uint16_t* xs, int64_t K, int64_t t0, int64_t t1, int64_t tstep,
                                            cu32x4 (&wv)[U][R], Make make, Done done, bool prefetched = true) {
    RowTask<R> t;
    if (t0 < t1) make(t0, t);
    if (!prefetched && t0 < t1) chain_load<R, U>(t, K, 0, wv);
    for (int64_t task = t0; task < t1; task += tstep) {
        float acc[R];
#pragma unroll
        for (int i = 0; i < R; i++) acc[i] = 0.f;
        chain_fma<R, U>(xs, K, 0, wv, acc);
        for (int64_t k0 = 512 * U; k0 < K; k0 += 512 * U) {
            chain_load<R, U>(t, K, k0, wv);
            chain_fma<R, U>(xs, K, k0, wv, acc);
        }
        if (task + tstep < t1) {   // next task's first chunks in flight during this epilogue
            make(task + tstep, t);
            chain_load<R, U>(t, K, 0, wv);
        }
#pragma unroll
        for (int i = 0; i < R; i++) acc[i] = wave_sum(acc[i]);
        done(task, acc);
    }
}

// RMSNorm of the full residual row x (agent-scope loads: written by other workgroups
// in this launch) into xs, the reference's rmsNorm semantics (normalization.cu:5-25;
// HF: transformers).  512 threads, 8 elements per thread per pass.
__device__ __forceinline__ void chain_norm_x(const ChainParams& p, const uint16_t* nw, uint16_t* xs, float* red) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t H = p.H;
    float ss = 0.f;
    for (int64_t k = (int64_t)tid * 8; k < H; k += 512 * 8) {
        const uint4 v = ld_sc1_16(p.x + k);
        *reinterpret_cast<uint4*>(xs + k) = v;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float a = bf_lo(w[j]), b = bf_hi(w[j]);
            ss += a * a;
            ss += b * b;
        }
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    ss = 0.f;
    for (int w = 0; w < kChainWaves; w++) ss += red[w];
    const float rms = sqrtf((ss / (float)H) + p.eps);
    const float inv = 1.0f / rms;
    const bool hf = p.numerics == QIE_NUMERICS_HF;
    for (int64_t k = (int64_t)tid * 8; k < H; k += 512 * 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(xs + k);
        const uint4 n = *reinterpret_cast<const uint4*>(nw + k);
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, nn[4] = {n.x, n.y, n.z, n.w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float a = bf_lo(vw[j]), b = bf_hi(vw[j]), wa = bf_lo(nn[j]), wb = bf_hi(nn[j]);
            const float ya = hf ? wa * rbf(a * inv) : (a / rms) * wa;
            const float yb = hf ? wb * rbf(b * inv) : (b / rms) * wb;
            o[j] = pack2(ya, yb);
        }
        *reinterpret_cast<uint4*>(xs + k) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
}

__global__ __launch_bounds__(512) void chain_kernel(ChainParams p) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem);          // [max(QD, H, I)] input vector
    __shared__ float red[kChainWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t H = p.H, QD = p.QD, I = p.I;
    cu32x4 wv2[kChainU2][2];
    cu32x4 wv4[kChainU4][4];
    auto stamp = [&](int i) {   // phase timing (tools/ubench.py UB_SET=chain): wall clock per workgroup
        if (p.dbg && tid == 0) p.dbg[blockIdx.x * 16 + i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // ================= phase O: x += W_o . att   (pairs of x rows)
    const int64_t o0 = chain_first(wave), o1 = H / 2, ts = chain_step();
    auto make_o = [&](int64_t pr, RowTask<2>& t) {
        t.wr[0] = reinterpret_cast<const cu32x4*>(p.wo + (2 * pr) * QD);
        t.wr[1] = reinterpret_cast<const cu32x4*>(p.wo + (2 * pr + 1) * QD);
    };
    {
        RowTask<2> t;
        make_o(o0 < o1 ? o0 : 0, t);
        chain_load<2, kChainU2>(t, QD, 0, wv2);
    }
    for (int64_t k = (int64_t)tid * 8; k < QD; k += 512 * 8)   // previous launch's output: plain loads
        *reinterpret_cast<uint4*>(xs + k) = *reinterpret_cast<const uint4*>(p.att + k);
    __syncthreads();
    chain_phase<2, kChainU2>(xs, QD, o0, o1, ts, wv2, make_o, [&](int64_t pr, float (&acc)[2]) {
        if (lane == 0) {
            uint32_t* xp = reinterpret_cast<uint32_t*>(p.x) + pr;
            const uint32_t old = ld_sc1(xp);
            st_sc1(xp, pack2(bf_lo(old) + rbf(acc[0]), bf_hi(old) + rbf(acc[1])));
        }
    });

    // ================= phase G: h = swiglu(W_gate . n, W_up . n), n = rms(x) * w_ffn
    const int64_t g0 = chain_first(wave), g1 = I / 2;
    auto make_g = [&](int64_t pr, RowTask<4>& t) {
        t.wr[0] = reinterpret_cast<const cu32x4*>(p.wg + (2 * pr) * H);
        t.wr[1] = reinterpret_cast<const cu32x4*>(p.wg + (2 * pr + 1) * H);
        t.wr[2] = reinterpret_cast<const cu32x4*>(p.wu + (2 * pr) * H);
        t.wr[3] = reinterpret_cast<const cu32x4*>(p.wu + (2 * pr + 1) * H);
    };
    stamp(1);
    chain_signal(p.ctr, 0);   // drains this phase's stores first: vmcnt counts loads too
    {
        RowTask<4> t;
        make_g(g0 < g1 ? g0 : 0, t);
        if (true) chain_load<4, kChainU4>(t, H, 0, wv4);
    }
    chain_wait(p.ctr, 0);
    stamp(2);
    chain_norm_x(p, p.ffn_norm, xs, red);
    const bool pf = true;
    chain_phase<4, kChainU4>(xs, H, g0, g1, ts, wv4, make_g, [&](int64_t pr, float (&acc)[4]) {
        if (lane == 0) {
            float o[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float g = rbf(acc[i]);
                const float u = rbf(acc[2 + i]);
                const float a = rbf(g * (1.0f / (1.0f + expf(-g))));
                o[i] = u * a;
            }
            st_sc1(reinterpret_cast<uint32_t*>(p.h) + pr, pack2(o[0], o[1]));
        }
    }, pf);

    // ================= phase D: x += W_down . h
    auto make_d = [&](int64_t pr, RowTask<2>& t) {
        t.wr[0] = reinterpret_cast<const cu32x4*>(p.wd + (2 * pr) * I);
        t.wr[1] = reinterpret_cast<const cu32x4*>(p.wd + (2 * pr + 1) * I);
    };
    stamp(3);
    chain_signal(p.ctr, 1);
    {
        RowTask<2> t;
        make_d(o0 < o1 ? o0 : 0, t);
        if (true) chain_load<2, kChainU2>(t, I, 0, wv2);
    }
    chain_wait(p.ctr, 1);
    stamp(4);
    for (int64_t k = (int64_t)tid * 8; k < I; k += 512 * 8)
        *reinterpret_cast<uint4*>(xs + k) = ld_sc1_16(p.h + k);
    __syncthreads();
    chain_phase<2, kChainU2>(xs, I, o0, o1, ts, wv2, make_d, [&](int64_t pr, float (&acc)[2]) {
        if (lane == 0) {
            uint32_t* xp = reinterpret_cast<uint32_t*>(p.x) + pr;
            const uint32_t old = ld_sc1(xp);
            st_sc1(xp, pack2(bf_lo(old) + rbf(acc[0]), bf_hi(old) + rbf(acc[1])));
        }
    }, pf);

    // ================= phase Q (next layer): qkv = W_qkv . (rms(x) * w_attn) + b
    if (p.attn_norm) {
        const int64_t N = QD + 2 * p.KD;
        const int64_t q0 = chain_first(wave), q1 = N / 2;
        auto make_q = [&](int64_t pr, RowTask<2>& t) {
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int64_t r = 2 * pr + i;
                const uint16_t* w = r < QD ? p.wq + r * H
                                           : (r < QD + p.KD ? p.wk + (r - QD) * H : p.wv + (r - QD - p.KD) * H);
                t.wr[i] = reinterpret_cast<const cu32x4*>(w);
            }
        };
        stamp(5);
        chain_signal(p.ctr, 2);
        {
            RowTask<2> t;
            make_q(q0 < q1 ? q0 : 0, t);
            if (true) chain_load<2, kChainU2>(t, H, 0, wv2);
        }
        chain_wait(p.ctr, 2);
        stamp(6);
        chain_norm_x(p, p.attn_norm, xs, red);
        chain_phase<2, kChainU2>(xs, H, q0, q1, ts, wv2, make_q, [&](int64_t pr, float (&acc)[2]) {
            if (lane == 0) {
                float o[2];
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int64_t r = 2 * pr + i;
                    const uint16_t* b = r < QD ? p.bq : (r < QD + p.KD ? p.bk : p.bv);
                    const int64_t bi = r < QD ? r : (r < QD + p.KD ? r - QD : r - QD - p.KD);
                    o[i] = b ? acc[i] + bf2f(b[bi]) : acc[i];
                }
                reinterpret_cast<uint32_t*>(p.qkv)[pr] = pack2(o[0], o[1]);   // next consumer: a new launch
            }
        }, pf);
    }

    // ================= the last workgroup to finish zeroes the counters
    __syncthreads();
    stamp(7);
    if (tid == 0) {
        const unsigned f = __hip_atomic_fetch_add(&p.ctr[kChainFin], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f == gridDim.x - 1) {
            for (int i = 0; i < kChainPhases * 8; i++)
                __hip_atomic_store(&p.ctr[i * kChainCtrStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.ctr[kChainFin], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Host launcher (engine.hip): one workgroup per CU.  Requirements checked here: bf16
// weights, H, QD, KD, I even and multiples of 8, every row 16-B aligned.
int chain_launch(const ChainParams& p, hipStream_t st) {
    QIE_REQUIRE(p.att && p.wo && p.x && p.ffn_norm && p.wg && p.wu && p.h && p.wd && p.ctr,
                "chain: missing operand");
    QIE_REQUIRE(p.H % 8 == 0 && p.QD % 8 == 0 && p.I % 8 == 0 && p.KD % 8 == 0, "chain: dims must be multiples of 8");
    QIE_REQUIRE(!p.attn_norm || (p.wq && p.wk && p.wv && p.qkv), "chain: next-layer QKV operands missing");
    const int64_t maxk = std::max(std::max(p.H, p.QD), p.I);
    const size_t shm = (size_t)maxk * 2;
    QIE_REQUIRE(shm <= 64 * 1024, "chain: input vector of %lld elements exceeds the LDS stage", (long long)maxk);
    const int cus = device_cu_count();
    hipLaunchKernelGGL(chain_kernel, dim3((unsigned)cus), dim3(512), shm, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

int chain_ctr_words() { return kChainCtrWords; }
int chain_err_word() { return kChainErr; }

}  // namespace qie
