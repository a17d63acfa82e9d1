// k_persist.hip — the batch-1 decode layers as ONE persistent launch (gfx950).
//
// Replaces the per-layer loop of llm()'s decode branch (layers/src/qwen_main.cu:271-359):
//   rms -> q,k,v (+bias) -> [qk-norm] -> RoPE -> KV append -> attention -> o -> +res ->
//   rms -> gate, up -> silu*up -> down -> +res
// for every layer of the step, which the engine otherwise runs as five hipGraph-captured
// launches per layer (engine.hip enqueue_layer_decode).  Those launches stream their weights
// at the HBM rate inside each kernel, but every launch starts its stream only once the previous
// kernel has fully drained, and the latency-bound middle of a layer (norm prologue, attention,
// split combine) streams nothing: DESIGN.md §3 "the floor of a 5-launch step".
//
// Structure (cdna_hip_programming.md §5.6, MI355X_MICROARCH.md price list):
//   * one 512-thread workgroup per CU for the whole step; every CU owns fixed row ranges of
//     each projection (QKV, O, gate/up, down) and streams them with 16-B non-temporal buffer
//     loads, two rows per wave task, up to 8 KiB-chunks per row in flight (the GEMV kernels'
//     exact per-lane fp32 order: chunks ascending, fma8, wave butterfly — so every projection
//     output is bit-identical to the launch path);
//   * run-ahead: a wave issues the first chunks of its NEXT task — also across a dependency
//     edge into the next projection — before it waits for that projection's input, so the HBM
//     stream keeps going while the layer's inputs travel between CUs;
//   * hand-offs between CUs are 8-byte {tag, two bf16} granules (one sc1 store each, the data
//     is the flag; MI355X_MICROARCH.md handoff rows, Guideline 16 R2), tag = (step epoch << 7)
//     + layer + 1: the step epoch is advanced by the step's finalize kernel, so no buffer needs
//     zeroing between launches (every location's previous tag differs from the one awaited);
//   * a consuming CU gathers the whole input vector of a projection into LDS (x for the QKV
//     norm, the attention output for O, x' for the gate/up norm, h for down); RMSNorm in the
//     SAME fp32 orders as the launch path's fused prologues (QKV: the 256-thread x-first
//     prologue; gate/up: the per-wave register form);
//   * attention: CUs [0, nkv * nsplit) run the fused decode attention body of attn_decode.hpp
//     (the stand-alone kernel's code, 8 waves) as job (kv head, split); its q / k / v row comes
//     from the QKV granules (gathered after its K / V step is in flight), its split partials and
//     ticket combine are unchanged, its output goes out as granules; the other CUs own the O
//     projection's rows and have their O weights in flight while the attention runs;
//   * every wait is bounded (s_memrealtime): on a timeout, or when another block already failed
//     (error word), the block gives up, the grid drains, and the engine's next synchronising
//     call fails with the error word (engine.hip pk_check) — never a hang.
#include "attn_decode.hpp"

#include <cstddef>
#include <vector>

namespace qie {

namespace pk {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// waves per workgroup (one workgroup per CU): 8 at head_dim 128 (the attention body runs on all
// 8), 4 at head_dim 64 (its MFMA tiles need a 16-dim P.V slice per wave: 64 / 16)
template <int HD>
constexpr int waves_for() { return HD == 128 ? 8 : 4; }
constexpr int kU = 8;        // 1-KiB wave-loads per row in flight (one pass)
constexpr int kStage = 1024; // outputs a CU owns in one projection (bf16 staging in LDS)
constexpr int kMaxBias = 256;
// granules per gathering thread: x-sized vectors (H / 2, and the attention output QD / 2) by
// one wave, h (I / 2) by four; persist_supported checks the model fits
constexpr int kGatherX = 40;   // H, QD <= 5,120 (64 threads x 40 granules)
constexpr int kGatherH = 38;   // I <= 19,456 (256 threads x 38 granules)

struct Params {
    const qie_layer_weights* layers;   // device copy, [n_layers]
    int n_layers, H, I, QD, KD, nq, nkv, hd;
    float eps;
    int numerics;
    uint16_t* x_res;                   // [H] residual stream (in: layer 0 input; out: after the last layer)
    unsigned long long *g_x, *g_qkv, *g_att, *g_x1, *g_h;
    const unsigned* epoch;
    unsigned* err;
    long long spin_ticks;              // bounded waits, s_memrealtime ticks (100 MHz)
    const DecodeAttnParams* attp;      // device [n_layers]: the attention role's parameters per layer
    const int32_t* pos;                // the sequence position (B = 1)
    int splits_target;
    unsigned long long* ts;            // diagnostics (qie_batch_pk_trace): [cu][layer][kTsSlots] s_memrealtime
    unsigned pf_mask;                  // waves that may run ahead into the next projection (bit w: wave w)
    int xw_even;                       // row share of a CU on an even XCD, per 100 of an odd one's (gate/up, down)
};
constexpr int kTsSlots = 12;

__device__ __forceinline__ float bl(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bh(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
    f[0] = bl(v.x); f[1] = bh(v.x); f[2] = bl(v.y); f[3] = bh(v.y);
    f[4] = bl(v.z); f[5] = bh(v.z); f[6] = bl(v.w); f[7] = bh(v.w);
}
// the GEMV kernels' per-chunk FMA chain (k_gemv.hip fma8): element order 0..7
__device__ __forceinline__ void fma8(float& acc, const float* xf, u32x4 w) {
    acc = fmaf(xf[0], bl(w.x), acc);
    acc = fmaf(xf[1], bh(w.x), acc);
    acc = fmaf(xf[2], bl(w.y), acc);
    acc = fmaf(xf[3], bh(w.y), acc);
    acc = fmaf(xf[4], bl(w.z), acc);
    acc = fmaf(xf[5], bh(w.z), acc);
    acc = fmaf(xf[6], bl(w.w), acc);
    acc = fmaf(xf[7], bh(w.w), acc);
}

// uniform loads through the scalar cache (constant address space): the layer table, the
// position and the epoch stay in SGPRs — a plain load of them may be a vector load (the kernel
// stores to global memory), and every buffer resource built from such a pointer then runs a
// readfirstlane waterfall loop per load
template <class T>
__device__ __forceinline__ T sld(const T* ptr) {
    return ((const __attribute__((address_space(4))) T*)ptr)[0];
}
// One pointer field of layer l's weight table, loaded where it is used: the table base is made
// opaque first, so the scalar load cannot be hoisted to the top of the layer (14 pointers kept
// live across a whole layer pushed the kernel's SGPRs into spills)
#define PK_LW(tab, l, field)                                                                          \
    ([&]() {                                                                                        \
        const unsigned char* b_ = reinterpret_cast<const unsigned char*>(tab) +                     \
                                  (size_t)(l) * sizeof(qie_layer_weights);                         \
        asm volatile("" : "+s"(b_));                                                                \
        return (const void*)sld(reinterpret_cast<const unsigned long long*>(b_ + offsetof(qie_layer_weights, field))); \
    }())

// a struct of dwords through the scalar cache (the attention role's parameters)
template <class T>
__device__ __forceinline__ T sld_struct(const T* src) {
    static_assert(sizeof(T) % 4 == 0, "dword struct");
    constexpr int n = (int)(sizeof(T) / 4);
    const unsigned char* b = reinterpret_cast<const unsigned char*>(src);
    asm volatile("" : "+s"(b));
    unsigned v[n];
#pragma unroll
    for (int i = 0; i < n; i++) v[i] = sld(reinterpret_cast<const unsigned*>(b) + i);
    T out;
    __builtin_memcpy(&out, v, sizeof(T));
    return out;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// ------------------------------------------------------------------ bounded hand-off waits
__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(unsigned long long* g, unsigned tag, uint32_t v) {
    __hip_atomic_store(g, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Threads t (0 <= t < nt) of the calling waves gather granules [0, n) of g into dst (u32
// payload each): thread t owns the M consecutive granules [t M, t M + M) (M even), read as 16-B
// sc1 buffer loads (two granules per load: each granule still validates itself by its tag).
// Whole sweeps: every granule still missing is re-loaded in ONE batch per pass — one memory round
// trip per pass, never one dependent re-poll per granule (the first form spun on each missing
// granule in turn: 6-10 us per gather, tools/pk_trace.py r06).  The byte offset is made opaque
// each pass, so the loads are re-issued, not hoisted out of the poll loop.  A failure (timeout,
// or another block's error word) marks the block dead (LDS flag, read after the next barrier).
template <int M>
__device__ __forceinline__ void gather(const unsigned long long* g, int n, unsigned tag, uint32_t* dst, int t, int nt,
                                       const Params& p, int* dead, unsigned code) {
    static_assert(M % 2 == 0 && M <= 64, "pairs, mask of 64");
    (void)nt;
    const int base = t * M;
    const __amdgpu_buffer_rsrc_t rs = rsrc(g, (int64_t)n * 8);   // past n: zeros (tag 0, never awaited)
    unsigned long long need = 0ull;
#pragma unroll
    for (int j = 0; j < M; j++)
        if (base + j < n) need |= 1ull << j;
    int vo = base * 8;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int pass = 0;; pass++) {
        asm volatile("" : "+v"(vo));
        u32x4 r[M / 2];
#pragma unroll
        for (int k = 0; k < M / 2; k++)
            if ((need >> (2 * k)) & 3ull) r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16 * k, 0, 16);
#pragma unroll
        for (int k = 0; k < M / 2; k++) {
            if (((need >> (2 * k)) & 1ull) && r[k].y == tag) {
                dst[base + 2 * k] = r[k].x;
                need &= ~(1ull << (2 * k));
            }
            if (((need >> (2 * k + 1)) & 1ull) && r[k].w == tag) {
                dst[base + 2 * k + 1] = r[k].z;
                need &= ~(1ull << (2 * k + 1));
            }
        }
        if (__builtin_amdgcn_ballot_w64(need != 0ull) == 0ull) return;   // this wave's share is in
        __builtin_amdgcn_s_sleep(2);
        if ((pass & 7) == 7) {
            bool stop = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > p.spin_ticks) {
                if (!stop) __hip_atomic_fetch_or(p.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                stop = true;
            }
            if (__builtin_amdgcn_ballot_w64(stop) != 0ull) {
                *dead = 1;
                return;
            }
        }
    }
}

// ------------------------------------------------------------------ GEMV tasks
// One task = two weight rows (row pointers), K columns, x (bf16) in LDS.  The first pass of
// a task can be issued ahead (run-ahead prefetch) into the wave's register set `wv`.
struct Task {
    const uint8_t* r0;
    const uint8_t* r1;
    int K;
};

// a wave-uniform pointer made provably uniform (two readfirstlanes): a buffer resource built
// from a pointer the compiler's divergence analysis cannot prove uniform is wrapped in a
// readfirstlane waterfall loop per load (cdna_hip_programming.md T20)
__device__ __forceinline__ const uint8_t* uni(const uint8_t* ptr) {
    const unsigned long long v = (unsigned long long)ptr;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (const uint8_t*)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void issue(const Task& t, int pass, u32x4 (&wv)[kU][2]) {
    const int lane = threadIdx.x & 63;
    const int K = __builtin_amdgcn_readfirstlane(t.K);
    const auto s0 = rsrc(uni(t.r0), (int64_t)K * 2), s1 = rsrc(uni(t.r1), (int64_t)K * 2);
    const int voff = lane * 16 + pass * kU * 1024;
#pragma unroll
    for (int u = 0; u < kU; u++) {   // unconditional: a chunk past K reads zeros (range check)
        wv[u][0] = __builtin_amdgcn_raw_buffer_load_b128(s0, voff, u * 1024, 2);
        wv[u][1] = __builtin_amdgcn_raw_buffer_load_b128(s1, voff, u * 1024, 2);
    }
}

// the task's two dot products with x (LDS), pass 0 already in wv; `next` is issued before the
// butterfly (the GEMV kernels' cross-task prefetch)
template <class Next>
__device__ __forceinline__ void run_task(const Task& t, const uint16_t* xs, u32x4 (&wv)[kU][2], float& a0, float& a1,
                                         Next&& next) {
    const int lane = threadIdx.x & 63;
    a0 = 0.f;
    a1 = 0.f;
    const int npass = (t.K + kU * 512 - 1) / (kU * 512);
    for (int pass = 0; pass < npass; pass++) {
        if (pass > 0) issue(t, pass, wv);
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int k = (pass * kU + u) * 512 + lane * 8;
            if (k < t.K) {
                const uint4 xv = *reinterpret_cast<const uint4*>(xs + k);
                float xf[8];
                unpack8(xv, xf);
                fma8(a0, xf, wv[u][0]);
                fma8(a1, xf, wv[u][1]);
            }
        }
    }
    next();
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
}

// ------------------------------------------------------------------ norms (launch-path orders)
// QKV's fused norm (k_gemv.hip x-first prologue, 256 threads): thread t sums the squares of its
// chunks k = 8 t + 2048 c, a 64-lane butterfly per wave, then the four wave sums in order.
// Threads 0..255 of the block run exactly that; the result is published in red[0].
__device__ __forceinline__ void ss_xfirst256(const uint16_t* x, int K, float* red) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 256) {
        float ss = 0.f;
        for (int c = 0; c * 2048 < K; c++) {
            const int k = tid * 8 + c * 2048;
            if (k >= K) continue;
            float f[8];
            unpack8(*reinterpret_cast<const uint4*>(x + k), f);
#pragma unroll
            for (int j = 0; j < 8; j++) ss += f[j] * f[j];
        }
        ss = wave_sum(ss);
        if (lane == 0) red[1 + wave] = ss;
    }
}
// gate/up's fused norm (k_gemv.hip XCH = 4): lane l sums chunks k = 8 l + 512 u, one butterfly
__device__ __forceinline__ float ss_wave(const uint16_t* x, int K) {
    const int lane = threadIdx.x & 63;
    float ss = 0.f;
    for (int u = 0; u * 512 < K; u++) {
        const int k = lane * 8 + u * 512;
        if (k >= K) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + k), f);
#pragma unroll
        for (int j = 0; j < 8; j++) ss += f[j] * f[j];
    }
    return wave_sum(ss);
}
// y = bf16((x / rms) * w) (REF, normalization.cu:5-25) or bf16(w * bf16(x * (1 / rms))) (HF)
__device__ __forceinline__ void normalize(const uint16_t* x, const uint16_t* nw, uint16_t* y, int K, float rms,
                                          bool hf) {
#pragma clang fp contract(off)
    const float inv = 1.0f / rms;
    for (int i = threadIdx.x; i * 8 < K; i += blockDim.x) {
        float f[8], wf[8];
        unpack8(*reinterpret_cast<const uint4*>(x + i * 8), f);
        unpack8(*reinterpret_cast<const uint4*>(nw + i * 8), wf);
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
        *reinterpret_cast<uint4*>(y + i * 8) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// [lo, hi) of n items over `parts` parts, part i
__device__ __forceinline__ void span(int n, int parts, int i, int& lo, int& hi) {
    lo = (int)((int64_t)n * i / parts);
    hi = (int)((int64_t)n * (i + 1) / parts);
}
// the same with CU weights: even CUs (blockIdx % 8 even: XCDs 0, 2, 4, 6 under round-robin
// placement) weigh we, odd ones 100 — a speed share, never correctness (every item is owned once)
__device__ __forceinline__ void wspan(int n, int parts, int i, int we, int& lo, int& hi) {
    auto W = [&](int c) { return (int64_t)((c + 1) / 2) * we + (int64_t)(c / 2) * 100; };
    const int64_t tot = W(parts);
    lo = (int)((int64_t)n * W(i) / tot);
    hi = (int)((int64_t)n * W(i + 1) / tot);
}

__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS writes visible; VMEM loads stay in flight
    __builtin_amdgcn_s_barrier();
}

// attention role hook (attn_decode.hpp): q / k / v row of kv head g from the QKV granules,
// outputs into an LDS staging row
template <int NT>
struct AttnHook {
    static constexpr bool on = true;
    const unsigned long long* g_qkv;
    uint16_t* row;          // LDS image of the whole q|k|v row (the body reads a.qkv = row)
    uint16_t* stage;        // LDS [G * hd]: this kv head's output
    int64_t o0;             // output index of stage[0]
    int g, G, hd, QD, KD;
    unsigned tag;
    const Params* p;
    int* dead;
    __device__ void gather() {
        // q of the kv head's G heads (G hd / 2 granules), then its k and v rows (hd / 2 each)
        const int nqg = G * hd / 2, nk = hd / 2;
        uint32_t* r32 = reinterpret_cast<uint32_t*>(row);
        const int t = threadIdx.x;
        if (2 * t < nqg) pk::gather<2>(g_qkv + g * nqg, nqg, tag, r32 + g * nqg, t, NT, *p, dead, 2u);
        const int tk = t - NT / 2;   // from the middle wave on: k, then v
        if (tk >= 0 && tk < nk) {
            const int kv = tk < nk / 2 ? (QD + g * hd) / 2 : (QD + KD + g * hd) / 2;
            const int tt = tk < nk / 2 ? tk : tk - nk / 2;
            pk::gather<2>(g_qkv + kv, nk, tag, r32 + kv, tt, nk / 2, *p, dead, 2u);
        }
        __syncthreads();
    }
    __device__ void out1(int64_t i, uint16_t v) { stage[i - o0] = v; }
    __device__ void out4(int64_t i, unsigned long long v) {
        *reinterpret_cast<unsigned long long*>(stage + (i - o0)) = v;
    }
};

// ------------------------------------------------------------------ the kernel
template <int HD, int NW = waves_for<HD>()>
__global__ __launch_bounds__(NW * 64, 1) void decode_layers_kernel(Params p) {
    constexpr int kWaves = NW, kThreads = NW * 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cu = blockIdx.x, ncu = gridDim.x;
    const int H = p.H, I = p.I, QD = p.QD, KD = p.KD, QKVD = QD + 2 * KD;
    const int G = p.nq / p.nkv;
    const bool hf = p.numerics == QIE_NUMERICS_HF;

    // ---- LDS carve (16-B aligned pieces)
    auto al = [](int b) { return (b + 15) & ~15; };
    unsigned char* q = smem;
    uint16_t* xraw = reinterpret_cast<uint16_t*>(q); q += al(H * 2);        // layer input x
    uint16_t* x1raw = reinterpret_cast<uint16_t*>(q); q += al(H * 2);       // x after O (+res)
    uint16_t* xn = reinterpret_cast<uint16_t*>(q); q += al((H > QD ? H : QD) * 2);   // normed x / attention out
    uint16_t* nw = reinterpret_cast<uint16_t*>(q); q += al(H * 2);          // norm weights
    uint16_t* hb = reinterpret_cast<uint16_t*>(q); q += al((I > QKVD ? I : QKVD) * 2);   // h / q|k|v row image
    uint16_t* stage = reinterpret_cast<uint16_t*>(q); q += al(kStage * 2);
    uint16_t* astage = reinterpret_cast<uint16_t*>(q); q += al(G * HD * 2);
    float* bias = reinterpret_cast<float*>(q); q += al(kMaxBias * 4);
    float* red = reinterpret_cast<float*>(q); q += 64;
    int* dead = reinterpret_cast<int*>(q);
    if (tid == 0) *dead = 0;

    const unsigned epoch = sld(p.epoch);
    auto tagl = [&](int l) { return (epoch << 7) + (unsigned)l + 1u; };

    // ---- attention jobs of this step: CUs [0, nA) = (kv head, split)
    const int pos = sld(p.pos);
    const int chunk = decm_chunk(pos + 1, p.splits_target, kDecMStep);
    const int nsplit = (pos + 1 + chunk - 1) / chunk;
    const int nA = p.nkv * nsplit;
    const bool att_cu = cu < nA;
    const int nO = ncu - nA;   // CUs owning O rows

    // ---- this CU's row ranges (pairs of outputs: a granule holds two bf16)
    int q0, q1, o0 = 0, o1 = 0, j0, j1, d0, d1;
    span(QKVD / 2, ncu, cu, q0, q1);
    if (!att_cu) span(H / 2, nO, cu - nA, o0, o1);
    wspan(I / 2, ncu, cu, p.xw_even, j0, j1);
    wspan(H / 2, ncu, cu, p.xw_even, d0, d1);
    // local task i of a projection -> wave (i + 1) % 8: wave 0 (the gathering wave) last
    const int wfirst = (wave + kWaves - 1) % kWaves;

    u32x4 wv[kU][2];
    bool pf = false;   // wv holds the first pass of this wave's first task of the next projection

    auto row = [](const void* base, int64_t r, int K) { return reinterpret_cast<const uint8_t*>(base) + r * K * 2; };
    const qie_layer_weights* LT = p.layers;
    auto qkv_task = [&](int l, int pi) {
        const int r = 2 * pi;
        const void* b = r < QD ? PK_LW(LT, l, wq) : (r < QD + KD ? PK_LW(LT, l, wk) : PK_LW(LT, l, wv));
        const int rr = r < QD ? r : (r < QD + KD ? r - QD : r - QD - KD);
        return Task{row(b, rr, H), row(b, rr + 1, H), H};
    };
    auto o_task = [&](int l, int pi) {
        const void* w = PK_LW(LT, l, wo);
        return Task{row(w, 2 * pi, QD), row(w, 2 * pi + 1, QD), QD};
    };
    auto gu_task = [&](int l, int j) { return Task{row(PK_LW(LT, l, w_gate), j, H), row(PK_LW(LT, l, w_up), j, H), H}; };
    auto dn_task = [&](int l, int pi) {
        const void* w = PK_LW(LT, l, w_down);
        return Task{row(w, 2 * pi, I), row(w, 2 * pi + 1, I), I};
    };
    // first task of this wave in a projection with n local tasks (none: false)
    auto pf_issue = [&](bool has, const Task& t) {
        has = has && ((p.pf_mask >> wave) & 1u);
        if (has) issue(t, 0, wv);
        pf = has;
    };

    // A gathering wave holds no run-ahead task (pf_issue never gives wave 0, nor the h gatherers,
    // one): redefining the register set at the end of its gather ends the set's live range before
    // the gather, so the gather's loads get those registers instead of spilling.
    auto drop_wv = [&]() {
#pragma unroll
        for (int u = 0; u < kU; u++) wv[u][0] = wv[u][1] = u32x4{0u, 0u, 0u, 0u};
        pf = false;
    };

    // run this wave's local tasks [0, n) of a projection; mk(i) = the task, epi(i, a0, a1) =
    // lane 0's epilogue; nextf() issues the first task of the following projection
    auto run_tasks = [&](int n, const uint16_t* xs, auto&& mk, auto&& epi, auto&& nextf) {
        int i = wfirst;
        if (i >= n) {
            nextf();
            return;
        }
        Task t = mk(i);
        if (!pf) issue(t, 0, wv);
        pf = false;
        for (; i < n; i += kWaves) {
            const bool more = i + kWaves < n;
            Task tn = more ? mk(i + kWaves) : t;
            float a0, a1;
            run_task(t, xs, wv, a0, a1, [&] {
                if (more) issue(tn, 0, wv);
                else nextf();
            });
            if (lane == 0) epi(i, a0, a1);
            t = tn;
        }
    };

    // layer 0's first QKV task goes out before anything else (waves 1..7; wave 0 gathers)
    pf_issue(wave != 0 && wfirst < q1 - q0, qkv_task(0, q0 + (wfirst < q1 - q0 ? wfirst : 0)));

    // phase timestamps (diagnostics only: one uniform branch when off)
    auto ts = [&](int l, int slot) {
        if (p.ts && tid == 0)
            p.ts[((size_t)cu * p.n_layers + l) * kTsSlots + slot] = __builtin_amdgcn_s_memrealtime();
    };
    for (int l = 0; l < p.n_layers; l++) {
        const unsigned tg = tagl(l);
        ts(l, 0);
        // ============ QKV: x -> rms -> q, k, v (+bias)
        if (wave == 0) {
            // this CU's bias values and the norm weights first (no wait behind the gather)
            for (int i = lane; i < 2 * (q1 - q0); i += 64) {
                const int r = 2 * q0 + i;
                const uint16_t* b = (const uint16_t*)(r < QD ? PK_LW(LT, l, bq) : (r < QD + KD ? PK_LW(LT, l, bk) : PK_LW(LT, l, bv)));
                const int rr = r < QD ? r : (r < QD + KD ? r - QD : r - QD - KD);
                bias[i] = b ? bf2f(b[rr]) : -0.0f;   // -0 is the exact identity of + (no bias: v = acc)
            }
            for (int i = lane; i * 8 < H; i += 64)
                *reinterpret_cast<uint4*>(nw + i * 8) = *reinterpret_cast<const uint4*>((const uint16_t*)PK_LW(LT, l, attn_norm) + i * 8);
            if (l == 0) {
                for (int i = lane; i * 8 < H; i += 64)
                    *reinterpret_cast<uint4*>(xraw + i * 8) = *reinterpret_cast<const uint4*>(p.x_res + i * 8);
            } else {
                gather<kGatherX>(p.g_x, H / 2, tg, reinterpret_cast<uint32_t*>(xraw), lane, 64, p, dead, 1u);
            }
            drop_wv();
        }
        bar();
        ts(l, 1);
        if (*dead) return;
        ss_xfirst256(xraw, H, red);
        bar();
        {
            const float ss = ((red[1] + red[2]) + red[3]) + red[4];
            normalize(xraw, nw, xn, H, sqrtf((ss / (float)H) + p.eps), hf);
        }
        bar();
        run_tasks(
            q1 - q0, xn, [&](int i) { return qkv_task(l, q0 + i); },
            [&](int i, float a0, float a1) {
                stage[2 * i] = f2bf(a0 + bias[2 * i]);
                stage[2 * i + 1] = f2bf(a1 + bias[2 * i + 1]);
            },
            [&] {   // run-ahead: the O projection's first task (CUs owning O rows)
                const int i = wfirst;
                pf_issue(!att_cu && wave != 0 && i < o1 - o0, att_cu ? qkv_task(l, q0) : o_task(l, o0 + (i < o1 - o0 ? i : 0)));
            });
        bar();
        ts(l, 2);
        if (wave == 0)
            for (int i = lane; i < q1 - q0; i += 64)
                st_granule(p.g_qkv + q0 + i, tg, reinterpret_cast<const uint32_t*>(stage)[i]);
        // ============ attention (CUs [0, nA))
        if (att_cu) {
            const int g = cu / nsplit, s = cu % nsplit;
            DecodeAttnParams a = sld_struct(p.attp + l);   // layer, q / k norms set by the host
            a.qkv = hb;   // generic pointer into LDS: the body reads its row from the gathered image
            AttnHook<kThreads> hk;
            hk.g_qkv = p.g_qkv;
            hk.row = hb;
            hk.stage = astage;
            hk.o0 = (int64_t)g * G * HD;
            hk.g = g;
            hk.G = G;
            hk.hd = HD;
            hk.QD = QD;
            hk.KD = KD;
            hk.tag = tg;
            hk.p = &p;
            hk.dead = dead;
            const bool comb = attn_decode_mfma2_body<HD, false, kWaves, false, kDecMStep, AttnHook<kThreads>>(
                a, g * a.nsplit_max + s, 0, &hk);
            // the combiner's ticket reset (and every partial store) is performed before anything
            // this CU publishes later — the next layer's splits take tickets only after that
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (comb || nsplit == 1) {
                __syncthreads();
                for (int i = tid; i < G * HD / 2; i += kThreads)
                    st_granule(p.g_att + g * (G * HD / 2) + i, tg, reinterpret_cast<const uint32_t*>(astage)[i]);
            }
            __syncthreads();
            ts(l, 3);
            if (*dead) return;
            // no run-ahead task is pending here (pf is false on attention CUs): redefining the
            // register set ends its live range before the body, so the body gets those registers
#pragma unroll
            for (int u = 0; u < kU; u++) wv[u][0] = wv[u][1] = u32x4{0u, 0u, 0u, 0u};
        }
        // ============ O: attention out -> O rows (+residual) on the CUs that own them
        if (!att_cu) {
            if (wave == 0) {
                gather<kGatherX>(p.g_att, QD / 2, tg, reinterpret_cast<uint32_t*>(xn), lane, 64, p, dead, 3u);
                drop_wv();
            }
            bar();
            ts(l, 4);
            if (*dead) return;
        }
        run_tasks(
            att_cu ? 0 : o1 - o0, xn, [&](int i) { return o_task(l, o0 + i); },
            [&](int i, float a0, float a1) {
#pragma clang fp contract(off)
                const int r = 2 * (o0 + i);
                stage[2 * i] = f2bf(bf2f(xraw[r]) + rbf(a0));
                stage[2 * i + 1] = f2bf(bf2f(xraw[r + 1]) + rbf(a1));
            },
            [&] {   // run-ahead: gate/up's first task
                const int i = wfirst, n = 2 * (j1 - j0);
                pf_issue(wave != 0 && i < n, gu_task(l, 2 * j0 + (i < n ? i : 0)));
            });
        bar();
        ts(l, 5);
        if (wave == 0 && !att_cu)
            for (int i = lane; i < o1 - o0; i += 64)
                st_granule(p.g_x1 + o0 + i, tg, reinterpret_cast<const uint32_t*>(stage)[i]);
        // ============ gate/up: x' -> rms -> silu(gate) * up
        if (wave == 0) {
            for (int i = lane; i * 8 < H; i += 64)
                *reinterpret_cast<uint4*>(nw + i * 8) = *reinterpret_cast<const uint4*>((const uint16_t*)PK_LW(LT, l, ffn_norm) + i * 8);
            gather<kGatherX>(p.g_x1, H / 2, tg, reinterpret_cast<uint32_t*>(x1raw), lane, 64, p, dead, 4u);
            const float ss = ss_wave(x1raw, H);
            if (lane == 0) red[0] = ss;
            drop_wv();
        }
        bar();
        ts(l, 6);
        if (*dead) return;
        normalize(x1raw, nw, xn, H, sqrtf((red[0] / (float)H) + p.eps), hf);
        bar();
        run_tasks(
            2 * (j1 - j0), xn, [&](int i) { return gu_task(l, 2 * j0 + i); },
            [&](int i, float a0, float a1) {
#pragma clang fp contract(off)
                const float gg = rbf(a0);
                const float u = rbf(a1);
                const float a = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                stage[i] = f2bf(u * a);
            },
            [&] {   // run-ahead: down's first task (waves 4..7; waves 0..3 gather h)
                const int i = wfirst, n = d1 - d0;
                pf_issue(wave >= kWaves / 2 && i < n, dn_task(l, d0 + (i < n ? i : 0)));
            });
        bar();
        ts(l, 7);
        if (wave == 0)
            for (int i = lane; i < j1 - j0; i += 64)
                st_granule(p.g_h + j0 + i, tg, reinterpret_cast<const uint32_t*>(stage)[i]);
        // ============ down: h -> down rows (+residual) -> next layer's x
        if (wave < kWaves / 2) {   // the first half gathers h; the second has down's first tasks in flight
            gather<kGatherH>(p.g_h, I / 2, tg, reinterpret_cast<uint32_t*>(hb), tid, kThreads / 2, p, dead, 5u);
            drop_wv();
        }
        bar();
        ts(l, 8);
        if (*dead) return;
        const bool last = l + 1 == p.n_layers;
        run_tasks(
            d1 - d0, hb, [&](int i) { return dn_task(l, d0 + i); },
            [&](int i, float a0, float a1) {
#pragma clang fp contract(off)
                const int r = 2 * (d0 + i);
                stage[2 * i] = f2bf(bf2f(x1raw[r]) + rbf(a0));
                stage[2 * i + 1] = f2bf(bf2f(x1raw[r + 1]) + rbf(a1));
            },
            [&] {   // run-ahead: the next layer's first QKV task
                const int i = wfirst;
                pf_issue(!last && wave != 0 && i < q1 - q0, qkv_task(last ? l : l + 1, q0 + (i < q1 - q0 ? i : 0)));
            });
        bar();
        ts(l, 9);
        if (wave == 0) {
            if (last) {
                for (int i = lane; i < d1 - d0; i += 64)
                    reinterpret_cast<uint32_t*>(p.x_res)[d0 + i] = reinterpret_cast<const uint32_t*>(stage)[i];
            } else {
                for (int i = lane; i < d1 - d0; i += 64)
                    st_granule(p.g_x + d0 + i, tagl(l + 1), reinterpret_cast<const uint32_t*>(stage)[i]);
            }
        }
    }
}

}  // namespace pk

int decode_attn_params(DecodeAttnParams* a, const void* qkv, int64_t B, const int32_t* pos, const void* q_norm,
                       const void* k_norm, const float* rope_cos, const float* rope_sin, int32_t n_heads,
                       const qie_kv_cache* cache, int32_t layer, float eps, int32_t numerics, void* out, void* ws);

// ------------------------------------------------------------------ host side
size_t persist_lds_bytes(int H, int I, int QD, int KD, int G, int hd) {
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const int QKVD = QD + 2 * KD;
    return al(H * 2) * 3 + al((size_t)(H > QD ? H : QD) * 2) + al((size_t)(I > QKVD ? I : QKVD) * 2) +
           al(pk::kStage * 2) + al((size_t)G * hd * 2) + al(pk::kMaxBias * 4) + 64 + 16;
}

// Which models / batches the persistent step covers (the launch path serves the rest):
// batch 1, bf16 weights, one device, head_dim 128, a contiguous KV cache, and per-CU output
// ranges that fit the kernel's LDS staging.
bool persist_supported(const qie_model_spec& s, int B, int tp, bool fp8, bool paged, int ncu, const char** why) {
    const int QD = s.n_heads * s.head_dim, KD = s.n_kv_heads * s.head_dim;
    const int G = s.n_heads / s.n_kv_heads;
    auto no = [&](const char* w) {
        if (why) *why = w;
        return false;
    };
    if (B != 1) return no("batch != 1");
    if (tp != 1) return no("tensor parallel");
    if (fp8) return no("fp8 weights");
    if (paged) return no("paged KV cache");
    if (s.head_dim != 128 && s.head_dim != 64) return no("head_dim not 64 or 128");
    if (s.hidden % 16 || s.ffn % 16 || QD % 16 || KD % 16) return no("widths not multiples of 16");
    // every CU owns at least one down granule: the x hand-off then orders every CU's reads of a
    // layer's buffers before any write of the next layer's (k_persist.hip header)
    if (s.hidden / 2 < ncu) return no("hidden / 2 < CUs");
    if (G > 8) return no("group > 8");
    const int nw = s.head_dim == 128 ? 8 : 4;
    if (s.hidden / 2 > 64 * pk::kGatherX || QD / 2 > 64 * pk::kGatherX || s.ffn / 2 > 32 * nw * pk::kGatherH)
        return no("widths beyond the gather capacity");
    const int nsplit_max = 32;
    if (s.n_kv_heads * nsplit_max >= ncu) return no("too few CUs for the attention jobs");
    const int QKVD = QD + 2 * KD;
    const int per_cu = std::max({QKVD / 2 / ncu + 2, s.hidden / 2 / (ncu - s.n_kv_heads * nsplit_max) + 2,
                                 s.ffn / 2 / ncu + 2});
    if (2 * per_cu > pk::kStage || 2 * (QKVD / 2 / ncu + 2) > pk::kMaxBias) return no("per-CU ranges too large");
    if (persist_lds_bytes(s.hidden, s.ffn, QD, KD, G, s.head_dim) + 48 * 1024 > 160 * 1024) return no("LDS");
    return true;
}

// The attention role's parameters of every layer (what the stand-alone decode attention
// launch of that layer would get: qie_attention_decode's fill), uploaded once per batch into
// d_attp (persist_attn_table_bytes).  h_layers: the engine's host copy of the layer table.
size_t persist_attn_table_bytes(int n_layers) { return sizeof(DecodeAttnParams) * (size_t)n_layers; }

int persist_attn_table(const qie_model_spec& s, const qie_layer_weights* h_layers, const void* qkv_scratch,
                       const int32_t* pos, const float* rope_cos, const float* rope_sin, const qie_kv_cache* cache,
                       void* dec_ws, void* d_attp, hipStream_t st) {
    std::vector<DecodeAttnParams> t(s.n_layers);
    for (int l = 0; l < s.n_layers; l++) {
        QIE_TRY(decode_attn_params(&t[l], qkv_scratch, 1, pos, h_layers[l].q_norm, h_layers[l].k_norm, rope_cos,
                                   rope_sin, s.n_heads, cache, l, s.rms_eps, s.numerics, (void*)qkv_scratch, dec_ws));
        QIE_REQUIRE(t[l].ks == kDecMStep && !t[l].pre_roped && t[l].nsplit_max <= kDecMSplits,
                    "persistent decode: unsupported attention step");
    }
    QIE_HIP(hipMemcpyAsync(d_attp, t.data(), sizeof(DecodeAttnParams) * t.size(), hipMemcpyHostToDevice, st));
    return 0;
}

int persist_decode_launch(const qie_model_spec& s, const qie_layer_weights* d_layers, const void* d_attp,
                          uint16_t* x_res, unsigned long long* granules, const unsigned* epoch, unsigned* err,
                          const int32_t* pos, int splits_target, unsigned long long* ts, hipStream_t st) {
    pk::Params p;
    p.layers = d_layers;
    p.n_layers = s.n_layers;
    p.H = s.hidden;
    p.I = s.ffn;
    p.QD = s.n_heads * s.head_dim;
    p.KD = s.n_kv_heads * s.head_dim;
    p.nq = s.n_heads;
    p.nkv = s.n_kv_heads;
    p.hd = s.head_dim;
    p.eps = s.rms_eps;
    p.numerics = s.numerics;
    p.x_res = x_res;
    const int QKVD = p.QD + 2 * p.KD;
    p.g_x = granules;
    p.g_qkv = p.g_x + s.hidden / 2;
    p.g_att = p.g_qkv + QKVD / 2;
    p.g_x1 = p.g_att + p.QD / 2;
    p.g_h = p.g_x1 + s.hidden / 2;
    p.epoch = epoch;
    p.err = err;
    p.spin_ticks = 20000000;   // 200 ms at 100 MHz: far beyond any step; only a fault waits it out
    p.attp = (const DecodeAttnParams*)d_attp;
    p.pos = pos;
    p.splits_target = splits_target;
    p.ts = ts;
    p.pf_mask = (unsigned)dev_env("QIE_PK_PF_MASK", 0xFF);
    p.xw_even = dev_env("QIE_PK_XW", 100);
    const size_t shm = persist_lds_bytes(p.H, p.I, p.QD, p.KD, p.nq / p.nkv, p.hd);
    const void* fn = s.head_dim == 128 ? (const void*)pk::decode_layers_kernel<128> : (const void*)pk::decode_layers_kernel<64>;
    static bool raised[2] = {false, false};
    bool& r = raised[s.head_dim == 128 ? 1 : 0];
    if (!r) {
        QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm + 4096));
        r = true;
    }
    if (s.head_dim == 128)
        hipLaunchKernelGGL(pk::decode_layers_kernel<128>, dim3((unsigned)device_cu_count()), dim3(64 * pk::waves_for<128>()),
                           shm, st, p);
    else
        hipLaunchKernelGGL(pk::decode_layers_kernel<64>, dim3((unsigned)device_cu_count()), dim3(64 * pk::waves_for<64>()),
                           shm, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

int persist_ts_slots() { return pk::kTsSlots; }

int64_t persist_granule_count(const qie_model_spec& s) {
    const int QD = s.n_heads * s.head_dim, KD = s.n_kv_heads * s.head_dim;
    return (int64_t)s.hidden / 2 * 2 + (QD + 2 * KD) / 2 + QD / 2 + s.ffn / 2;
}

}  // namespace qie
