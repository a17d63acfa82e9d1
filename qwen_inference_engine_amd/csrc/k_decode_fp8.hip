// k_decode_fp8.hip — batched decode projections on fp8 weights (2 <= M <= 16 rows).
//
// Replaces matrix_mul (layers/src/matrix_mul.cu:165-288) for the batched decode step of
// BASELINE config 4 (Qwen2-7B, e4m3 weights with a power-of-two row scale, batch 8), plus
// the launch_rms that precedes the QKV and gate/up projections (normalization.cu:5-25).
//
// The general skinny kernel (k_gemv.hip skinny_mfma_kernel) re-reads its A fragments (the
// M activation rows) from LDS or L2 for every 64-k unit of every column tile and merges
// its waves' partial tiles behind two barriers per tile; at config 4 it was issue-bound
// (16 VALU per MFMA, 47 % of wave-cycles waiting for issue, profiles/r02_pmc_skinny_b8.txt).
// Here the work is laid out so that the loop is only loads, conversions and MFMAs:
//   * a block of KS waves owns whole 16-column tiles; wave w owns the SAME K slice
//     [w·KU·64, (w+1)·KU·64) of every tile, so its A fragments (16 rows × its K slice,
//     KU·2 16-B vectors per lane) are loaded ONCE per launch and stay in registers;
//   * the RMSNorm is fused: the block's waves together hold every row's whole K range, so
//     the sum of squares is one wave reduction + one LDS exchange, and each wave
//     normalises its own fragments in registers (no qie_rmsnorm launch in front; the norm
//     weights are staged in LDS, the quotient is a Markstein step, see d8_rms_pair);
//   * weights: one 16-B buffer load per lane per 64-k unit (16 e4m3 codes of one row;
//     lanes 16g..16g+15 = rows, g = k quarter), non-temporal, in half-tile steps with
//     the next step always in flight (two register sets); one v_cvt_scalef32_pk_bf16_fp8 per code pair, two
//     v_mfma_f32_16x16x32_bf16 per unit (rows ≥ M are padding, never stored);
//   * the KS partial C tiles meet in a double-buffered LDS area: ONE barrier per tile,
//     the epilogue (row scale, bias / residual / SwiGLU / fp32 / arg-max keys) by a wave
//     that rotates with the tile so no wave carries every epilogue.
// Numerics: the dequantised products (e4m3 × 2^k is exact in bf16) accumulate in fp32 per
// wave over its K slice, the KS slices are added in wave order, times the row scale; the
// epilogues round exactly as the reference's separate kernels (bf16 after each op).
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <type_traits>

namespace qie {

typedef unsigned int d8_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 d8_bf16x8 __attribute__((ext_vector_type(8)));
typedef float d8_f32x4 __attribute__((ext_vector_type(4)));

struct Dec8Params {
    const uint16_t* x;         // [M][ldx] bf16 activation rows
    int64_t ldx;
    const uint16_t* norm_w;    // fused RMSNorm weights (null: rows used as they are)
    float eps;
    int numerics;
    const uint8_t* w[3];       // segment bases: [rows][K] e4m3 codes, then rows fp32 scales
    const uint16_t* bias[3];   // per segment, may be null
    int32_t seg_rows[3];
    int32_t t01[2];            // tiles in segment 0, in segments 0 + 1
    int32_t K, N, M;
    int32_t n_tiles;
    uint16_t* y;               // [M][ldy] (fp32 for QIE_EPI_F32)
    int64_t ldy;
    unsigned long long* keys;  // arg-max keys per row (STORE), may be null
    int64_t key_col0;
    int dbg;                   // development build only (QIE_DEC8_DBG): 2 skips the fused norm
    // split-K (SPL instantiations only; long K such as the down projection's 18,944): the K
    // units are cut into `parts` slices of KS * KU units (the last one ragged), block b serves
    // part b % parts; each part's reduced 16 x 16 fp32 tile goes write-through to slab
    // [tile][part] and the last arriving part (ticket cnt[tile]) sums them in part order
    int parts;
    float* slab;
    unsigned* cnt;
};

// One bf16 pair of qie_rmsnorm's rms_apply8 (k_misc.hip, normalization.cu:18-23).
// REF: x / rms as q = x * (1 / rms) plus one FMA residual step (Markstein) — the correctly
// rounded quotient whenever nothing underflows, i.e. for every |x / rms| above 2^-100
// (smaller non-zero activations may land 1 fp32 ulp off before the bf16 rounding); three
// VALU ops instead of the ~10 of the IEEE division sequence, which made the fused prologue
// VALU-bound (13 µs per launch at config 4).  rms = +inf enters as rr = 0, inv = 0, so the
// quotient is 0 for finite x and NaN for infinite x, as the division gives.
// HF: w * bf16(x * (1 / rms)).
template <bool HF>
__device__ __forceinline__ uint32_t d8_rms_pair(uint32_t xv, uint32_t wv, float rr, float inv) {
#pragma clang fp contract(off)
    const float a[2] = {bf_lo(xv), bf_hi(xv)}, w[2] = {bf_lo(wv), bf_hi(wv)};
    float y[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const float q = a[j] * inv;
        y[j] = HF ? w[j] * rbf(q) : fmaf(fmaf(-q, rr, a[j]), inv, q) * w[j];
    }
    return pack2(y[0], y[1]);
}

// (split-K: two blocks per CU — at most 128 VGPRs; one block per CU ran the down projection
// at 24.8 instead of 18.5 µs)
// (The bound's second argument is HIP's minimum waves per SIMD: 4 = 128 VGPRs.  Measured
// and dropped: the LDS-form QKV at 128 VGPRs, two blocks per CU so that config 4's 288
// column tiles run in one round — 10.3 vs 8.85 µs, it spills.)
template <int EPI, int KU, int KS, bool SPL = false, bool T16 = false, bool LF = false>
__global__ __launch_bounds__(KS * 64, SPL ? 4 : 1) void dec8_kernel(Dec8Params p) {
#pragma clang fp contract(off)
    static_assert(!SPL || EPI != QIE_EPI_SWIGLU, "split-K: single-segment epilogues");
    constexpr int NB = EPI == QIE_EPI_SWIGLU ? 2 : 1;   // B tiles per column tile (gate, up)
    constexpr int kNT = 2;                               // buffer-load policy: nt (streamed once)
    // per-wave partial C tiles: RDF slots of KS x NB 16 x 16 fp32 tiles, sized so that the
    // kernel's static LDS stays within 64 KiB.  A block whose tiles fit keeps each tile's
    // partials until its last tile and reduces them all after ONE barrier (the per-tile
    // barrier held every wave to the slowest at each tile: config-4 gate/up 28.7 vs 24.7 µs
    // without it, measured with the hand-off removed); with M <= 8 only rows 0..7 (lanes
    // 0..31) matter, so a slot holds two tiles.  More tiles: per-tile hand-off through two slots.
    constexpr int RDF = (57344 / (KS * NB * 1024)) < 2 ? 2 : (57344 / (KS * NB * 1024));
    __shared__ __attribute__((aligned(16))) float red[RDF][KS][NB][256];
    __shared__ float ssq[KS][16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const int M = p.M, K = p.K, T = p.n_tiles;
    // block -> (first tile bi, tile stride G, K part); without split: part 0, G = grid
    const int part = SPL ? (int)blockIdx.x % p.parts : 0;
    const int bi = SPL ? (int)blockIdx.x / p.parts : (int)blockIdx.x;
    const int G = SPL ? (int)gridDim.x / p.parts : (int)gridDim.x;
    if (bi >= T || bi >= G) return;   // block-uniform, before any barrier
    const int my = (T - 1 - bi) / G + 1;
    const int arow = fr < M ? fr : M - 1;
    const int kw = (part * KS + wave) * (KU * 64);
    // units of this wave past K (the ragged last part): A fragments 0, weight loads out of
    // the buffer range (0) — wave-uniform, and no load sits under a branch
    const int kval = SPL ? (K - kw) / 64 : KU;   // valid units (may be <= 0 or > KU)

    // LDS form of the fused RMSNorm (round 5; M <= 8, one block of KS waves holding whole
    // rows: K = KS x 512): thread t loads chunk t (8 values) of every REAL row once, the
    // rows' sums of squares meet by a transposed butterfly + one LDS exchange, each thread
    // normalises its chunks into an LDS image of the M rows (aliasing the partial-tile area,
    // unused until the first tile ends), and every lane then reads its A fragments from
    // that image.  The register form below loads and normalises 16 rows per wave — the
    // padding rows of the 16-row MFMA operand included, i.e. twice the x traffic through
    // the CU and twice the normalisation VALU at M = 8.  QIE_DEC8_DBG & 32 (dev): register form.
    // A separate instantiation (LF), launched only with a norm and M <= 8: one kernel
    // holding both forms spilled (the register form's live A fragments + the chunk loads).
    constexpr bool LFORM = LF && !SPL && KU == 8 && RDF * NB >= 8;   // image of 8 rows x 512 per wave fits red[]
    static_assert(!LF || LFORM, "dec8: LDS-form norm needs KU = 8, no split, an 8-row image in red[]");
    d8_u32x4 xc[LFORM ? 8 : 1];
    if constexpr (LFORM) {
#pragma unroll
        for (int j = 0; j < 8; j++)
            xc[j] = j < M ? *reinterpret_cast<const d8_u32x4*>(p.x + (int64_t)j * p.ldx + 8 * tid) : d8_u32x4{0u, 0u, 0u, 0u};
    }

    // ---- A fragments of this wave's K slice: row arow, k = kw + 64 u + 16 g + [0, 16)
    d8_u32x4 av[KU][2];
    if constexpr (!LFORM) {
        const d8_u32x4* xp = reinterpret_cast<const d8_u32x4*>(p.x + (int64_t)arow * p.ldx + (SPL ? 0 : kw) + 16 * g);
#pragma unroll
        for (int u = 0; u < KU; u++) {
            if constexpr (SPL) {
                const int ok = u < kval;
                const int o = ok ? (kw / 8 + 8 * u) : 0;
                const d8_u32x4 z = d8_u32x4{0u, 0u, 0u, 0u};
                const d8_u32x4 v0 = xp[o], v1 = xp[o + 1];
                av[u][0] = ok ? v0 : z;
                av[u][1] = ok ? v1 : z;
            } else {
                av[u][0] = xp[8 * u];
                av[u][1] = xp[8 * u + 1];
            }
        }
    }
    // this wave's slice of the norm weights: one 16-B load per lane (k = kw + 8 lane), staged
    // in LDS for the apply below (a register copy per fragment doubled the prologue's
    // footprint and spilled)
    __shared__ __attribute__((aligned(16))) d8_u32x4 nw_s[KS][KU * 8];
    const bool nrm = p.norm_w != nullptr && !QIE_DBG(p.dbg & 2);   // launch-uniform
    const d8_u32x4 nwv = *reinterpret_cast<const d8_u32x4*>((nrm ? p.norm_w : p.x) + kw + 8 * (lane < KU * 8 ? lane : 0));

    // A step = half a tile's units (KH per B tile) of one column tile; two steps are in
    // flight (double-buffered registers), i.e. one tile of weights per wave ahead
    constexpr int KH = KU / 2;
    struct Step {
        d8_u32x4 wv[NB][KH];
        float sc[NB];
        float ep[4];   // residual values (rows 4 g + r) or the bias (ep[0])
    };
    // loads of step s: every load unconditional (clamped), so none sits under a branch
    // (a load under a branch costs a vmcnt(0) at the join)
    // hf (which half of the tile) is a constant at every call site: the epilogue operands
    // ride with the second half only
    auto issue = [&](Step& t, int it, int hf) {
        const int tile = bi + it * G;
        const int sg = NB == 2 ? 0 : (tile < p.t01[0] ? 0 : (tile < p.t01[1] ? 1 : 2));
        const int tb0 = sg == 0 ? 0 : (sg == 1 ? p.t01[0] : p.t01[1]);
        const int rows = p.seg_rows[sg];
        int r = (tile - tb0) * 16 + fr;
        r = r < rows ? r : rows - 1;
        // plain layout: lane (fr, g) reads row r, columns kw + 64 u + 16 g + [0, 16) — one load
        // instruction touches 16 rows x 64 B; 16-row tiled layout (T16, qie_fp8_tile16): the
        // same fragment is bytes 16 lane of the unit's 1-KiB block — 8 whole 128-B lines
        constexpr int UST = T16 ? 1024 : 64;
        const int voff = T16 ? (tile - tb0) * 16 * K + kw * 16 + hf * (KH * 1024) + lane * 16
                             : r * K + kw + 16 * g + hf * (KH * 64);
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const uint8_t* base = p.w[NB == 2 ? b : sg];
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0,
                                                              (int)((int64_t)rows * (K + 4)), 0x00020000);
#pragma unroll
            for (int u = 0; u < KH; u++) {
                if constexpr (SPL)
                    t.wv[b][u] = __builtin_amdgcn_raw_buffer_load_b128(
                        rs, hf * KH + u < kval ? voff + u * UST : 0x7ffffff0, 0, kNT);
                else
                    t.wv[b][u] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, u * UST, kNT);
            }
            if (hf) t.sc[b] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, rows * K + r * 4, 0, 0));
        }
        if (!hf) return;
        const int n = tile * 16 + fr;
        const int nc = n < p.N ? n : p.N - 1;
        if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int i = 4 * g + rr < M ? 4 * g + rr : M - 1;
                t.ep[rr] = bf2f(p.y[(int64_t)i * p.ldy + nc]);
            }
        } else if constexpr (EPI == QIE_EPI_STORE) {
            const uint16_t* bp = p.bias[sg];
            const float v = bf2f((bp ? bp : p.x)[bp ? r : 0]);
            t.ep[0] = bp ? v : 0.f;
        }
    };

    Step sa, sb;
    issue(sa, 0, 0);
    __builtin_amdgcn_sched_barrier(0);

    // ---- fused RMSNorm: row arow's sum of squares over the whole K (this wave's slice,
    // the 4 k quarters by lane exchange, the KS slices through LDS), then the fragments are
    // normalised in place (qie_rmsnorm's arithmetic)
    if constexpr (LFORM) {
        // sums of squares of this thread's chunk of each row (8 values in order)
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t e4[4] = {xc[j].x, xc[j].y, xc[j].z, xc[j].w};
            float a = 0.f;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float l = bf_lo(e4[i]), hh = bf_hi(e4[i]);
                a += l * l + hh * hh;
            }
            v[j] = a;
        }
        // transposed butterfly: 8 row partials over 64 lanes -> lane l holds the wave's sum
        // of row 4 (l>>5) + 2 ((l>>4)&1) + ((l>>3)&1) (lane ^ 32, ^ 16, ^ 8 halve the rows,
        // then the 8-lane group sums); fixed order, independent of M
        float w4[4], w2[2];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            float a = v[i], b = v[4 + i];
            lane_swap<32>(a, b);
            w4[i] = a + b;
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            float a = w4[i], b = w4[2 + i];
            lane_swap<16>(a, b);
            w2[i] = a + b;
        }
        const bool b8 = (lane & 8) != 0;
        const float w1 = (b8 ? w2[1] : w2[0]) + dpp_f<0x128>(b8 ? w2[0] : w2[1]);   // row_ror 8 = lane ^ 8
        const float ssw = group_sum<8>(w1);
        if ((lane & 7) == 0) ssq[wave][4 * (lane >> 5) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1)] = ssw;
        __syncthreads();
        // lanes 0..7: row (lane & 7)'s statistics; chunk j reads row j's by readlane
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < KS; w++) tot += ssq[w][lane & 7];
        const float rms = sqrtf((tot / (float)K) + p.eps);
        const float inv = 1.0f / rms;
        const float rr = rms < INFINITY ? rms : 0.f;
        uint16_t* xs = reinterpret_cast<uint16_t*>(&red[0][0][0][0]);
        auto apply = [&](auto hf) {
            constexpr bool HF = decltype(hf)::value;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (j >= M) break;   // uniform
                const float ij = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, inv), j));
                const float rj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, rr), j));
                d8_u32x4 y;
                y.x = d8_rms_pair<HF>(xc[j].x, nwv.x, rj, ij);
                y.y = d8_rms_pair<HF>(xc[j].y, nwv.y, rj, ij);
                y.z = d8_rms_pair<HF>(xc[j].z, nwv.z, rj, ij);
                y.w = d8_rms_pair<HF>(xc[j].w, nwv.w, rj, ij);
                *reinterpret_cast<d8_u32x4*>(xs + (int64_t)j * K + 8 * tid) = y;
            }
        };
        if (p.numerics == QIE_NUMERICS_HF) apply(std::true_type{});
        else apply(std::false_type{});
        __syncthreads();
#pragma unroll
        for (int u = 0; u < KU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++)
                av[u][h] = *reinterpret_cast<const d8_u32x4*>(xs + (int64_t)arow * K + kw + 64 * u + 16 * g + 8 * h);
        __syncthreads();   // the image is red[]: every wave has its fragments before any tile ends
    } else if (nrm) {   // register form
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < KU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t e4[4] = {av[u][h].x, av[u][h].y, av[u][h].z, av[u][h].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float l = bf_lo(e4[j]), hh = bf_hi(e4[j]);
                    ss += l * l + hh * hh;
                }
            }
        ss = xor32_sum(xor16_sum(ss));
        if (g == 0) ssq[wave][fr] = ss;
        if (lane < KU * 8) nw_s[wave][lane] = nwv;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < KS; w++) tot += ssq[w][fr];
        const float rms = sqrtf((tot / (float)K) + p.eps);
        const float inv = 1.0f / rms;
        const float rr = rms < INFINITY ? rms : 0.f;
        // the numerics are launch-uniform: one unrolled copy per mode, only one runs
        auto apply = [&](auto hf) {
            constexpr bool HF = decltype(hf)::value;
#pragma unroll
            for (int u = 0; u < KU; u++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const d8_u32x4 nv = nw_s[wave][8 * u + 2 * g + h];   // k = kw + 64 u + 16 g + 8 h
                    av[u][h].x = d8_rms_pair<HF>(av[u][h].x, nv.x, rr, inv);
                    av[u][h].y = d8_rms_pair<HF>(av[u][h].y, nv.y, rr, inv);
                    av[u][h].z = d8_rms_pair<HF>(av[u][h].z, nv.z, rr, inv);
                    av[u][h].w = d8_rms_pair<HF>(av[u][h].w, nv.w, rr, inv);
                    // one fragment at a time: left alone the scheduler hoists every
                    // product of the prologue first and spills
                    __builtin_amdgcn_sched_barrier(0);
                }
        };
        __builtin_amdgcn_sched_barrier(0);
        if (p.numerics == QIE_NUMERICS_HF) apply(std::true_type{});
        else apply(std::false_type{});
        __builtin_amdgcn_sched_barrier(0);
    }

    unsigned long long kbest[4] = {0ull, 0ull, 0ull, 0ull};
    d8_f32x4 acc[NB];
    auto mma = [&](const Step& t, int hf) {
        if (hf == 0) {
#pragma unroll
            for (int b = 0; b < NB; b++) acc[b] = d8_f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < KH; u++) {
            const int ua = hf * KH + u;   // (hf is a compile-time constant at every call)
            const d8_bf16x8 a0 = __builtin_bit_cast(d8_bf16x8, av[ua][0]);
            const d8_bf16x8 a1 = __builtin_bit_cast(d8_bf16x8, av[ua][1]);
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const uint2 c0 = fp8x4_to_bf16x4(t.wv[b][u].x), c1 = fp8x4_to_bf16x4(t.wv[b][u].y);
                const uint2 c2 = fp8x4_to_bf16x4(t.wv[b][u].z), c3 = fp8x4_to_bf16x4(t.wv[b][u].w);
                const d8_u32x4 lo = d8_u32x4{c0.x, c0.y, c1.x, c1.y};
                const d8_u32x4 hi = d8_u32x4{c2.x, c2.y, c3.x, c3.y};
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, __builtin_bit_cast(d8_bf16x8, lo), acc[b], 0, 0, 0);
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, __builtin_bit_cast(d8_bf16x8, hi), acc[b], 0, 0, 0);
            }
        }
    };
    // tile end (after its second step): partial tiles -> LDS, one barrier, epilogue
    // the epilogue of one output tile from its fp32 sums (before the row scale)
    auto emit = [&](int tile, const float (&sum)[NB][4], const float* scv, const float* epv) {
        const int n = tile * 16 + fr;
        float c[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int r = 0; r < 4; r++) c[b][r] = sum[b][r] * scv[b];
        if (n >= p.N) return;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int i = 4 * g + r;
            if (i >= M) continue;
            uint16_t* yr = p.y + (int64_t)i * p.ldy;
            if constexpr (EPI == QIE_EPI_SWIGLU) {
                const float gg = rbf(c[0][r]);
                const float uu = rbf(c[1][r]);
                const float a = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                yr[n] = f2bf(uu * a);
            } else if constexpr (EPI == QIE_EPI_RESIDUAL) {
                yr[n] = f2bf(epv[r] + rbf(c[0][r]));
            } else if constexpr (EPI == QIE_EPI_F32) {
                reinterpret_cast<float*>(p.y)[(int64_t)i * p.ldy + n] = c[0][r];
            } else {
                const uint16_t o = f2bf(c[0][r] + epv[0]);
                yr[n] = o;
                if (p.keys) {
                    const unsigned long long kk = sel_key(bf2f(o), (uint32_t)(n + p.key_col0));
                    kbest[r] = kk > kbest[r] ? kk : kbest[r];
                }
            }
        }
    };
    const bool half = M <= 8;                                   // rows 0..7: lanes 0..31
    // (dev A/B QIE_DEC8_DBG & 16: the per-tile hand-off everywhere; split-K needs the deferred form)
    // Blocks of one or two tiles keep the per-tile form: deferring saves at most one barrier
    // there and reloads the row scales / epilogue operands the steps already hold (O, one
    // tile per block: 5.95 -> 6.29 µs deferred)
    const bool defer = (SPL || (my >= 3 && !QIE_DBG(p.dbg & 16))) && my <= (half ? 2 * RDF : RDF);   // block-uniform
    // where tile it's partial of wave w, B tile b, lives (lane-indexed float4)
    auto slot_at = [&](int it, int w, int b) -> float* {
        if (defer && half) return &red[it >> 1][w][b][(it & 1) * 128 + lane * 4];
        return &red[defer ? it : (it & 1)][w][b][lane * 4];
    };
    // the KS waves' partials of tile it, summed in wave order (the same order either way;
    // lanes past row 7 read another tile's slot in the packed form: their rows are >= M)
    auto reduce = [&](int it, float (&sum)[NB][4]) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
            float4 v4 = *reinterpret_cast<const float4*>(slot_at(it, 0, b));
#pragma unroll
            for (int w = 1; w < KS; w++) {
                const float4 v = *reinterpret_cast<const float4*>(slot_at(it, w, b));
                v4.x += v.x; v4.y += v.y; v4.z += v.z; v4.w += v.w;
            }
            sum[b][0] = v4.x; sum[b][1] = v4.y; sum[b][2] = v4.z; sum[b][3] = v4.w;
        }
    };
    // the row scales and epilogue operands of a tile, reloaded (deferred epilogues; the
    // per-tile path has them from the tile's step loads, issue())
    auto load_epi = [&](int tile, float (&scv)[NB], float (&epv)[4]) {
        const int sg = NB == 2 ? 0 : (tile < p.t01[0] ? 0 : (tile < p.t01[1] ? 1 : 2));
        const int tb0 = sg == 0 ? 0 : (sg == 1 ? p.t01[0] : p.t01[1]);
        const int rows = p.seg_rows[sg];
        int r = (tile - tb0) * 16 + fr;
        r = r < rows ? r : rows - 1;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.w[NB == 2 ? b : sg]), (short)0,
                                                              (int)((int64_t)rows * (K + 4)), 0x00020000);
            scv[b] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, rows * K + r * 4, 0, 0));
        }
        epv[0] = epv[1] = epv[2] = epv[3] = 0.f;
        const int n = tile * 16 + fr;
        const int nc = n < p.N ? n : p.N - 1;
        if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int i = 4 * g + rr < M ? 4 * g + rr : M - 1;
                epv[rr] = bf2f(p.y[(int64_t)i * p.ldy + nc]);
            }
        } else if constexpr (EPI == QIE_EPI_STORE) {
            const uint16_t* bp = p.bias[sg];
            epv[0] = bp ? bf2f(bp[r]) : 0.f;
        }
    };
    // tile end (after its second step): this wave's partial tile -> LDS; deferred: nothing
    // else until the block's last tile; else one barrier and the rotating wave's epilogue
    auto finish = [&](const Step& t, int it) {
        if (!(defer && half) || lane < 32) {
#pragma unroll
            for (int b = 0; b < NB; b++)
                *reinterpret_cast<float4*>(slot_at(it, wave, b)) = make_float4(acc[b][0], acc[b][1], acc[b][2], acc[b][3]);
        }
        if (defer) return;   // block-uniform
        // one barrier per tile: the next write of a slot is two tiles away, behind the
        // next tile's barrier, which the epilogue wave reaches only after its reads
        __syncthreads();
        if constexpr (!SPL) {   // (split-K blocks always defer: dec8_launch caps their tiles)
            if (wave != it % KS) return;   // wave-uniform
            float sum[NB][4];
            reduce(it, sum);
            emit(bi + it * G, sum, t.sc, t.ep);
        }
    };

    // split-K tail of tile it (wave it % KS... any wave): publish this part's sums
    // write-through, drain, take the ticket; the last arriver sums every part in part order
    // (independent of arrival order), reloads the row scale and epilogue operands, emits
    auto split_tail = [&](int it) {
        const int tile = bi + it * G;
        float* tb = p.slab + (int64_t)tile * p.parts * 256;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(tb, (short)0, p.parts * 1024, 0x00020000);
        float ks[NB][4];
        reduce(it, ks);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(d8_u32x4, d8_f32x4{ks[0][0], ks[0][1], ks[0][2], ks[0][3]}), rs,
                                               part * 1024 + lane * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(p.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __shfl(old, 0, 64);
        if (old != (unsigned)p.parts - 1) return;   // wave-uniform
        const int rows = p.seg_rows[0];
        int r = tile * 16 + fr;
        r = r < rows ? r : rows - 1;
        const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.w[0]), (short)0,
                                                          (int)((int64_t)rows * (K + 4)), 0x00020000);
        float scv[NB], epv[4] = {0.f, 0.f, 0.f, 0.f};
        scv[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, rows * K + r * 4, 0, 0));
        const int n = tile * 16 + fr;
        const int nc = n < p.N ? n : p.N - 1;
        if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int i = 4 * g + rr < M ? 4 * g + rr : M - 1;
                epv[rr] = bf2f(p.y[(int64_t)i * p.ldy + nc]);
            }
        } else if constexpr (EPI == QIE_EPI_STORE) {
            const uint16_t* bp = p.bias[0];
            epv[0] = bp ? bf2f(bp[r]) : 0.f;
        }
        float sum[NB][4];
        for (int q = 0; q < p.parts; q++) {
            const d8_f32x4 v = __builtin_bit_cast(d8_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 1024 + lane * 16, 0, 16));
#pragma unroll
            for (int j = 0; j < 4; j++) sum[0][j] = q == 0 ? v[j] : sum[0][j] + v[j];
        }
        if (lane == 0) __hip_atomic_store(p.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        emit(tile, sum, scv, epv);
    };

    // steps alternate sa (first half of a tile) / sb (second half); the next step is
    // always issued before this one is computed
    __builtin_amdgcn_sched_barrier(0);
    int it = 0;
    for (; it + 1 < my; it++) {
        issue(sb, it, 1);
        mma(sa, 0);
        issue(sa, it + 1, 0);
        mma(sb, 1);
        finish(sb, it);
    }
    issue(sb, it, 1);
    mma(sa, 0);
    mma(sb, 1);
    finish(sb, it);
    if (defer) {   // block-uniform: every wave's partials of every tile are in red[]
        __syncthreads();
        for (int t2 = wave; t2 < my; t2 += KS) {
            if constexpr (SPL) {
                split_tail(t2);
            } else {
                float sum[NB][4], scv[NB], epv[4];
                load_epi(bi + t2 * G, scv, epv);
                reduce(t2, sum);
                emit(bi + t2 * G, sum, scv, epv);
            }
        }
    }
    if constexpr (EPI == QIE_EPI_STORE) {
        if (p.keys) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                unsigned long long v = kbest[r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {   // max over the 16 columns of row 4 g + r
                    const unsigned long long s = __shfl_xor(v, o, 64);
                    v = s > v ? s : v;
                }
                if (fr == 0 && 4 * g + r < M && v) atomicMax(p.keys + 4 * g + r, v);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// dec8r (round 4): dec8 with the A fragments in LDS and a 4-deep register ring of weight
// steps.  In dec8 the A fragments (16 rows x the wave's K slice, rows >= M padding) held 64
// VGPRs per wave for the whole launch, leaving room for only two half-tile steps in flight
// (~112 KB per CU at config 4's gate/up, 4.0 TB/s, where the bf16 GEMV keeps ~200 KB in
// flight per CU and streams at 6.3 TB/s).  Here the normalised fragments go to LDS once
// (only the AR = 8 or 16 real row slots; a lane's own slice, so no barrier), each unit reads
// its two 16-B fragments back with ds_read_b128, and the freed registers hold FOUR
// half-tile steps, three in flight while one is computed.  Steps past the block's last
// tile load through a zero-sized buffer range (no memory traffic, no branch).  Numerics,
// tiles, the epilogue and the fused norm are dec8's.
template <int EPI, int KU, int KS, int AR>
__global__ __launch_bounds__(KS * 64) void dec8r_kernel(Dec8Params p) {
#pragma clang fp contract(off)
    constexpr int NB = EPI == QIE_EPI_SWIGLU ? 2 : 1;
    constexpr int kNT = 2;
    __shared__ __attribute__((aligned(16))) float red[2][KS][NB][256];
    __shared__ float ssq[KS][16];
    __shared__ __attribute__((aligned(16))) d8_u32x4 nw_s[KS][KU * 8];
    __shared__ __attribute__((aligned(16))) d8_u32x4 a_s[KS][KU][2][AR * 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const int M = p.M, K = p.K, T = p.n_tiles;
    if ((int)blockIdx.x >= T) return;
    const int my = (T - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    const int arow = fr < M ? fr : M - 1;
    const int kw = wave * (KU * 64);
    const int aidx = (fr & (AR - 1)) * 4 + g;   // this lane's A slot (rows >= M: any real row)

    d8_u32x4 av[KU][2];
    {
        const d8_u32x4* xp = reinterpret_cast<const d8_u32x4*>(p.x + (int64_t)arow * p.ldx + kw + 16 * g);
#pragma unroll
        for (int u = 0; u < KU; u++) {
            av[u][0] = xp[8 * u];
            av[u][1] = xp[8 * u + 1];
        }
    }
    const bool nrm = p.norm_w != nullptr && !QIE_DBG(p.dbg & 2);
    const d8_u32x4 nwv = *reinterpret_cast<const d8_u32x4*>((nrm ? p.norm_w : p.x) + kw + 8 * (lane < KU * 8 ? lane : 0));

    constexpr int KH = KU / 2;
    struct Step {
        d8_u32x4 wv[NB][KH];
        float sc[NB];
        float ep[4];
    };
    auto issue = [&](Step& t, int it, int hf) {
        const bool live = it < my;                                   // past the last tile: no traffic
        const int itc = live ? it : my - 1;
        const int tile = (int)blockIdx.x + itc * (int)gridDim.x;
        const int sg = NB == 2 ? 0 : (tile < p.t01[0] ? 0 : (tile < p.t01[1] ? 1 : 2));
        const int tb0 = sg == 0 ? 0 : (sg == 1 ? p.t01[0] : p.t01[1]);
        const int rows = p.seg_rows[sg];
        int r = (tile - tb0) * 16 + fr;
        r = r < rows ? r : rows - 1;
        const int voff = r * K + kw + 16 * g + hf * (KH * 64);
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const uint8_t* base = p.w[NB == 2 ? b : sg];
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0,
                                                              live ? (int)((int64_t)rows * (K + 4)) : 0, 0x00020000);
#pragma unroll
            for (int u = 0; u < KH; u++) t.wv[b][u] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, u * 64, kNT);
            if (hf) t.sc[b] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, rows * K + r * 4, 0, 0));
        }
        if (!hf) return;
        const int n = tile * 16 + fr;
        const int nc = n < p.N ? n : p.N - 1;
        if constexpr (EPI == QIE_EPI_RESIDUAL) {
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int i = 4 * g + rr < M ? 4 * g + rr : M - 1;
                t.ep[rr] = bf2f(p.y[(int64_t)i * p.ldy + nc]);
            }
        } else if constexpr (EPI == QIE_EPI_STORE) {
            const uint16_t* bp = p.bias[sg];
            const float v = bf2f((bp ? bp : p.x)[bp ? r : 0]);
            t.ep[0] = bp ? v : 0.f;
        }
    };

    Step s0, s1, s2, s3;
    issue(s0, 0, 0);
    issue(s1, 0, 1);
    __builtin_amdgcn_sched_barrier(0);

    if (nrm) {
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < KU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t e4[4] = {av[u][h].x, av[u][h].y, av[u][h].z, av[u][h].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float l = bf_lo(e4[j]), hh = bf_hi(e4[j]);
                    ss += l * l + hh * hh;
                }
            }
        ss = xor32_sum(xor16_sum(ss));
        // opaque: the apply below re-unpacks the fragments instead of keeping the 128 unpacked
        // floats of the sum of squares alive across the exchange (they spilled)
#pragma unroll
        for (int u = 0; u < KU; u++) asm volatile("" : "+v"(av[u][0]), "+v"(av[u][1]));
        if (g == 0) ssq[wave][fr] = ss;
        if (lane < KU * 8) nw_s[wave][lane] = nwv;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < KS; w++) tot += ssq[w][fr];
        const float rms = sqrtf((tot / (float)K) + p.eps);
        const float inv = 1.0f / rms;
        const float rr = rms < INFINITY ? rms : 0.f;
        auto apply = [&](auto hf) {
            constexpr bool HF = decltype(hf)::value;
#pragma unroll
            for (int u = 0; u < KU; u++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const d8_u32x4 nv = nw_s[wave][8 * u + 2 * g + h];
                    av[u][h].x = d8_rms_pair<HF>(av[u][h].x, nv.x, rr, inv);
                    av[u][h].y = d8_rms_pair<HF>(av[u][h].y, nv.y, rr, inv);
                    av[u][h].z = d8_rms_pair<HF>(av[u][h].z, nv.z, rr, inv);
                    av[u][h].w = d8_rms_pair<HF>(av[u][h].w, nv.w, rr, inv);
                    __builtin_amdgcn_sched_barrier(0);
                }
        };
        __builtin_amdgcn_sched_barrier(0);
        if (p.numerics == QIE_NUMERICS_HF) apply(std::true_type{});
        else apply(std::false_type{});
        __builtin_amdgcn_sched_barrier(0);
    }
    // the fragments to LDS: each lane's own slot (row slots >= AR are never stored: rows >= M)
    if (fr < AR) {
#pragma unroll
        for (int u = 0; u < KU; u++) {
            a_s[wave][u][0][aidx] = av[u][0];
            a_s[wave][u][1][aidx] = av[u][1];
        }
    }
    // a wave reads back only its own slots: its LDS ops retire in order, no barrier
    __builtin_amdgcn_sched_barrier(0);
    issue(s2, 1, 0);   // after the prologue: its registers were the fragments'
    __builtin_amdgcn_sched_barrier(0);

    unsigned long long kbest[4] = {0ull, 0ull, 0ull, 0ull};
    d8_f32x4 acc[NB];
    auto mma = [&](const Step& t, int hf) {
        if (hf == 0) {
#pragma unroll
            for (int b = 0; b < NB; b++) acc[b] = d8_f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < KH; u++) {
            const int ua = hf * KH + u;
            const d8_bf16x8 a0 = __builtin_bit_cast(d8_bf16x8, a_s[wave][ua][0][aidx]);
            const d8_bf16x8 a1 = __builtin_bit_cast(d8_bf16x8, a_s[wave][ua][1][aidx]);
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const uint2 c0 = fp8x4_to_bf16x4(t.wv[b][u].x), c1 = fp8x4_to_bf16x4(t.wv[b][u].y);
                const uint2 c2 = fp8x4_to_bf16x4(t.wv[b][u].z), c3 = fp8x4_to_bf16x4(t.wv[b][u].w);
                const d8_u32x4 lo = d8_u32x4{c0.x, c0.y, c1.x, c1.y};
                const d8_u32x4 hi = d8_u32x4{c2.x, c2.y, c3.x, c3.y};
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, __builtin_bit_cast(d8_bf16x8, lo), acc[b], 0, 0, 0);
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, __builtin_bit_cast(d8_bf16x8, hi), acc[b], 0, 0, 0);
            }
            // one unit at a time: hoisting every unit's reads and conversions would spill
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto finish = [&](const Step& t, int it) {
        const int buf = it & 1;
#pragma unroll
        for (int b = 0; b < NB; b++)
            *reinterpret_cast<float4*>(&red[buf][wave][b][lane * 4]) = make_float4(acc[b][0], acc[b][1], acc[b][2], acc[b][3]);
        __syncthreads();
        if (wave != it % KS) return;
        const int tile = (int)blockIdx.x + it * (int)gridDim.x;
        const int n = tile * 16 + fr;
        float c[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            float4 s = *reinterpret_cast<const float4*>(&red[buf][0][b][lane * 4]);
#pragma unroll
            for (int w = 1; w < KS; w++) {
                const float4 v = *reinterpret_cast<const float4*>(&red[buf][w][b][lane * 4]);
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
            c[b][0] = s.x * t.sc[b];
            c[b][1] = s.y * t.sc[b];
            c[b][2] = s.z * t.sc[b];
            c[b][3] = s.w * t.sc[b];
        }
        if (n >= p.N) return;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int i = 4 * g + r;
            if (i >= M) continue;
            uint16_t* yr = p.y + (int64_t)i * p.ldy;
            if constexpr (EPI == QIE_EPI_SWIGLU) {
                const float gg = rbf(c[0][r]);
                const float uu = rbf(c[1][r]);
                const float a = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                yr[n] = f2bf(uu * a);
            } else if constexpr (EPI == QIE_EPI_RESIDUAL) {
                yr[n] = f2bf(t.ep[r] + rbf(c[0][r]));
            } else if constexpr (EPI == QIE_EPI_F32) {
                reinterpret_cast<float*>(p.y)[(int64_t)i * p.ldy + n] = c[0][r];
            } else {
                const uint16_t o = f2bf(c[0][r] + t.ep[0]);
                yr[n] = o;
                if (p.keys) {
                    const unsigned long long kk = sel_key(bf2f(o), (uint32_t)(n + p.key_col0));
                    kbest[r] = kk > kbest[r] ? kk : kbest[r];
                }
            }
        }
    };

    // ring of four half-tile steps: step 2 it + hf of tile it sits in s[(2 it + hf) & 3];
    // every step issues the one three steps ahead before computing
    __builtin_amdgcn_sched_barrier(0);
    for (int it = 0; it < my; it += 2) {
        issue(s3, it + 1, 1);
        mma(s0, 0);
        issue(s0, it + 2, 0);
        mma(s1, 1);
        finish(s1, it);
        if (it + 1 >= my) break;   // block-uniform
        issue(s1, it + 2, 1);
        mma(s2, 0);
        issue(s2, it + 3, 0);
        mma(s3, 1);
        finish(s3, it + 1);
    }
    if constexpr (EPI == QIE_EPI_STORE) {
        if (p.keys) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                unsigned long long v = kbest[r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const unsigned long long s = __shfl_xor(v, o, 64);
                    v = s > v ? s : v;
                }
                if (fr == 0 && 4 * g + r < M && v) atomicMax(p.keys + 4 * g + r, v);
            }
        }
    }
}

template <int EPI, int KU, int KS, int AR>
static int dec8r_launch(const Dec8Params& p, hipStream_t st) {
    const void* fn = (const void*)dec8r_kernel<EPI, KU, KS, AR>;
    static int per_cu = 0;
    if (per_cu == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, KS * 64, 0) != hipSuccess || nb < 1) nb = 1;
        per_cu = nb;
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(p.n_tiles, (int64_t)device_cu_count() * per_cu));
    hipLaunchKernelGGL((dec8r_kernel<EPI, KU, KS, AR>), dim3(grid), dim3(KS * 64), 0, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

template <int EPI, int KU, int KS, bool SPL = false, bool T16 = false, bool LF = false>
static int dec8_launch(const Dec8Params& p, hipStream_t st) {
    const void* fn = (const void*)dec8_kernel<EPI, KU, KS, SPL, T16, LF>;
    static int per_cu = 0;   // resident blocks per CU (one per instantiation, cached)
    if (per_cu == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, KS * 64, 0) != hipSuccess || nb < 1) nb = 1;
        per_cu = nb;
    }
    const int64_t slots = (int64_t)device_cu_count() * per_cu;
    int grid;
    if constexpr (SPL) {   // parts x G blocks, G tiles in flight per part (one round if they fit)
        // and at most RDF tiles per block (the kernel keeps every tile's partials in LDS;
        // RDF as in dec8_kernel, full 16-row slots)
        constexpr int RDF = (57344 / (KS * 1024)) < 2 ? 2 : (57344 / (KS * 1024));
        const int64_t g = std::max<int64_t>((p.n_tiles + RDF - 1) / RDF, std::min<int64_t>(p.n_tiles, slots / p.parts));
        grid = (int)(g * p.parts);
    } else {
        // dev A/B QIE_DEC8_GRID_MUL: generations of resident blocks (1: all tiles in one; config 4
        // measured 2 / 3 / 4: gate/up 25.3 -> 28.0 / 32.4 / 34.8 µs — unlike the bf16 GEMV's grid)
        const int gm = std::max(1, dev_env("QIE_DEC8_GRID_MUL", 1));
        grid = (int)std::max<int64_t>(1, std::min<int64_t>(p.n_tiles, slots * gm));
    }
    hipLaunchKernelGGL((dec8_kernel<EPI, KU, KS, SPL, T16, LF>), dim3(grid), dim3(KS * 64), 0, st, p);
    QIE_LAUNCH_CHECK();
    return 0;
}

// Split-K workspace (slabs + tickets), one per stream — streams of one device may run
// projections at the same time (tensor-parallel ranks on one GPU in the tests) — reserved by
// qie_batch_create (dec8_reserve) so that the captured decode step finds it; tickets are
// zero at rest (the last arriver resets its tile's).
namespace {
constexpr int kDec8MaxTiles = 2048, kDec8MaxParts = 16;   // N <= 32,768 (dec8_applies)
struct Dec8Ws {
    float* slab = nullptr;
    unsigned* cnt = nullptr;
};
std::mutex g_d8_mu;
std::map<hipStream_t, Dec8Ws> g_d8_ws;
}  // namespace

int dec8_reserve(hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_d8_mu);
    Dec8Ws& w = g_d8_ws[st];
    if (w.slab) return 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 1;
    QIE_HIP(hipMalloc((void**)&w.slab, (size_t)kDec8MaxTiles * kDec8MaxParts * 1024));
    QIE_HIP(hipMalloc((void**)&w.cnt, (size_t)kDec8MaxTiles * 4));
    QIE_HIP(hipMemsetAsync(w.cnt, 0, (size_t)kDec8MaxTiles * 4, st));
    QIE_HIP(hipStreamSynchronize(st));
    return 0;
}

static bool dec8_workspace(hipStream_t st, Dec8Params* p) {
    if (dec8_reserve(st) != 0) return false;
    std::lock_guard<std::mutex> lk(g_d8_mu);
    const Dec8Ws& w = g_d8_ws[st];
    p->slab = w.slab;
    p->cnt = w.cnt;
    return true;
}

template <int KU, int KS, bool T16>
static int dec8_epi_split(const Dec8Params& p, int epi, hipStream_t st) {
    switch (epi) {
        case QIE_EPI_RESIDUAL: return dec8_launch<QIE_EPI_RESIDUAL, KU, KS, true, T16>(p, st);
        case QIE_EPI_F32: return dec8_launch<QIE_EPI_F32, KU, KS, true, T16>(p, st);
        default: return dec8_launch<QIE_EPI_STORE, KU, KS, true, T16>(p, st);
    }
}

template <int KU, int KS, bool T16>
static int dec8_epi(const Dec8Params& p, int epi, hipStream_t st) {
    if constexpr (KU == 8 && KS == 7 && !T16) {   // the ring form (config 4's K = 3,584), M <= 8 (dev A/B QIE_DEC8R)
        if (p.M <= 8 && dev_env("QIE_DEC8R", 0) != 0) {
            switch (epi) {
                case QIE_EPI_SWIGLU: return dec8r_launch<QIE_EPI_SWIGLU, KU, KS, 8>(p, st);
                case QIE_EPI_RESIDUAL: return dec8r_launch<QIE_EPI_RESIDUAL, KU, KS, 8>(p, st);
                case QIE_EPI_F32: return dec8r_launch<QIE_EPI_F32, KU, KS, 8>(p, st);
                default: return dec8r_launch<QIE_EPI_STORE, KU, KS, 8>(p, st);
            }
        }
    }
    // fused norm at M <= 8 on the 7 x 8-unit shape (K = 3,584: config 4's QKV and gate/up):
    // the LDS form (dev A/B: QIE_DEC8_DBG & 32 keeps the register form)
    if constexpr (KU == 8 && KS == 7) {
        if (p.norm_w && p.M <= 8 && !QIE_DBG(p.dbg & 2) && !QIE_DBG(p.dbg & 32)) {
            if (epi == QIE_EPI_SWIGLU) return dec8_launch<QIE_EPI_SWIGLU, KU, KS, false, T16, true>(p, st);
            if (epi == QIE_EPI_STORE) return dec8_launch<QIE_EPI_STORE, KU, KS, false, T16, true>(p, st);
        }
    }
    switch (epi) {
        case QIE_EPI_SWIGLU: return dec8_launch<QIE_EPI_SWIGLU, KU, KS, false, T16>(p, st);
        case QIE_EPI_RESIDUAL: return dec8_launch<QIE_EPI_RESIDUAL, KU, KS, false, T16>(p, st);
        case QIE_EPI_F32: return dec8_launch<QIE_EPI_F32, KU, KS, false, T16>(p, st);
        default: return dec8_launch<QIE_EPI_STORE, KU, KS, false, T16>(p, st);
    }
}

// K slice shapes: (units per wave KU, waves KS) with KU * KS * 64 = K.  7 waves x 8 units at
// K = 3,584 (14 x 4 measured the same for QKV and 0.45 µs slower for O at config 4).
// Long K without such a shape (the down projection's 18,944 = 296 units): split-K over
// parts of 8 waves x 4 units (10 parts at 18,944, the last one ragged; 128 VGPRs, two blocks
// per CU), single-segment epilogues without a fused norm only (a norm needs the whole row in
// one block).  Config 4 (fp8, B = 8), same box: the general skinny kernel 2,895 tok/s (down
// 24.9 µs live), split 8 x 8 units 2,990 (23.4), 8 x 4 units 3,010 (23.0); the first form,
// which published each tile's parts as it finished it, stalled every wave on its ticket
// round trip behind the per-tile barrier: 2,760 (31.5).
static bool dec8_shape(int64_t K, int* ku, int* ks) {
    if (K % 64 != 0) return false;
    const int64_t units = K / 64;
    static const int shapes[][2] = {{8, 7}, {8, 8}, {2, 7}, {4, 8}, {8, 4}};
    for (const auto& s : shapes)
        if ((int64_t)s[0] * s[1] == units) {
            *ku = s[0];
            *ks = s[1];
            return true;
        }
    return false;
}
static int dec8_split_parts(const qie_linear_args* a, int* ku) {
    if (a->K % 64 != 0 || a->norm_w || a->epilogue == QIE_EPI_SWIGLU || a->seg_rows[1] > 0) return 0;
    if (a->N > (int64_t)kDec8MaxTiles * 16) return 0;   // the ticket array
    // (tiled weights can be read by this kernel only: the dev switch does not apply to them)
    if (!(a->flags & QIE_LINEAR_FP8_T16) && dev_env("QIE_DEC8_SPLIT", 1) == 0) return 0;
    const int64_t units = a->K / 64;
    *ku = dev_env("QIE_DEC8_SPLIT_KU", 4) == 8 ? 8 : 4;
    const int64_t parts = (units + 8 * *ku - 1) / (8 * *ku);
    return parts >= 2 && parts <= kDec8MaxParts ? (int)parts : 0;
}

// true when dec8_linear takes this projection (the engine then skips its separate norm)
bool dec8_applies(const qie_linear_args* a) {
    // tiled weights (QIE_LINEAR_FP8_T16) are read by this kernel only, at any 1 <= M <= 16
    const bool t16 = (a->flags & QIE_LINEAR_FP8_T16) != 0;
    if (!(a->flags & QIE_LINEAR_FP8) || a->M < (t16 ? 1 : 2) || a->M > 16) return false;
    if (t16 && dev_env("QIE_T16_SKINNY", 0) != 0) return false;   // dev A/B: tiled projections on the skinny kernel
    if (!t16 && dev_env("QIE_DEC8", 1) == 0) return false;
    int ku, ks;
    if (!dec8_shape(a->K, &ku, &ks) && dec8_split_parts(a, &ku) == 0) return false;
    // vocabulary-sized projections (tens of tiles per block) keep the general skinny kernel:
    // its 16 waves per CU keep more bytes in flight than one 7-wave block (lm_head 119 vs 194 µs)
    // (tiled vocabulary projections go to the skinny kernel, which reads the layout too)
    if (a->N <= 0 || a->N > 32768 || a->ldx % 8 != 0 || a->K >= (1 << 20)) return false;
    if (a->epilogue != QIE_EPI_SWIGLU) {
        // column tiles must not straddle segments
        if (a->seg_rows[0] % 16 != 0 || (a->seg_rows[1] > 0 && (a->seg_rows[0] + a->seg_rows[1]) % 16 != 0))
            return false;
    }
    // tiled weights: whole 16-row tiles per segment
    if (t16) {
        if (a->epilogue == QIE_EPI_SWIGLU ? a->N % 16 != 0
                                          : (a->seg_rows[0] % 16 != 0 || a->seg_rows[1] % 16 != 0 || a->seg_rows[2] % 16 != 0))
            return false;
    }
    // every segment's codes + scales must fit a 32-bit buffer range
    for (int s = 0; s < 3; s++)
        if ((int64_t)(a->epilogue == QIE_EPI_SWIGLU ? a->N : a->seg_rows[s]) * (a->K + 4) >= (int64_t)1 << 31)
            return false;
    return true;
}

// *done = false: not taken (a split-K projection whose workspace cannot be made during a
// graph capture); the caller runs its general kernel
int dec8_linear(const qie_linear_args* a, hipStream_t st, bool* done) {
    *done = true;
    QIE_REQUIRE(dec8_applies(a), "qie_linear: internal: fp8 batched-decode path does not apply");
    const bool t16 = (a->flags & QIE_LINEAR_FP8_T16) != 0;
    Dec8Params p;
    p.x = (const uint16_t*)a->x;
    p.ldx = a->ldx;
    p.norm_w = (const uint16_t*)a->norm_w;
    p.eps = a->norm_eps;
    p.numerics = a->numerics;
    p.K = (int32_t)a->K;
    p.N = (int32_t)a->N;
    p.M = (int32_t)a->M;
    p.y = (uint16_t*)a->y;
    p.ldy = a->ldy;
    p.keys = (unsigned long long*)a->argmax_keys;
    p.key_col0 = a->key_col0;
    p.dbg = dev_env("QIE_DEC8_DBG", 0);
    p.parts = 1;
    p.slab = nullptr;
    p.cnt = nullptr;
    p.n_tiles = (int32_t)((a->N + 15) / 16);
    for (int s = 0; s < 3; s++) {
        p.w[s] = (const uint8_t*)a->w[s];
        p.bias[s] = (const uint16_t*)a->bias[s];
    }
    if (a->epilogue == QIE_EPI_SWIGLU) {
        p.seg_rows[0] = p.seg_rows[1] = p.seg_rows[2] = (int32_t)a->N;
        p.t01[0] = p.t01[1] = p.n_tiles;
    } else {
        const int64_t r0 = a->seg_rows[0] > 0 ? a->seg_rows[0] : a->N;
        const int64_t r1 = a->seg_rows[1];
        p.seg_rows[0] = (int32_t)r0;
        p.seg_rows[1] = (int32_t)(r1 > 0 ? r1 : 1);
        p.seg_rows[2] = (int32_t)std::max<int64_t>(1, a->N - r0 - r1);
        p.t01[0] = (int32_t)(r0 / 16);
        p.t01[1] = (int32_t)((r0 + r1) / 16);
        QIE_REQUIRE(r0 + r1 <= a->N && (r1 == 0 || a->w[1]) && (r0 + r1 == a->N || a->w[2]) && a->w[0],
                    "qie_linear: segment rows do not match the weights");
    }
    int ku = 0, ks = 0;
    if (!dec8_shape(a->K, &ku, &ks)) {
        p.parts = dec8_split_parts(a, &ku);
        if (!dec8_workspace(st, &p)) {
            *done = false;
            return 0;
        }
        if (t16) return ku == 4 ? dec8_epi_split<4, 8, true>(p, a->epilogue, st) : dec8_epi_split<8, 8, true>(p, a->epilogue, st);
        return ku == 4 ? dec8_epi_split<4, 8, false>(p, a->epilogue, st) : dec8_epi_split<8, 8, false>(p, a->epilogue, st);
    }
    if (t16) {
        if (ku == 8 && ks == 7) return dec8_epi<8, 7, true>(p, a->epilogue, st);
        if (ku == 8 && ks == 8) return dec8_epi<8, 8, true>(p, a->epilogue, st);
        if (ku == 2 && ks == 7) return dec8_epi<2, 7, true>(p, a->epilogue, st);
        if (ku == 4 && ks == 8) return dec8_epi<4, 8, true>(p, a->epilogue, st);
        return dec8_epi<8, 4, true>(p, a->epilogue, st);
    }
    if (ku == 8 && ks == 7) return dec8_epi<8, 7, false>(p, a->epilogue, st);
    if (ku == 8 && ks == 8) return dec8_epi<8, 8, false>(p, a->epilogue, st);
    if (ku == 2 && ks == 7) return dec8_epi<2, 7, false>(p, a->epilogue, st);
    if (ku == 4 && ks == 8) return dec8_epi<4, 8, false>(p, a->epilogue, st);
    return dec8_epi<8, 4, false>(p, a->epilogue, st);
}

}  // namespace qie
