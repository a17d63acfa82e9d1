// k_attention.hip — GQA attention over the qie KV cache (gfx950).
//
// Replaces selfattention (layers/src/self_attension.cu:10-149) + launch_attn
// (helpers.cuh:121-130).  The reference runs one block per q head, walks a
// managed-memory linked list of 4-token pages for EVERY key, reduces each dot
// product through a 128-thread smem tree and does the softmax serially on
// thread 0.  Here:
//   * cache layout [seq][L][nkv][max_ctx][hd]: one (layer, kv head) is a
//     contiguous stream, read with 16-byte loads (hd/8 lanes per key);
//   * one workgroup per (kv head, sequence split, query row) serves all
//     nq/nkv query heads of the group, so K/V bytes are read once per group;
//   * online softmax (running max / sum) per split, then a combine
//     ("flash-decoding"), instead of materialising the score row in smem;
//   * row m attends to [0, pos[m]]: decode (pos = new token) and causal prefill
//     (pos = row position) are the same kernel — identical to the reference's
//     mkv = seq_len (decode) and causal mask with -1e9 (prefill).
// Scores: s = dot(q, k) / sqrtf(hd) in fp32; p = expf(s - max); out bf16.
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"
#include "attn_decode.hpp"


#include <cstdlib>
#include <type_traits>

namespace qie {

struct AttnParams {
    const uint16_t* q;
    const int32_t* pos;
    int rows_per_seq;
    const uint16_t* kc;
    const uint16_t* vc;
    KvMap km;
    int layer, nkv, nq, max_ctx;
    int nsplit;
    float* part_o;    // [M][nq][nsplit][HD]
    float* part_ml;   // [M][nq][nsplit][2]
    uint16_t* out;    // [M][nq*HD]
};

template <int HD, bool PG>
__global__ __launch_bounds__(256) void attn_split_kernel(AttnParams a) {
    constexpr int LPT = HD / 8;   // lanes per key row
    constexpr int TPW = 64 / LPT; // keys per wave step
    __shared__ float sm_o[4][kMaxGroup][HD];
    __shared__ float sm_m[4][kMaxGroup], sm_l[4][kMaxGroup];

    const int64_t m = blockIdx.y;
    const int g = blockIdx.x / a.nsplit, s = blockIdx.x % a.nsplit;
    const int G = a.nq / a.nkv;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane / LPT, dl = lane % LPT;
    const int ctx = a.pos[m] + 1;
    int chunk = (ctx + a.nsplit - 1) / a.nsplit;
    chunk = (chunk + 4 * TPW - 1) / (4 * TPW) * (4 * TPW);
    const int t0 = s * chunk;
    const int t1 = min(ctx, t0 + chunk);
    const int64_t seq = m / a.rows_per_seq;

    float qf[kMaxGroup][8];
    const uint16_t* qrow = a.q + m * (int64_t)a.nq * HD + (int64_t)g * G * HD + dl * 8;
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++) {
        if (gi < G) {
            uint4 v = *reinterpret_cast<const uint4*>(qrow + gi * HD);
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                qf[gi][2 * j] = bf_lo(w[j]);
                qf[gi][2 * j + 1] = bf_hi(w[j]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) qf[gi][j] = 0.f;
        }
    }
    float mr[kMaxGroup], lr[kMaxGroup], o[kMaxGroup][8];
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++) {
        mr[gi] = -INFINITY;
        lr[gi] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) o[gi][j] = 0.f;
    }
    const float scale = sqrtf((float)HD);
    const int64_t head_off = kv_run_off(a.km, (int64_t)a.layer * a.nkv + g, HD);
    const uint16_t* kb = a.kc + head_off + dl * 8;
    const uint16_t* vb = a.vc + head_off + dl * 8;

    for (int t = t0 + wave * TPW + sub; t < t1; t += 4 * TPW) {
        const int64_t to = kv_tok<PG>(a.km, seq, t, HD);
        uint4 kv = *reinterpret_cast<const uint4*>(kb + to);
        uint4 vv = *reinterpret_cast<const uint4*>(vb + to);
        float kf[8], vf[8];
        uint32_t kw[4] = {kv.x, kv.y, kv.z, kv.w}, vw[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            kf[2 * j] = bf_lo(kw[j]);
            kf[2 * j + 1] = bf_hi(kw[j]);
            vf[2 * j] = bf_lo(vw[j]);
            vf[2 * j + 1] = bf_hi(vw[j]);
        }
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) continue;
            float d = 0.f;
#pragma unroll
            for (int j = 0; j < 8; j++) d = fmaf(qf[gi][j], kf[j], d);
#pragma unroll
            for (int off = LPT / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            const float sc = d / scale;
            const float mn = fmaxf(mr[gi], sc);
            const float c1 = expf(mr[gi] - mn);
            const float e = expf(sc - mn);
            lr[gi] = lr[gi] * c1 + e;
#pragma unroll
            for (int j = 0; j < 8; j++) o[gi][j] = o[gi][j] * c1 + e * vf[j];
            mr[gi] = mn;
        }
    }

    // merge the TPW key slots of this wave (lanes with equal dl)
#pragma unroll
    for (int off = LPT; off < 64; off <<= 1) {
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) continue;
            const float m2 = __shfl_xor(mr[gi], off, 64);
            const float l2 = __shfl_xor(lr[gi], off, 64);
            float o2[8];
#pragma unroll
            for (int j = 0; j < 8; j++) o2[j] = __shfl_xor(o[gi][j], off, 64);
            const float mn = fmaxf(mr[gi], m2);
            if (mn == -INFINITY) continue;
            const float c1 = expf(mr[gi] - mn), c2 = expf(m2 - mn);
            lr[gi] = lr[gi] * c1 + l2 * c2;
#pragma unroll
            for (int j = 0; j < 8; j++) o[gi][j] = o[gi][j] * c1 + o2[j] * c2;
            mr[gi] = mn;
        }
    }
    if (sub == 0) {
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) continue;
#pragma unroll
            for (int j = 0; j < 8; j++) sm_o[wave][gi][dl * 8 + j] = o[gi][j];
            if (dl == 0) {
                sm_m[wave][gi] = mr[gi];
                sm_l[wave][gi] = lr[gi];
            }
        }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
        const int gi = idx / HD, d = idx % HD;
        float mn = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; w++) mn = fmaxf(mn, sm_m[w][gi]);
        float l = 0.f, ov = 0.f;
        if (mn != -INFINITY) {
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const float c = expf(sm_m[w][gi] - mn);
                l += sm_l[w][gi] * c;
                ov += sm_o[w][gi][d] * c;
            }
        }
        const int h = g * G + gi;
        if (a.nsplit == 1) {
            a.out[m * (int64_t)a.nq * HD + (int64_t)h * HD + d] = f2bf(ov / l);
        } else {
            const int64_t pi = (m * a.nq + h) * (int64_t)a.nsplit + s;
            a.part_o[pi * HD + d] = ov;
            if (d == 0) {
                a.part_ml[pi * 2] = mn;
                a.part_ml[pi * 2 + 1] = l;
            }
        }
    }
}

template <int HD>
__global__ __launch_bounds__(HD) void attn_combine_kernel(AttnParams a) {
    const int64_t m = blockIdx.y;
    const int h = blockIdx.x, d = threadIdx.x;
    const int64_t base = (m * a.nq + h) * (int64_t)a.nsplit;
    float mn = -INFINITY;
    for (int s = 0; s < a.nsplit; s++) mn = fmaxf(mn, a.part_ml[(base + s) * 2]);
    float l = 0.f, ov = 0.f;
    for (int s = 0; s < a.nsplit; s++) {
        const float ms = a.part_ml[(base + s) * 2];
        if (ms == -INFINITY) continue;
        const float c = expf(ms - mn);
        l += a.part_ml[(base + s) * 2 + 1] * c;
        ov += a.part_o[(base + s) * HD + d] * c;
    }
    a.out[m * (int64_t)a.nq * HD + (int64_t)h * HD + d] = f2bf(ov / l);
}


// ---------------------------------------------------------------------------
// Prefill: causal flash attention on MFMA (v_mfma_f32_16x16x32_bf16).
// K/V tiles of 64 keys staged in LDS (double-buffered, register prefetch).
//   S^T = K . Q^T  — A = K tile (row = key, k = d) from an XOR-swizzled LDS image,
//                    B = Q^T from registers (lane: q = lane & 15, 8 contiguous d);
//                    so each lane holds 4 keys x 4 key-tiles of ONE query row and
//                    the softmax row statistics need only lanes l, l^16, l^32, l^48.
//   O  += P . V    — A = P straight from the S^T accumulators (bf16), k permuted as
//                    key(j) = 32c + 4g + j (j < 4), 32c + 16 + 4g + (j - 4);
//                    B = V with the SAME key permutation, read by two
//                    ds_read_b64_tr_b16 per fragment from a row-major V image.
// Scores: dot / sqrtf(hd) (fp32), masked keys (> query position) get -inf (the
// reference's -1e9, self_attension.cu:88-92, underflows to the same 0).
struct PrefillAttnParams {
    const uint16_t* q;       // [M][nq*HD]
    const int32_t* pos;      // [M]; non-decreasing within each sequence's rows
    int rows_per_seq;
    const uint16_t* kc;
    const uint16_t* vc;
    KvMap km;
    int layer, nkv, nq, max_ctx;
    int64_t M;
    uint16_t* out;
    int full_tiles;          // 1: tiles wholly at or below a group's first position skip the causal mask (dev A/B 0)
};


// ---------------------------------------------------------------------------
// Prefill kernel: each wave owns two 16-row query groups, so every K fragment
// (S^T = K.Q^T) and every V fragment (O += P.V) read from LDS feeds up to two MFMAs.
// Causal balance: the sequence's 16-row groups are paired (j, n-1-j) and wave j of the
// grid gets pair j, so every wave (and every workgroup of 4 waves) has the same number of
// (group, key tile) products; a workgroup stages K/V tiles up to its latest row and each
// group skips the tiles past its own last position (the contiguous 128-row q tiles this
// replaces left the workgroup with the last tile 16x the work of the first: 2x the
// makespan of the balanced split on 256 CUs).  Scores go to the log2 domain once
// (dot * log2(e) / sqrt(hd)) and are exponentiated with v_exp_f32: the reference build
// compiles with -use_fast_math, i.e. __expf / __fdividef.
template <int HD, bool PG, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_prefill_mfma2_kernel(PrefillAttnParams a) {
    constexpr int KT = 64;
    constexpr int CPR = HD / 8;
    constexpr int KSTEPS = HD / 32;
    constexpr int DT = HD / 16;
    constexpr int QG = 2;                  // 16-row query groups per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);
    uint16_t* Vs = reinterpret_cast<uint16_t*>(smem + 2 * KT * HD * 2);
    // V image chunk swizzle: the 16-B chunk c of key row r sits at c ^ vswz(r).  A
    // ds_read_b64_tr_b16 half-wave reads 8 rows x 32 B at one column; unswizzled, the rows
    // (a whole number of 256-B bank rows apart) hit the same banks: 8-way conflicts.
    auto vswz = [](int r) { return 2 * (r & (CPR / 2 - 1)); };

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const int h = blockIdx.y, seq = blockIdx.z;
    const int R = a.rows_per_seq;
    const int ngr = (R + 15) / 16, npair = (ngr + 1) / 2;
    const int64_t row0 = (int64_t)seq * R;
    const int G = a.nq / a.nkv, kvh = h / G;
    const int64_t head_off = kv_run_off(a.km, (int64_t)a.layer * a.nkv + kvh, HD);
    const uint16_t* kb = a.kc + head_off;
    const uint16_t* vb = a.vc + head_off;
    // this wave's groups: pair j = (j, ngr-1-j); the workgroup's latest row is wave 0's
    // second group (positions are non-decreasing within a sequence)
    const int j = blockIdx.x * NW + wave;
    const int grp[QG] = {j, ngr - 1 - j};
    bool gact[QG];
    gact[0] = j < npair;
    gact[1] = j < npair && grp[1] != j;
    const int kmax = a.pos[row0 + min(16 * (ngr - 1 - (int)blockIdx.x * NW) + 15, R - 1)];
    const int nkt = kmax / KT + 1;

    int qpos[QG], gpos[QG], gmin[QG];
    bf16x8_t qf[QG][KSTEPS];
#pragma unroll
    for (int q = 0; q < QG; q++) {
        const int gq = gact[q] ? grp[q] : 0;
        const int qrow = min(16 * gq + fr, R - 1);
        qpos[q] = a.pos[row0 + qrow];
        gpos[q] = __builtin_amdgcn_readfirstlane(gact[q] ? a.pos[row0 + min(16 * gq + 15, R - 1)] : -1);   // -1: no tile
        // the group's first position (positions are non-decreasing): a key tile ending at or
        // before it is unmasked for every row of the group
        gmin[q] = __builtin_amdgcn_readfirstlane(a.full_tiles ? a.pos[row0 + min(16 * gq, R - 1)] : -1);
        const uint16_t* qp = a.q + (row0 + qrow) * (int64_t)a.nq * HD + (int64_t)h * HD;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ks++) qf[q][ks] = *reinterpret_cast<const bf16x8_t*>(qp + ks * 32 + g * 8);
    }

    // K/V tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4): one wave-instruction
    // = 1 KiB = RPI key rows, lane-linear in LDS, the chunk swizzle applied on the SOURCE
    // address (LDS position p of row r holds chunk p ^ swz(r)); no staging registers and no
    // ds_write pass.  A 64-key tile never straddles a page (page_tokens is a multiple of
    // 128); rows past kmax re-read row kmax (same page) and are masked by position.
    constexpr int RPI = 512 / HD;                 // key rows per 1 KiB wave-instruction
    constexpr int IPW = KT / RPI / NW;            // wave-instructions per wave per operand
    // Buffer loads to LDS on a per-tile resource (round 5): the lane byte offsets inside a
    // tile are constants of the launch and the tile base is scalar, so a tile's DMAs cost no
    // VALU (the flat form recomputed 64-bit addresses and the row clamp per tile: ~40 VALU).
    // The resource covers the tile's rows up to kmax only: rows past it read as zeros (their
    // keys are masked, and P = 0 times a zero V row stays 0 whatever the cache holds there).
    uint32_t koff[IPW], voff[IPW];
#pragma unroll
    for (int i = 0; i < IPW; i++) {
        const int r = (wave * IPW + i) * RPI + lane / CPR, pch = lane % CPR;
        koff[i] = (uint32_t)(r * HD + (pch ^ (r & (CPR - 1))) * 8) * 2;
        voff[i] = (uint32_t)(r * HD + (pch ^ vswz(r)) * 8) * 2;
    }
    auto issue = [&](int kt, int buf) {
        const int64_t tb = kv_tok<PG>(a.km, seq, kt * KT, HD);
        const int rows = min(KT, kmax + 1 - kt * KT);
        const auto rk = __builtin_amdgcn_make_buffer_rsrc((void*)(kb + tb), (short)0, rows * HD * 2, 0x00020000);
        const auto rv = __builtin_amdgcn_make_buffer_rsrc((void*)(vb + tb), (short)0, rows * HD * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < IPW; i++) {
            const int inst = wave * IPW + i;
            buf_lds16(rk, Ks + buf * KT * HD + inst * 512, koff[i]);
            buf_lds16(rv, Vs + buf * KT * HD + inst * 512, voff[i]);
        }
    };

    f32x4_t oacc[QG][DT];
#pragma unroll
    for (int q = 0; q < QG; q++)
#pragma unroll
        for (int d = 0; d < DT; d++) oacc[q][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float m_run[QG], l_run[QG];
#pragma unroll
    for (int q = 0; q < QG; q++) {
        m_run[q] = -INFINITY;
        l_run[q] = 0.f;
    }
    const float sl2 = 1.4426950408889634f / sqrtf((float)HD);   // log2(e) / sqrt(hd)

    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    // which of the wave's two groups take a key tile is a run of tiles per case (positions
    // are non-decreasing, and group 1 is the later one): both groups for tiles [0, nkt0),
    // group 1 alone up to nkt1, then barriers only up to the workgroup's nkt.  One loop per
    // case with the tile body instantiated for it: no MFMA sits behind a per-instruction
    // exec-mask branch (the compiler could not prove on[] uniform and wrapped every MFMA in
    // s_and_saveexec / s_cbranch_execz / s_or_b64), and — unlike a three-way branch inside
    // one loop — the accumulators need no register copies where the cases meet.
    auto tile = [&](const int kt, const uint16_t* K, const uint16_t* Vt, auto q0c, auto q1c) {
            constexpr bool ON[QG] = {decltype(q0c)::value, decltype(q1c)::value};
            f32x4_t sacc[QG][4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
#pragma unroll
                for (int q = 0; q < QG; q++) sacc[q][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
                const int r = t * 16 + fr;
#pragma unroll
                for (int ks = 0; ks < KSTEPS; ks++) {
                    const int ch = ks * 4 + g;
                    const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(K + r * HD + ((ch ^ (r & (CPR - 1))) * 8));
#pragma unroll
                    for (int q = 0; q < QG; q++)
                        if (ON[q]) sacc[q][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[q][ks], sacc[q][t], 0, 0, 0);
                }
            }
            float pv[QG][4][4];   // this tile's probabilities (fp32), split into bf16 parts at P.V
#pragma unroll
            for (int q = 0; q < QG; q++) {
                if (!ON[q]) continue;
                float (&sv)[4][4] = pv[q];
                float mt = -INFINITY;
                // (an fma form, exp2(fma(s, sl2, -m)), saves 16 VALU per tile but rounds
                // differently: config 2's 128-decision parity run then had a flip at a top-2 gap
                // 0.34 against the oracle's own 0.31 spread — not taken)
                if (kt * KT + KT - 1 <= gmin[q]) {   // wave-uniform: no key of the tile is masked
#pragma unroll
                    for (int t = 0; t < 4; t++)
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const float sc = sacc[q][t][r] * sl2;
                            sv[t][r] = sc;
                            mt = fmaxf(mt, sc);
                        }
                } else {
#pragma unroll
                    for (int t = 0; t < 4; t++)
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const int key = kt * KT + t * 16 + g * 4 + r;
                            const float sc = key <= qpos[q] ? sacc[q][t][r] * sl2 : -INFINITY;
                            sv[t][r] = sc;
                            mt = fmaxf(mt, sc);
                        }
                }
                mt = xor32_max(xor16_max(mt));
                const float m_new = fmaxf(m_run[q], mt);   // finite: tile 0 holds key 0 <= every position
                const float alpha = __builtin_amdgcn_exp2f(m_run[q] - m_new);
                float ls = 0.f;
#pragma unroll
                for (int t = 0; t < 4; t++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float e = __builtin_amdgcn_exp2f(sv[t][r] - m_new);
                        sv[t][r] = e;
                        ls += e;
                    }
                ls = xor32_sum(xor16_sum(ls));
                l_run[q] = l_run[q] * alpha + ls;
                m_run[q] = m_new;
                // O *= alpha only where some row's max grew: alpha == 1 exactly otherwise
                // (exp2(0)), and tile 0's O is zero — skipping is bit-identical (a wave-uniform
                // ballot; once the running maxima settle most tiles skip the 32 products)
                if (kt > 0 && __builtin_amdgcn_ballot_w64(alpha != 1.0f) != 0) {
                    float ar[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) ar[r] = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
                    for (int d = 0; d < DT; d++)
#pragma unroll
                        for (int r = 0; r < 4; r++) oacc[q][d][r] *= ar[r];
                }
            }
            // (Measured and dropped: softmax then P.V per group, so that group 1's softmax
            // could issue beside group 0's MFMAs, V fragments read per group: 76.8 vs 75.3 µs.)
            const int q4 = fr >> 2, p4 = fr & 3;
#pragma unroll
            for (int c = 0; c < 2; c++) {
                // P = hi + lo: two bf16 parts carry 16 of the 24 mantissa bits of each fp32
                // probability; the dropped remainder is < 2^-16 of p, a relative error per
                // P.V product (<= 2^-17) below the fp32 summation-order spread of the
                // reference's own sum over keys
                bf16x8_t ph[QG], pl[QG];
#pragma unroll
                for (int q = 0; q < QG; q++) {
                    if (!ON[q]) continue;
                    float e8[8];
#pragma unroll
                    for (int jj = 0; jj < 8; jj++) e8[jj] = pv[q][2 * c + (jj >> 2)][jj & 3];
                    uint4 pp[2];
                    split_bf16x8<2>(e8, pp);
                    ph[q] = __builtin_bit_cast(bf16x8_t, pp[0]);
                    pl[q] = __builtin_bit_cast(bf16x8_t, pp[1]);
                }
#pragma unroll
                for (int d = 0; d < DT; d++) {
                    // rows vr and vr + 16 share vswz: one column offset serves both reads
                    const int vr = 32 * c + 4 * g + q4;
                    const uint16_t* a0 = Vt + vr * HD + (((2 * d + (p4 >> 1)) ^ vswz(vr)) * 8) + (p4 & 1) * 4;
                    const i16x4_t v0 =
                        __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)(a0));
                    const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) i16x4_t*)(a0 + 16 * HD));
                    const bf16x8_t vb8 =
                        __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                    for (int q = 0; q < QG; q++) {
                        if (!ON[q]) continue;
                        oacc[q][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph[q], vb8, oacc[q][d], 0, 0, 0);
                        oacc[q][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl[q], vb8, oacc[q][d], 0, 0, 0);
                    }
                }
            }
        };
    int kt = 0;
    auto run = [&](const int kend, auto q0c, auto q1c) {
        for (; kt < kend; kt++) {
            // into the other buffer: every wave finished tile kt-1 before the last barrier
            if (kt + 1 < nkt) issue(kt + 1, cur ^ 1);
            if constexpr (decltype(q0c)::value || decltype(q1c)::value)
                tile(kt, Ks + cur * KT * HD, Vs + cur * KT * HD, q0c, q1c);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of tile kt+1
            __syncthreads();                                     // ... and every other wave's
            cur ^= 1;
        }
    };
    // tiles each group takes: kt * KT <= gpos (gpos = -1: none); gpos[1] >= gpos[0]
    const int nkt0 = gpos[0] >= 0 ? min(nkt, gpos[0] / KT + 1) : 0;
    const int nkt1 = gpos[1] >= 0 ? min(nkt, gpos[1] / KT + 1) : 0;
    if (nkt1 > 0) {
        run(nkt0, std::true_type{}, std::true_type{});
        run(nkt1, std::false_type{}, std::true_type{});
    } else {
        run(nkt0, std::true_type{}, std::false_type{});
    }
    run(nkt, std::false_type{}, std::false_type{});
#pragma unroll
    for (int q = 0; q < QG; q++) {
        if (!gact[q]) continue;
        float lr[4];
#pragma unroll
        for (int r = 0; r < 4; r++) lr[r] = __shfl(l_run[q], g * 4 + r, 64);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int row = 16 * grp[q] + g * 4 + r;
            if (row >= R) continue;
            uint16_t* orow = a.out + (row0 + row) * (int64_t)a.nq * HD + (int64_t)h * HD;
#pragma unroll
            for (int d = 0; d < DT; d++) orow[16 * d + fr] = f2bf(oacc[q][d][r] / lr[r]);
        }
    }
}


template <int HD, bool PG, int NWA, bool PR, int KS = kDecMStep>
__global__ __launch_bounds__(64 * NWA) void attn_decode_mfma2_kernel(DecodeAttnParams a) {
    attn_decode_mfma2_body<HD, PG, NWA, PR, KS>(a, blockIdx.x, blockIdx.y);
}


// Diagnostics: lane l reads the 8 bytes at element 4*l of an LDS array holding
// value == element index; out[l][e] = what ds_read_b64_tr_b16 delivered.
__global__ void tr16_probe_kernel(int32_t* out) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = (uint16_t)i;
    __syncthreads();
    i16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)(lds + 4 * threadIdx.x));
    for (int e = 0; e < 4; e++) out[threadIdx.x * 4 + e] = (uint16_t)v[e];
}

static int attn_nsplit(int64_t M, int32_t max_ctx) {
    int per = dev_env("QIE_ATTN_SPLIT_TOKENS", 0);
    if (per <= 0) per = M > 8 ? 512 : 64;
    int ns = (max_ctx + per - 1) / per;
    const int cap = M > 8 ? 8 : 64;
    if (ns > cap) ns = cap;
    if (ns < 1) ns = 1;
    return ns;
}

static thread_local const float* g_rope_cur = nullptr;
void set_decode_rope_cur(const float* rc) { g_rope_cur = rc; }

static int fill_dec_params(DecodeAttnParams& a, const void* qkv, int64_t B, const int32_t* pos, const void* q_norm,
                           const void* k_norm, const float* rope_cos, const float* rope_sin, int32_t n_heads,
                           const qie_kv_cache* cache, int32_t layer, float eps, int32_t numerics, void* out, void* ws) {
    a.qkv = (const uint16_t*)qkv;
    a.pos = pos;
    a.q_norm = (const uint16_t*)q_norm;
    a.k_norm = (const uint16_t*)k_norm;
    a.cs = rope_cos;
    a.sn = rope_sin;
    a.kc = (uint16_t*)cache->k;
    a.vc = (uint16_t*)cache->v;
    QIE_TRY(kv_map_make(cache, &a.km, "qie_attention_decode"));
    a.layer = layer;
    a.nkv = cache->n_kv_heads;
    a.nq = n_heads;
    a.max_ctx = cache->max_ctx;
    const int senv = std::min(dev_env("QIE_DEC_SPLITS", 0), kDecMaxSplits);
    // split target: 32 (one-step splits up to 4k keys); at B >= 8, 8 — config 4 (B = 8, ctx
    // 1,025-1,280) then runs two-step splits, half as many split blocks and combine inputs
    // per row: 3,610 -> 3,637-3,645 tok/s same-box (at B = 1 the headline wants the CUs:
    // targets 16 / 8 ran 349 / 340 vs 361 tok/s)
    a.splits_target = senv > 0 ? senv : (B >= 8 ? 8 : kDecMSplits);
    a.dbg = dev_env("QIE_DEC_DBG", 0);
    a.sc1 = dev_env("QIE_DEC_SC1", 1);   // 9.79 -> 9.56 us per launch (ctx 2.3k, Qwen2-7B)
    // keys per block step (the launch picks the kernel instantiation with the same KS): 128.
    // QIE_DEC_KS (dev A/B): 64 (hd 128, not pre-rotated), 256 (hd 64: ONE step where
    // Qwen2-0.5B's config-2 contexts, 129-256 keys, walk two dependent 128-key steps in one
    // block per kv head — measured equal, attention 7.94 vs 7.96 µs live, 1,446 vs 1,454 tok/s:
    // the second step's chain is not what the launch waits on).
    const int hd = cache->head_dim;
    const int ks_env = dev_env("QIE_DEC_KS", 0);
    // (a step never straddles a page: 256-key steps need pages of >= 256 tokens)
    const bool ks256_ok = hd == 64 && (cache->block_table == nullptr || cache->page_tokens >= 256);
    int ks = kDecMStep;
    if (ks_env == 128 || (ks_env == 256 && ks256_ok) || (ks_env == 64 && hd == 128 && !(numerics & QIE_ATTN_PREROPED)))
        ks = ks_env;
    a.ks = ks;
    a.nsplit_max = std::min(a.splits_target, (cache->max_ctx + ks - 1) / ks);
    QIE_REQUIRE(a.nsplit_max <= kDecMaxSplits, "qie_attention_decode: max_ctx %d too long", cache->max_ctx);
    a.eps = eps;
    a.numerics = numerics & QIE_NUMERICS_MASK;
    a.pre_roped = (numerics & QIE_ATTN_PREROPED) != 0;
    QIE_REQUIRE(!a.pre_roped || (q_norm == nullptr && k_norm == nullptr && a.numerics == QIE_NUMERICS_REF),
                "qie_attention_decode: QIE_ATTN_PREROPED needs REF numerics without qk-norm");
    const int64_t cnt = ((B * a.nkv * 4 + 255) / 256) * 256;
    a.counters = (unsigned*)ws;
    a.part_o = (float*)((char*)ws + cnt);
    a.part_ml = a.part_o + B * n_heads * (int64_t)a.nsplit_max * cache->head_dim;
    a.out = (uint16_t*)out;
    a.rc = dev_env("QIE_DEC_ROPECUR", 1) ? g_rope_cur : nullptr;
    a.pv3 = dev_env("QIE_DEC_PV3", 1);
    // The speculative step is issued before the position is known, so the grid's idle
    // splits (s >= this step's split count: the graph's grid is sized for max_ctx) load a
    // step too and drop it (config 4, max_ctx 1,344: 32-64 idle blocks of 352, 2-4 MB per
    // launch).  Measured, it still pays at B = 8 (3,478.6 vs 3,465.7 tok/s without it) as at
    // B = 1 (358.7 vs 357.2).  QIE_DEC_SPEC (dev A/B): 0 turns it off.
    a.spec_ok = dev_env("QIE_DEC_SPEC", 1) != 0;
    return 0;
}

// the persistent decode kernel's attention role (k_persist.hip) runs the same body with the
// same parameters the stand-alone launch would get
int decode_attn_params(DecodeAttnParams* a, const void* qkv, int64_t B, const int32_t* pos, const void* q_norm,
                       const void* k_norm, const float* rope_cos, const float* rope_sin, int32_t n_heads,
                       const qie_kv_cache* cache, int32_t layer, float eps, int32_t numerics, void* out, void* ws) {
    return fill_dec_params(*a, qkv, B, pos, q_norm, k_norm, rope_cos, rope_sin, n_heads, cache, layer, eps, numerics,
                           out, ws);
}

}  // namespace qie

using namespace qie;

extern "C" {

int64_t qie_attention_workspace_bytes(int64_t M, int32_t n_heads, int32_t head_dim, int32_t max_ctx) {
    const int ns = attn_nsplit(M, max_ctx);
    if (ns == 1) return 0;
    return M * n_heads * (int64_t)ns * (head_dim + 2) * 4;
}

int qie_attention(const void* q, int64_t M, const int32_t* pos, int32_t rows_per_seq,
                  const qie_kv_cache* cache, int32_t layer, int32_t n_heads, void* out, void* ws,
                  void* stream) {
    QIE_REQUIRE(q && pos && cache && cache->k && cache->v && out && M >= 0 && rows_per_seq > 0,
                "qie_attention: bad arguments");
    QIE_REQUIRE(cache->head_dim == 64 || cache->head_dim == 128,
                "qie_attention: head_dim must be 64 or 128 (got %d)", cache->head_dim);
    QIE_REQUIRE(n_heads % cache->n_kv_heads == 0 && n_heads / cache->n_kv_heads <= kMaxGroup,
                "qie_attention: n_heads/n_kv_heads must be an integer <= %d", kMaxGroup);
    QIE_REQUIRE(layer >= 0 && layer < cache->n_layers, "qie_attention: bad layer");
    if (M == 0) return 0;
    if (rows_per_seq >= 32 && M % rows_per_seq == 0) {
        PrefillAttnParams pa;
        pa.q = (const uint16_t*)q;
        pa.pos = pos;
        pa.rows_per_seq = rows_per_seq;
        pa.kc = (const uint16_t*)cache->k;
        pa.vc = (const uint16_t*)cache->v;
        QIE_TRY(kv_map_make(cache, &pa.km, "qie_attention"));
        pa.layer = layer;
        pa.nkv = cache->n_kv_heads;
        pa.nq = n_heads;
        pa.max_ctx = cache->max_ctx;
        pa.M = M;
        pa.out = (uint16_t*)out;
        pa.full_tiles = dev_env("QIE_ATTN_PF_FULL", 1);
        const size_t shm = (size_t)2 * 2 * 64 * cache->head_dim * 2;
        const bool pg = pa.km.table != nullptr;
        // balanced causal split: ceil(ceil(R / 16) / 2) group pairs, NW per workgroup
        const int npair = ((rows_per_seq + 15) / 16 + 1) / 2;
        // 8 waves (16 row groups) per workgroup: each staged K/V tile feeds twice the rows, half
        // the LDS-DMA traffic of 4-wave workgroups (P = 2,048, 7B: 74.1-74.7 -> 69.9-70.7 us,
        // bit-identical; tools/attn_nw_check.py).  Dev A/B: QIE_ATTN_PF_NW = 4.
        const int nw = dev_env("QIE_ATTN_PF_NW", 8) == 4 ? 4 : 8;
        dim3 g2((unsigned)((npair + nw - 1) / nw), (unsigned)n_heads, (unsigned)(M / rows_per_seq));
        auto k2 = nw == 8 ? (cache->head_dim == 128 ? (pg ? attn_prefill_mfma2_kernel<128, true, 8> : attn_prefill_mfma2_kernel<128, false, 8>)
                                                    : (pg ? attn_prefill_mfma2_kernel<64, true, 8> : attn_prefill_mfma2_kernel<64, false, 8>))
                          : (cache->head_dim == 128 ? (pg ? attn_prefill_mfma2_kernel<128, true, 4> : attn_prefill_mfma2_kernel<128, false, 4>)
                                                    : (pg ? attn_prefill_mfma2_kernel<64, true, 4> : attn_prefill_mfma2_kernel<64, false, 4>));
        hipLaunchKernelGGL(k2, g2, dim3(64 * nw), shm, (hipStream_t)stream, pa);
        QIE_LAUNCH_CHECK();
        return 0;
    }
    AttnParams a;
    a.q = (const uint16_t*)q;
    a.pos = pos;
    a.rows_per_seq = rows_per_seq;
    a.kc = (const uint16_t*)cache->k;
    a.vc = (const uint16_t*)cache->v;
    QIE_TRY(kv_map_make(cache, &a.km, "qie_attention"));
    a.layer = layer;
    a.nkv = cache->n_kv_heads;
    a.nq = n_heads;
    a.max_ctx = cache->max_ctx;
    a.nsplit = attn_nsplit(M, cache->max_ctx);
    const int64_t part = M * n_heads * (int64_t)a.nsplit;
    a.part_o = (float*)ws;
    a.part_ml = ws ? (float*)ws + part * cache->head_dim : nullptr;
    a.out = (uint16_t*)out;
    QIE_REQUIRE(a.nsplit == 1 || ws, "qie_attention: workspace required");
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)(a.nkv * a.nsplit), (unsigned)M);
    const bool pg = a.km.table != nullptr;
    if (cache->head_dim == 128) {
        hipLaunchKernelGGL((pg ? attn_split_kernel<128, true> : attn_split_kernel<128, false>), grid, dim3(256), 0, st, a);
        QIE_LAUNCH_CHECK();
        if (a.nsplit > 1) hipLaunchKernelGGL(attn_combine_kernel<128>, dim3(n_heads, (unsigned)M), dim3(128), 0, st, a);
    } else {
        hipLaunchKernelGGL((pg ? attn_split_kernel<64, true> : attn_split_kernel<64, false>), grid, dim3(256), 0, st, a);
        QIE_LAUNCH_CHECK();
        if (a.nsplit > 1) hipLaunchKernelGGL(attn_combine_kernel<64>, dim3(n_heads, (unsigned)M), dim3(64), 0, st, a);
    }
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_debug_tr16_probe(int32_t* out_dev) {
    QIE_REQUIRE(out_dev, "qie_debug_tr16_probe: null");
    hipLaunchKernelGGL(tr16_probe_kernel, dim3(1), dim3(64), 0, nullptr, out_dev);
    QIE_LAUNCH_CHECK();
    return 0;
}

int64_t qie_attention_decode_workspace_bytes(int64_t B, int32_t n_heads, int32_t n_kv_heads, int32_t head_dim,
                                             int32_t max_ctx) {
    // an upper bound for every splits_target <= kDecMaxSplits (nsplit_max in fill_dec_params)
    const int64_t ns = std::min<int64_t>(kDecMaxSplits, (max_ctx + 63) / 64);   // 64- or 128-key steps
    const int64_t cnt = ((B * n_kv_heads * 4 + 255) / 256) * 256;
    return cnt + B * n_heads * ns * (head_dim + 2) * 4;
}

int qie_attention_decode(const void* qkv, int64_t B, const int32_t* pos, const void* q_norm, const void* k_norm,
                         const float* rope_cos, const float* rope_sin, int32_t n_heads, const qie_kv_cache* cache,
                         int32_t layer, float eps, int32_t numerics, void* out, void* ws, void* stream) {
    QIE_REQUIRE(qkv && pos && cache && cache->k && cache->v && rope_cos && rope_sin && out && ws && B > 0,
                "qie_attention_decode: bad arguments");
    QIE_REQUIRE(cache->head_dim == 64 || cache->head_dim == 128,
                "qie_attention_decode: head_dim must be 64 or 128 (got %d)", cache->head_dim);
    QIE_REQUIRE(n_heads % cache->n_kv_heads == 0 && n_heads / cache->n_kv_heads <= kMaxGroup,
                "qie_attention_decode: n_heads/n_kv_heads must be an integer <= %d", kMaxGroup);
    QIE_REQUIRE(layer >= 0 && layer < cache->n_layers, "qie_attention_decode: bad layer");
    DecodeAttnParams a;
    QIE_TRY(fill_dec_params(a, qkv, B, pos, q_norm, k_norm, rope_cos, rope_sin, n_heads, cache, layer, eps, numerics,
                            out, ws));
    dim3 grid((unsigned)(a.nkv * a.nsplit_max), (unsigned)B);
    const bool pg = a.km.table != nullptr;
    // hd 128: 8 waves per workgroup (one 16-key S tile and a 16-dim P.V slice per wave);
    // hd 64 keeps 4 (a 16-dim slice per wave is the MFMA tile's minimum)
    // 4 waves per workgroup (8 at hd 128, one 16-key tile and a 16-dim P.V slice per wave,
    // measured slower: 12.9 vs 9.8 us per launch at ctx 2.3k)
    const bool pr = a.pre_roped != 0;
    auto k2 = cache->head_dim == 128
                  ? (pr ? (pg ? attn_decode_mfma2_kernel<128, true, 4, true> : attn_decode_mfma2_kernel<128, false, 4, true>)
                        : (pg ? attn_decode_mfma2_kernel<128, true, 4, false> : attn_decode_mfma2_kernel<128, false, 4, false>))
                  : (pr ? (pg ? attn_decode_mfma2_kernel<64, true, 4, true> : attn_decode_mfma2_kernel<64, false, 4, true>)
                        : (pg ? attn_decode_mfma2_kernel<64, true, 4, false> : attn_decode_mfma2_kernel<64, false, 4, false>));
    if (a.ks == 64 && cache->head_dim == 128 && !pr)   // 64-key steps (dev A/B)
        k2 = pg ? attn_decode_mfma2_kernel<128, true, 4, false, 64> : attn_decode_mfma2_kernel<128, false, 4, false, 64>;
    if (a.ks == 256 && cache->head_dim == 64)   // one 256-key step (short contexts at hd 64)
        k2 = pr ? (pg ? attn_decode_mfma2_kernel<64, true, 4, true, 256> : attn_decode_mfma2_kernel<64, false, 4, true, 256>)
                : (pg ? attn_decode_mfma2_kernel<64, true, 4, false, 256> : attn_decode_mfma2_kernel<64, false, 4, false, 256>);
    QIE_REQUIRE(a.ks == 128 || (a.ks == 64 && cache->head_dim == 128 && !pr) || (a.ks == 256 && cache->head_dim == 64),
                "qie_attention_decode: internal: no kernel for %d-key steps at hd %d", a.ks, cache->head_dim);
    hipLaunchKernelGGL(k2, grid, dim3(256), 0, (hipStream_t)stream, a);
    QIE_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"

