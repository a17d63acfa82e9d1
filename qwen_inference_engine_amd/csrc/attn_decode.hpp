// attn_decode.hpp — the fused MFMA decode attention body (k_attention.hip) and the helpers
// it shares with the prefill kernel, as a header so that the persistent decode kernel
// (k_persist.hip) runs the SAME body (same arithmetic, bit-identical outputs) as one of its
// roles.  Replaces selfattention (layers/src/self_attension.cu:10-149) for one query row.
#pragma once
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

namespace qie {

constexpr int kMaxGroup = 8;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int kv16_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// 16 bytes per lane global -> LDS (LDS-DMA); `lds` is the wave-instruction's 1-KiB base,
// lane l lands at lds + 16 l
__device__ __forceinline__ void dma16(const uint16_t* src, uint16_t* lds) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

// 16 bytes per lane from a buffer resource into LDS (buffer_load_dwordx4 … lds); `lds` is the
// wave-instruction's 1-KiB base.  (The builtin exists for the device pass only: the host
// pass, which emits the kernel's launch stub, must not instantiate it.)
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t rs, uint16_t* lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds), 16, voff, 0, 0, 0);
#else
    (void)rs; (void)lds; (void)voff;
#endif
}

// ---------------------------------------------------------------------------
// Fused decode attention: q-projection post-processing (qk-norm + RoPE) in the
// prologue, KV append of the new token (qkv_post fused away), split-K over the context,
// and the split combine done by the last arriving workgroup of each (row, kv head):
// write-through (sc1) partials + ticket, one agent acquire in the combiner.
// Grid: (nkv * nsplit_max, B); row m has one query token at position pos[m].
struct DecodeAttnParams {
    const uint16_t* qkv;      // [B][(nq + 2 nkv) * HD] projection output (bias added)
    const int32_t* pos;
    const uint16_t* q_norm;
    const uint16_t* k_norm;
    const float* cs;
    const float* sn;
    uint16_t* kc;
    uint16_t* vc;
    KvMap km;
    int layer, nkv, nq, max_ctx, nsplit_max;
    int splits_target;        // ~splits per (row, kv head) at long context
    int dbg;                  // timing experiments only (QIE_DEC_DBG): 1 no combine,
                              // 8/16 stop after prologue / P.V, 64 exit at once
    int sc1;                  // combine reads the partials with sc1 loads instead of an acquire
    int pre_roped;            // q and the new k arrive rotated by the QKV projection's epilogue
                              // (REF numerics, no qk-norm): the prologue only moves them
    float eps;
    int numerics;
    float* part_o;            // [B][nq][nsplit_max][HD]
    float* part_ml;           // [B][nq][nsplit_max][2]
    unsigned* counters;       // [B][nkv], zero at rest
    uint16_t* out;            // [B][nq * HD]
    // engine-maintained RoPE row of each sequence's CURRENT position (finalize / set_state
    // write it, tagged with the position; [B][rope_cur_stride(HD)]): the prologue's RoPE
    // loads need no position, so with the speculative K / V step every load of the launch
    // goes out at once.  Null (operator API) or a stale tag: the table row at pos.
    const float* rc;
    int pv3;                  // P.V with three bf16 parts of P (else two; dev A/B)
    int spec_ok;              // the speculative K / V step may be issued (see fill_dec_params)
    int ks;                   // keys per block step (host: picks the kernel instance)
};

constexpr int kDecMaxSplits = 512;   // 64k keys per (row, kv head)

__device__ __forceinline__ void unpack_bf8(const uint4& r, float* f) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; j++) { f[2 * j] = bf_lo(w[j]); f[2 * j + 1] = bf_hi(w[j]); }
}
__device__ __forceinline__ uint4 sel4(bool c, const uint4& a, const uint4& b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
// Opaque register pass-through: math on the value cannot be hoisted above this point,
// so the wait for its load lands here (after the K/V loads were issued), not before them.
__device__ __forceinline__ void pin4(uint4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}
__device__ __forceinline__ void pin4(float4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

// Split fp32 probabilities into bf16 parts (hi, then the remainder's hi, ...) two lanes'
// values at a time: one v_cvt_pk_bf16_f32 per pair and packed fp32 subtractions.  A scalar
// (__bf16) cast per element compiled to one cvt_pk per element (half of it wasted) plus a
// shift and a subtraction each — 7 VALU per element for three parts, now 4.5.  Same RNE
// rounding, same exact remainders: bit-identical parts.
typedef float pf32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 pbf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(pf32x2_t v) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, pbf16x2_t));
}
__device__ __forceinline__ pf32x2_t unpk_bf16(uint32_t u) {
    return pf32x2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// e[0..7] -> NP bf16x8 parts (NP = 2: hi + lo; 3: hi + mid + lo)
template <int NP>
__device__ __forceinline__ void split_bf16x8(const float* e, uint4* parts) {
    uint32_t w[NP][4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        pf32x2_t r = pf32x2_t{e[2 * j], e[2 * j + 1]};
#pragma unroll
        for (int k = 0; k < NP; k++) {
            w[k][j] = cvt_pk_bf16(r);
            if (k + 1 < NP) r = r - unpk_bf16(w[k][j]);
        }
    }
#pragma unroll
    for (int k = 0; k < NP; k++) parts[k] = make_uint4(w[k][0], w[k][1], w[k][2], w[k][3]);
}

// ---------------------------------------------------------------------------
// Decode attention on MFMA (default decode path).  The q heads of one kv head
// (G <= 8, padded to 16) play the role of the 16 "query rows" of the prefill
// kernel above, so GQA decode is a 16 x 32 x HD flash step per wave:
//   S^T = K . Q^T : A = K rows straight from HBM into registers (lane: key l&15,
//                   8 contiguous d), B = Q^T from LDS (bf16 after norm + RoPE);
//   O  += P . V   : A = P from the S^T accumulators, split into bf16 hi + lo parts
//                   (two MFMAs) so the fp32 probabilities keep ~16 mantissa bits;
//                   B = V through a per-wave LDS slot read with ds_read_b64_tr_b16.
// Block = (kv head, split) x 4 waves; a block step covers 128 keys (32 per wave);
// waves run an online softmax, are merged in LDS, and the splits are merged by
// the last-arriving block (release / acquire, as the VALU kernel).  The VALU
// kernel spent ~7 us of ~11 in dot products and cross-lane reductions here.
constexpr int kDecMStep = 128;      // keys per block step (4 waves x 32)
constexpr int kDecMSplits = 32;     // default split target
constexpr int kDecMOneSplit = 2;    // contexts of up to this many steps run as ONE split

__host__ __device__ __forceinline__ int decm_chunk(int ctx, int target, int ks = kDecMStep) {
    // Short contexts: one block walks both steps instead of two one-step splits that pay
    // the publish + ticket + combine round trips (Qwen2-0.5B, ctx 129-256: 8.8 -> 7.4 us
    // per launch, 1,235 -> 1,271 tok/s).  Longer contexts want the CUs: a split's K/V comes
    // through one CU, so at ctx 2k ten two-step splits took 13.1 us against 10.5 for twenty
    // one-step ones — also with the second step's loads issued up front (13.6 vs 10.7,
    // measured and dropped: that second register set halved the occupancy).
    if (ctx <= kDecMOneSplit * ks) return kDecMOneSplit * ks;
    const int per = ks * target;
    const int steps = (ctx + per - 1) / per;
    return ks * (steps < 1 ? 1 : steps);
}


// ---------------------------------------------------------------------------
// Decode attention, MFMA: as the prefill kernel's 16-row flash step, but the 4 waves of
// a block split the head dimension for P.V instead of the keys, so no cross-wave
// softmax merge is needed:
//   * S^T for the step's 128 keys: wave w computes keys 32w..32w+31 (2 MFMA tiles),
//     writes the raw dots to LDS, one barrier, then EVERY wave holds all 128 scores;
//   * each wave runs the (identical) online softmax over the 128 keys itself and
//     accumulates O for ITS d-slice (HD/4 dims: 2 tiles at hd 128) over the 4 key
//     blocks of 32 (P in natural key order, V slice via ds_read_b64_tr_b16);
//   * the split's partial O leaves straight from the accumulators (the v1 kernel's
//     LDS merge of 4 waves cost ~2.7 us of a 13.5 us launch).
struct DecPro {
    uint4 raw, nraw;
    float4 c0, s0, c1, s1;
    bool is_q, is_k, is_v, pro, nrm, hf;
};

// this lane's RoPE coefficients from a table row (cos row cp, sin row sp)
template <int HD>
__device__ __forceinline__ void dec_rope_load(DecPro& d, int dl, const float* cp, const float* sp) {
    const int rb = d.hf ? (dl * 8) % (HD / 2) : dl * 4;
    const int rb2 = d.hf ? rb + 4 : rb;
    d.c0 = *reinterpret_cast<const float4*>(cp + rb);
    d.s0 = *reinterpret_cast<const float4*>(sp + rb);
    d.c1 = *reinterpret_cast<const float4*>(cp + rb2);
    d.s1 = *reinterpret_cast<const float4*>(sp + rb2);
}

template <int HD, bool PR>
__device__ __forceinline__ DecPro dec_pro_issue(const DecodeAttnParams& a, const uint16_t* row, int g, int G, int grp,
                                                int dl, const float* cp, const float* sp, bool has_new) {
    DecPro d;
    d.is_q = grp < G;
    d.is_k = grp == G;
    d.is_v = grp == G + 1;
    d.pro = d.is_q || ((d.is_k || d.is_v) && has_new);
    d.hf = a.numerics == QIE_NUMERICS_HF;
    const uint16_t* src = d.is_q ? row + (g * G + grp) * HD
                                 : (d.is_k ? row + a.nq * HD + g * HD : row + (a.nq + a.nkv) * HD + g * HD);
    if (!(d.is_q || d.is_k || d.is_v)) src = row;
    d.raw = *reinterpret_cast<const uint4*>(src + dl * 8);
    if constexpr (PR) {   // rotated upstream, no qk-norm: nothing else to load
        d.nrm = false;
        return d;
    }
    const uint16_t* nwp = d.is_q ? a.q_norm : a.k_norm;
    d.nrm = nwp != nullptr && !d.is_v;
    d.nraw = *reinterpret_cast<const uint4*>((nwp ? nwp : row) + dl * 8);
    dec_rope_load<HD>(d, dl, cp, sp);
    return d;
}

// qk-norm + RoPE of the q heads and the new k, then q -> LDS (bf16), new k/v -> cache
// and LDS.  Branch-free (only the stores are predicated), stores predicated, loads unconditional).
template <int HD, bool PR>
__device__ __forceinline__ void dec_pro_finish(const DecodeAttnParams& a, DecPro& d, int dl, int grp, int64_t poff,
                                               uint16_t* kb, uint16_t* vb, uint16_t (*q_s)[HD],
                                               uint16_t (*kv_new)[HD]) {
#pragma clang fp contract(off)
    constexpr int LPT = HD / 8;
    if constexpr (PR) {   // q / new k already rotated: move them
        pin4(d.raw);
        if (d.is_q) {
            *reinterpret_cast<uint4*>(&q_s[grp][dl * 8]) = d.raw;
        } else if (d.pro) {
            *reinterpret_cast<uint4*>((d.is_k ? kb : vb) + poff + dl * 8) = d.raw;
            *reinterpret_cast<uint4*>(&kv_new[d.is_k ? 0 : 1][dl * 8]) = d.raw;
        }
        return;
    }
    pin4(d.raw); pin4(d.nraw); pin4(d.c0); pin4(d.s0); pin4(d.c1); pin4(d.s1);
    float x[8], wv[8];
    unpack_bf8(d.raw, x);
    unpack_bf8(d.nraw, wv);
    // qk-norm (Qwen3) and HF numerics are launch-uniform: branch around them instead of
    // computing both forms per element (Qwen2, REF: neither — 8 divisions and the HF RoPE
    // products per lane were dead work on the critical path)
    if (a.q_norm != nullptr || a.k_norm != nullptr) {   // per lane: d.nrm picks q_norm / k_norm
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) ss += x[j] * x[j];
        ss = group_sum<LPT>(ss);
        const float rms = sqrtf((ss / (float)HD) + a.eps);
        if (d.hf) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float xn = rbf(wv[j] * rbf(x[j] * (1.0f / rms)));
                x[j] = d.nrm ? xn : x[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float xn = rbf((x[j] / rms) * wv[j]);
                x[j] = d.nrm ? xn : x[j];
            }
        }
    }
    const float cv[8] = {d.c0.x, d.c0.y, d.c0.z, d.c0.w, d.c1.x, d.c1.y, d.c1.z, d.c1.w};
    const float sv[8] = {d.s0.x, d.s0.y, d.s0.z, d.s0.w, d.s1.x, d.s1.y, d.s1.z, d.s1.w};
    float y[8];
    if (d.hf) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = __shfl_xor(x[j], LPT / 2, 64);
        const float sg = dl < LPT / 2 ? -1.f : 1.f;   // rotate_half: first half takes -x[j + hd/2]
#pragma unroll
        for (int j = 0; j < 8; j++) y[j] = rbf(rbf(x[j] * cv[j]) + rbf((sg * o[j]) * sv[j]));
    } else {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            y[j] = rbf(x[j] * cv[j / 2] - x[j + 1] * sv[j / 2]);
            y[j + 1] = rbf(x[j + 1] * cv[j / 2] + x[j] * sv[j / 2]);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = d.is_v ? x[j] : y[j];
    const uint4 packed = make_uint4(pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]), pack2(x[6], x[7]));
    if (d.is_q) {
        *reinterpret_cast<uint4*>(&q_s[grp][dl * 8]) = packed;
    } else if (d.pro) {
        uint16_t* dst = (d.is_k ? kb : vb) + poff + dl * 8;
        *reinterpret_cast<uint4*>(dst) = packed;
        *reinterpret_cast<uint4*>(&kv_new[d.is_k ? 0 : 1][dl * 8]) = packed;
    }
}

// Body of the decode attention for workgroup (bx, by); true when this workgroup wrote a
// combined (row, kv head) output (its stores are write-through, sc1).
// Hooks of the body (X): the stand-alone kernel runs it with AttnNoHook — q / k / v rows from
// a.qkv, outputs to a.out.  The persistent decode kernel (k_persist.hip) passes a hook whose
// gather() fills the q / k / v row image (a.qkv points at it) from the projection's hand-off
// granules AFTER this block's K / V loads are issued (they need no q), and whose out2 / out4
// take the block's output values (to publish them as granules).  The arithmetic is the same.
struct AttnNoHook {
    static constexpr bool on = false;
    __device__ void gather() {}
    __device__ void out1(int64_t, uint16_t) {}
    __device__ void out4(int64_t, unsigned long long) {}
};

template <int HD, bool PG, int NWA, bool PR, int KS, class X = AttnNoHook>
__device__ __forceinline__ bool attn_decode_mfma2_body(const DecodeAttnParams& a, const int bx, const int by,
                                                       X* hook = nullptr) {
#pragma clang fp contract(off)
    constexpr int LPT = HD / 8;          // prologue: lanes per head row
    constexpr int KSTEPS = HD / 32;      // MFMA k-steps over d for S
    constexpr int CPR = HD / 8;          // 16-byte chunks per K row
    constexpr int DW = HD / NWA;         // output dims per wave
    constexpr int DTW = DW / 16;         // output d tiles per wave (2 at hd 128 x 4 waves, else 1)
    constexpr int CPW = DW / 8;          // 16-byte chunks of a V row per wave
    constexpr int VCH = KS * CPW / 64;   // V chunks per lane per step
    constexpr int TPW = KS / (16 * NWA);  // 16-key S tiles per wave per step
    constexpr int NT = 64 * NWA;         // threads
    static_assert(DTW >= 1 && TPW >= 1, "attn_decode: NWA too large for HD");
    __shared__ __attribute__((aligned(16))) uint16_t q_s[16][HD];
    __shared__ __attribute__((aligned(16))) uint16_t kv_new[2][HD];
    __shared__ __attribute__((aligned(16))) uint16_t v_s[NWA][KS * DW];
    __shared__ __attribute__((aligned(16))) float s_s[16][KS + 4];
    __shared__ int last_flag;

    const int64_t m = by;
    const int g = bx / a.nsplit_max, s = bx % a.nsplit_max;
    const int G = a.nq / a.nkv;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fr = lane & 15, gq = lane >> 4;
    const int grp = tid / LPT, dl = tid % LPT;
    const int QKVD = (a.nq + 2 * a.nkv) * HD;
    const uint16_t* row = a.qkv + m * (int64_t)QKVD;
    const int64_t head_off = kv_run_off(a.km, (int64_t)a.layer * a.nkv + g, HD);
    uint16_t* kb = a.kc + head_off;
    uint16_t* vb = a.vc + head_off;
    uint4 kf[TPW][KSTEPS], vr[VCH];
    // step loads of keys [kb0, kb0 + 128), rows past `last` re-read row `last`
    auto load_step_at = [&](int kb0, int last) {
        // a 128-key step never straddles a page (chunks and pages are multiples of 128)
        const int64_t so = kv_tok<PG>(a.km, m, kb0, HD);
#pragma unroll
        for (int t = 0; t < TPW; t++) {
            const int key = min(kb0 + 16 * TPW * wave + 16 * t + fr, last);
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ks++)
                kf[t][ks] = *reinterpret_cast<const uint4*>(kb + so + (int64_t)(key - kb0) * HD + 32 * ks + 8 * gq);
        }
#pragma unroll
        for (int i = 0; i < VCH; i++) {
            const int c = lane + 64 * i;
            const int key = min(kb0 + c / CPW, last);
            vr[i] = *reinterpret_cast<const uint4*>(vb + so + (int64_t)(key - kb0) * HD + wave * DW + (c % CPW) * 8);
        }
    };
    // Speculative step: the split of every context of 257 ..
    // 128 * splits keys is keys [128 s, 128 s + 128) (decm_chunk's one-step rule), so its
    // K / V loads go out with the position load instead of one HBM round trip behind it.
    // The rotated q / k / v row goes out first (position-independent): vmcnt retires in
    // order, and the prologue that waits for it must not wait behind the whole K / V step.
    // Without the pre-rotation the same holds when the engine keeps the current position's
    // RoPE row (a.rc, tagged with the position): the prologue's loads then need no position
    // either, and a stale tag (a position set some other way) reloads the table row.
    // (Paged, measured in round 5: the step's page from the block-table entry of (row,
    // 128 s) needs no position either, but the speculative form ran config 4 at 3,563 vs
    // 3,624 tok/s for the plain one — the table round trip still precedes the K / V loads.)
    constexpr bool SPEC = !PG;
    const bool spec = (PR || a.rc != nullptr) && a.spec_ok;   // uniform
    const int p = a.pos[m];
    const float* rcm = a.rc ? a.rc + m * rope_cur_stride(HD) : a.cs;
    const int rtag = a.rc ? __float_as_int(rcm[0]) : -1;
    DecPro pr;
    if (SPEC && spec) {
        if constexpr (X::on) {   // the row is gathered after the K / V step is in flight
            load_step_at(KS * s, a.max_ctx - 1);
            __builtin_amdgcn_sched_barrier(0);
            hook->gather();
            pr = dec_pro_issue<HD, PR>(a, row, g, G, grp, dl, rcm + 8, rcm + 8 + HD / 2, false);
        } else {
            pr = dec_pro_issue<HD, PR>(a, row, g, G, grp, dl, rcm + 8, rcm + 8 + HD / 2, false);
            __builtin_amdgcn_sched_barrier(0);
            load_step_at(KS * s, a.max_ctx - 1);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else if constexpr (X::on) {
        hook->gather();
    }
    const int ctx = p + 1;
    const int chunk = decm_chunk(ctx, a.splits_target, KS);
    const int nsplit = (ctx + chunk - 1) / chunk;
    if (s >= nsplit || QIE_DBG(a.dbg & 64)) return false;
    const int t0 = s * chunk, t1 = min(ctx, t0 + chunk);
    const int nstep = (t1 - t0 + KS - 1) / KS;
    const bool has_new = (t1 == ctx);
    auto load_step = [&](int st) { load_step_at(t0 + st * KS, t1 - 1); };

    // ---------------- loads: prologue operands, then step 0's K tiles and V slice
    if (SPEC && spec) {
        pr.pro = pr.is_q || ((pr.is_k || pr.is_v) && has_new);
        if (!PR && rtag != p)   // uniform: the kept row is not this position's
            dec_rope_load<HD>(pr, dl, a.cs + (int64_t)p * (HD / 2), a.sn + (int64_t)p * (HD / 2));
    } else {
        pr = dec_pro_issue<HD, PR>(a, row, g, G, grp, dl, a.cs + (int64_t)p * (HD / 2), a.sn + (int64_t)p * (HD / 2),
                                   has_new);
    }
    __builtin_amdgcn_sched_barrier(0);
    // (uniform) the speculative step is this split's first step iff the split starts at key
    // KS s: one-step splits, and split 0 of every context (the one-split contexts of <= 2
    // steps, Qwen2-0.5B's ctx 129-256, re-issued the same loads behind the position: +1.2 us)
    if (!(SPEC && spec) || t0 != KS * s) load_step(0);
    if (SPEC && spec) {
        // rows past the context hold whatever the cache has there: their scores are masked
        // to -inf (P = 0), and their V rows are zeroed so that 0 * V stays 0 for any bits
#pragma unroll
        for (int i = 0; i < VCH; i++)
            if (t0 + (lane + 64 * i) / CPW >= t1) vr[i] = make_uint4(0, 0, 0, 0);
    }
    dec_pro_finish<HD, PR>(a, pr, dl, grp, kv_tok<PG>(a.km, m, p, HD), kb, vb, q_s, kv_new);
    for (int idx = tid; idx < (16 - G) * CPR; idx += NT)   // padded q rows
        *reinterpret_cast<uint4*>(&q_s[G + idx / CPR][(idx % CPR) * 8]) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (QIE_DBG(a.dbg & 8)) {
        if (tid == 0) a.out[m] = (uint16_t)(kf[0][0].x + vr[VCH - 1].y + kf[TPW - 1][KSTEPS - 1].z);
        return false;
    }

    bf16x8_t qb[KSTEPS];
    uint4 knew[KSTEPS];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ks++) {
        qb[ks] = *reinterpret_cast<const bf16x8_t*>(&q_s[fr][32 * ks + 8 * gq]);
        knew[ks] = *reinterpret_cast<const uint4*>(&kv_new[0][32 * ks + 8 * gq]);
    }
    const float scale = sqrtf((float)HD);
    // dot / scale as q = dot * (1 / scale) plus one FMA residual step (Markstein): the
    // correctly rounded quotient for every dot above 2^-100 in magnitude (k_decode_fp8.hip
    // d8_rms_pair), three VALU ops instead of the IEEE division sequence's ~10 with its
    // serial latency — 8 quotients per lane per step on the step's critical path
    const float inv_scale = 1.0f / scale;
    auto qdiv = [&](float d) {
        const float q = d * inv_scale;
        if constexpr (HD == 64 || HD == 256) return q;   // sqrt(hd) a power of two: exact
        else return fmaf(fmaf(-q, scale, d), inv_scale, q);
    };
    float m_run = -INFINITY, l_run = 0.f;
    f32x4_t oacc[DTW];
#pragma unroll
    for (int d = 0; d < DTW; d++) oacc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    uint16_t* vw = &v_s[wave][0];
    const int q4 = fr >> 2, p4 = fr & 3;

    for (int st = 0; st < nstep; st++) {
        const int kb0 = t0 + st * KS;
        // Only the step holding the new token takes its K / V rows from LDS, and only a step
        // past the split's end masks scores (the last step of the last split; both uniform,
        // scalar branches around in-place selects): the other steps carry no per-element
        // compare / select.  (A whole second copy of the step body per case took the hd-128
        // kernel from 216 to 298 registers.)
        const bool hasp = p >= kb0 && p < kb0 + KS;
        const bool full = kb0 + KS <= t1;
        if (hasp) {
#pragma unroll
            for (int t = 0; t < TPW; t++) {
                const bool nw = kb0 + 16 * TPW * wave + 16 * t + fr == p;
#pragma unroll
                for (int ks = 0; ks < KSTEPS; ks++) kf[t][ks] = sel4(nw, knew[ks], kf[t][ks]);
            }
#pragma unroll
            for (int i = 0; i < VCH; i++) {
                const int c = lane + 64 * i;
                const int r = c / CPW, ch = c % CPW;
                const uint4 vn = *reinterpret_cast<const uint4*>(&kv_new[1][wave * DW + ch * 8]);
                vr[i] = sel4(kb0 + r == p, vn, vr[i]);
            }
        }
        // ---- S^T for this wave's 32 keys -> LDS (raw dots)
#pragma unroll
        for (int t = 0; t < TPW; t++) {
            f32x4_t sacc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KSTEPS; ks++)
                sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[t][ks]), qb[ks], sacc, 0, 0, 0);
            // C map: col = head fr, rows = keys 4 gq + r of the tile; scores s = dot / sqrt(hd)
            // (self_attension.cu) divided once here, not by every wave that reads them
            *reinterpret_cast<float4*>(&s_s[fr][16 * TPW * wave + 16 * t + 4 * gq]) =
                make_float4(qdiv(sacc[0]), qdiv(sacc[1]), qdiv(sacc[2]), qdiv(sacc[3]));
        }
        // ---- this wave's V slice -> LDS (the new token's row from kv_new)
#pragma unroll
        for (int i = 0; i < VCH; i++) {
            const int c = lane + 64 * i;
            const int r = c / CPW, ch = c % CPW;
            *reinterpret_cast<uint4*>(vw + r * DW + ch * 8) = vr[i];
        }
        if (st + 1 < nstep) load_step(st + 1);
        __syncthreads();   // scores and V slices visible
        // ---- online softmax over the step's 128 keys (every wave, identical); lane:
        // head fr, keys 32 c + 8 gq + j (natural order, the P.V k slots)
        float e[KS / 32][8];
        float mt = -INFINITY;
#pragma unroll
        for (int c = 0; c < KS / 32; c++) {
            const float4 lo = *reinterpret_cast<const float4*>(&s_s[fr][32 * c + 8 * gq]);
            const float4 hi = *reinterpret_cast<const float4*>(&s_s[fr][32 * c + 8 * gq + 4]);
            e[c][0] = lo.x; e[c][1] = lo.y; e[c][2] = lo.z; e[c][3] = lo.w;
            e[c][4] = hi.x; e[c][5] = hi.y; e[c][6] = hi.z; e[c][7] = hi.w;
        }
        if (!full) {
#pragma unroll
            for (int c = 0; c < KS / 32; c++)
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (kb0 + 32 * c + 8 * gq + j >= t1) e[c][j] = -INFINITY;
        }
#pragma unroll
        for (int c = 0; c < KS / 32; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) mt = fmaxf(mt, e[c][j]);
        mt = xor32_max(xor16_max(mt));
        const float m_new = fmaxf(m_run, mt);
        const float m_use = m_new == -INFINITY ? 0.f : m_new;
        // __expf (v_exp_f32 on x * log2 e, ~2 ulp): every wave exponentiates all 128 scores,
        // and the libm expf sequence was ~0.8 us of the step; the reference build itself
        // compiles with -use_fast_math, i.e. the same approximation.
        const float alpha = __expf(m_run - m_use);
        float ls = 0.f;
#pragma unroll
        for (int c = 0; c < KS / 32; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                e[c][j] = __expf(e[c][j] - m_use);
                ls += e[c][j];
            }
        ls = xor32_sum(xor16_sum(ls));
        l_run = l_run * alpha + ls;
        m_run = m_new;
        // bit-identical skip, as in the prefill kernel: step 0's O is zero, and alpha == 1
        // exactly where no row's max grew (wave-uniform ballot)
        if (st > 0 && __builtin_amdgcn_ballot_w64(alpha != 1.0f) != 0) {
            float ar[4];
#pragma unroll
            for (int r = 0; r < 4; r++) ar[r] = __shfl(alpha, gq * 4 + r, 64);
#pragma unroll
            for (int d = 0; d < DTW; d++)
#pragma unroll
                for (int r = 0; r < 4; r++) oacc[d][r] *= ar[r];
        }
        // ---- O[:, slice] += P . V[:, slice], P = hi + mid + lo: three bf16 parts hold all
        // 24 bits of the fp32 probability, so every P.V product is the reference's fp32
        // product (self_attension.cu:127-135) — only the accumulation order differs
#pragma unroll
        for (int c = 0; c < KS / 32; c++) {
            uint4 pp[3];
            split_bf16x8<3>(e[c], pp);
            const bf16x8_t ph = __builtin_bit_cast(bf16x8_t, pp[0]), pm = __builtin_bit_cast(bf16x8_t, pp[1]),
                           pl = __builtin_bit_cast(bf16x8_t, pp[2]);
#pragma unroll
            for (int d = 0; d < DTW; d++) {
                const uint16_t* a0 = vw + (32 * c + 8 * gq + q4) * DW + 16 * d + 4 * p4;
                const i16x4_t v0 =
                    __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)(a0));
                const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) i16x4_t*)(a0 + 4 * DW));
                const bf16x8_t vb8 = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                oacc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vb8, oacc[d], 0, 0, 0);
                oacc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pm, vb8, oacc[d], 0, 0, 0);
                if (!QIE_DBG(!a.pv3)) oacc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl, vb8, oacc[d], 0, 0, 0);
            }
        }
        __syncthreads();   // scores / V slots free for the next step
    }
    if (QIE_DBG(a.dbg & 16)) {
        if (tid == 0) a.out[m] = (uint16_t)(oacc[0][0] + m_run);
        return false;
    }

    // ---------------- this wave's d-slice of the split result (rows = heads 4 gq + r)
    const int nq = a.nq;
    float lr[4];
#pragma unroll
    for (int r = 0; r < 4; r++) lr[r] = __shfl(l_run, gq * 4 + r, 64);
    if (nsplit == 1) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int h = 4 * gq + r;
            if (h >= G) continue;
#pragma unroll
            for (int d = 0; d < DTW; d++) {
                const int64_t oi = m * (int64_t)nq * HD + (int64_t)(g * G + h) * HD + wave * DW + 16 * d + fr;
                if constexpr (X::on) hook->out1(oi, f2bf(oacc[d][r] / lr[r]));
                else a.out[oi] = f2bf(oacc[d][r] / lr[r]);
            }
        }
        return false;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int h = 4 * gq + r;
        if (h >= G) continue;
        const int64_t pi = (m * nq + g * G + h) * (int64_t)a.nsplit_max + s;
        // write-through (sc1) stores: published by the drain + ticket below, no release
        // fence (cdna_hip_programming.md, in-launch split-K reduction)
#pragma unroll
        for (int d = 0; d < DTW; d++)
            __hip_atomic_store(&a.part_o[pi * HD + wave * DW + 16 * d + fr], oacc[d][r], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave == 0 && gq == 0 && fr < G) {
        const int64_t pi = (m * nq + g * G + fr) * (int64_t)a.nsplit_max + s;
        __hip_atomic_store(&a.part_ml[pi * 2], m_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.part_ml[pi * 2 + 1], l_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---------------- publish this split; the last arriver combines (acquire)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    __syncthreads();
    if (QIE_DBG(a.dbg & 1)) return false;
    unsigned* cnt = a.counters + m * a.nkv + g;
    if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag = (old == (unsigned)nsplit - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!last_flag || QIE_DBG(a.dbg & 128)) return false;   // (dev timing exit 128: ticket taken, no combine)
    // Default: 16-B sc1 buffer loads on a uniform (SGPR) resource instead of the acquire
    // (MI355X_MICROARCH.md hand-off row 1): 9.79 -> 9.56 us per launch.  (Round 2 measured
    // 8-B agent-scope atomic loads at 11.4 vs 10.7 us, and 16-B sc1 loads at 73 us — that
    // form put the resource in VGPRs, a waterfall loop per load.)
    if (!a.sc1) {
        if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // Per-thread online combine: thread (head gi, d4) loads the (m, l) of EVERY split of its
    // head together with its 16-byte slice of every split's partial O (one batch of JB
    // splits = one round trip; ctx <= JB * 128 keys in one), then merges them itself — no
    // per-head wave pass, LDS weight table or barrier between the two load rounds.
    constexpr int JB = KS == 64 ? 40 : (KS == 128 ? 24 : 16);   // splits per combine round trip
    const bool has_item = tid < G * (HD / 4);
    const int gi = has_item ? tid / (HD / 4) : 0, d4 = tid % (HD / 4);
    const int64_t hbase = (m * nq + g * G + gi) * (int64_t)a.nsplit_max;
    const float4* src4 = reinterpret_cast<const float4*>(a.part_o) + hbase * (HD / 4) + d4;
    const float2* ml2 = reinterpret_cast<const float2*>(a.part_ml) + hbase;
    float mx = -INFINITY, ls = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j0 = 0; j0 < nsplit; j0 += JB) {
        float4 v[JB];
        float2 w[JB];
        if (a.sc1) {
            // sc1 loads (L2 / memory side, never a stale L1 line) in place of the acquire:
            // every partial was stored sc1 by a wave that drained (vmcnt 0) before its
            // workgroup's barrier and ticket add, and this workgroup's add came last
            // (MI355X_MICROARCH.md hand-off table, row 1).  Buffer loads on a uniform
            // resource: the resource stays in SGPRs.
            const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)a.part_o, 0, 0x7fffffff, 0x00020000);
            const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)a.part_ml, 0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int jj = 0; jj < JB; jj++) {
                const int j = min(j0 + jj, nsplit - 1);
                const u32x4_t q4 = __builtin_amdgcn_raw_buffer_load_b128(
                    ro, (int)(((hbase + j) * (HD / 4) + d4) * 16), 0, 16);
                const u32x2_t q2 = __builtin_amdgcn_raw_buffer_load_b64(rm, (int)((hbase + j) * 8), 0, 16);
                v[jj] = make_float4(__uint_as_float(q4.x), __uint_as_float(q4.y), __uint_as_float(q4.z),
                                    __uint_as_float(q4.w));
                w[jj] = make_float2(__uint_as_float(q2.x), __uint_as_float(q2.y));
            }
        } else {
#pragma unroll
            for (int jj = 0; jj < JB; jj++) {
                const int j = min(j0 + jj, nsplit - 1);
                v[jj] = src4[(int64_t)j * (HD / 4)];
                w[jj] = ml2[j];
            }
        }
        float mb = mx;
#pragma unroll
        for (int jj = 0; jj < JB; jj++) mb = fmaxf(mb, j0 + jj < nsplit ? w[jj].x : -INFINITY);
        const float sc = __expf(mx - mb);   // 0 on the first batch (mx = -inf, mb finite)
        ls *= sc;
        acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc;
#pragma unroll
        for (int jj = 0; jj < JB; jj++) {
            const float c = j0 + jj < nsplit ? __expf(w[jj].x - mb) : 0.f;
            ls = fmaf(w[jj].y, c, ls);
            acc.x = fmaf(c, v[jj].x, acc.x);
            acc.y = fmaf(c, v[jj].y, acc.y);
            acc.z = fmaf(c, v[jj].z, acc.z);
            acc.w = fmaf(c, v[jj].w, acc.w);
        }
        mx = mb;
    }
    if (has_item) {
        uint16_t* dst = a.out + m * (int64_t)nq * HD + (int64_t)(g * G + gi) * HD + d4 * 4;
        // divided (not multiplied by 1/l): the softmax normalisation's one rounding
        const unsigned long long pk = (unsigned long long)pack2(acc.x / ls, acc.y / ls) |
                                      ((unsigned long long)pack2(acc.z / ls, acc.w / ls) << 32);
        if constexpr (X::on) hook->out4(m * (int64_t)nq * HD + (int64_t)(g * G + gi) * HD + d4 * 4, pk);
        else __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

}  // namespace qie
