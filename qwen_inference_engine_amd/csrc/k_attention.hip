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

#include <cstdlib>

namespace qie {

struct AttnParams {
    const uint16_t* q;
    const int32_t* pos;
    int rows_per_seq;
    const uint16_t* kc;
    const uint16_t* vc;
    int64_t seq_stride;
    int layer, nkv, nq, max_ctx;
    int nsplit;
    float* part_o;    // [M][nq][nsplit][HD]
    float* part_ml;   // [M][nq][nsplit][2]
    uint16_t* out;    // [M][nq*HD]
};

constexpr int kMaxGroup = 8;

template <int HD>
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
    const int64_t head_off = (((int64_t)a.layer * a.nkv + g) * a.max_ctx) * HD;
    const uint16_t* kb = a.kc + seq * a.seq_stride + head_off + dl * 8;
    const uint16_t* vb = a.vc + seq * a.seq_stride + head_off + dl * 8;

    for (int t = t0 + wave * TPW + sub; t < t1; t += 4 * TPW) {
        uint4 kv = *reinterpret_cast<const uint4*>(kb + (int64_t)t * HD);
        uint4 vv = *reinterpret_cast<const uint4*>(vb + (int64_t)t * HD);
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
// Fused decode attention: q-projection post-processing (qk-norm + RoPE) in the
// prologue, KV append of the new token (qkv_post fused away), 64-token splits
// with a two-pass block softmax, and the split combine done by the last
// arriving workgroup of each (row, kv head) — agent-scope release before the
// ticket, agent-scope acquire before reading the other splits' partials
// (cdna_hip_programming.md §5 "In-launch split-K reduction").
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
    int64_t seq_stride;
    int layer, nkv, nq, max_ctx, nsplit_max;
    float eps;
    int numerics;
    float* part_o;            // [B][nq][nsplit_max][HD]
    float* part_ml;           // [B][nq][nsplit_max][2]
    unsigned* counters;       // [B][nkv], zero at rest
    uint16_t* out;            // [B][nq * HD]
};

constexpr int kDecChunk = 64;

template <int HD>
__global__ __launch_bounds__(256) void attn_decode_kernel(DecodeAttnParams a) {
#pragma clang fp contract(off)
    constexpr int LPT = HD / 8;          // lanes per key row
    constexpr int TPB = 256 / LPT;       // keys per block step (16 or 32)
    constexpr int NT = kDecChunk / TPB;  // keys per thread
    __shared__ __attribute__((aligned(16))) float q_s[kMaxGroup][HD];
    __shared__ __attribute__((aligned(16))) uint16_t kv_new[2][HD];
    __shared__ float red_m[4][kMaxGroup], red_l[4][kMaxGroup];
    __shared__ float red_o[4][kMaxGroup][HD];
    __shared__ int last_flag;

    const int64_t m = blockIdx.y;
    const int g = blockIdx.x / a.nsplit_max, s = blockIdx.x % a.nsplit_max;
    const int G = a.nq / a.nkv;
    const int p = a.pos[m], ctx = p + 1;
    const int nsplit = (ctx + kDecChunk - 1) / kDecChunk;
    if (s >= nsplit) return;
    const int t0 = s * kDecChunk, t1 = min(ctx, t0 + kDecChunk);
    const bool has_new = (t1 == ctx);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = tid / LPT, dl = tid % LPT;
    const int QKVD = (a.nq + 2 * a.nkv) * HD;
    const uint16_t* row = a.qkv + m * (int64_t)QKVD;
    const bool hf = a.numerics == QIE_NUMERICS_HF;
    const int64_t head_off = (((int64_t)a.layer * a.nkv + g) * a.max_ctx) * HD;
    uint16_t* kb = a.kc + m * a.seq_stride + head_off;
    uint16_t* vb = a.vc + m * a.seq_stride + head_off;

    // ---------------- prologue: q heads (norm + RoPE), new K (norm + RoPE), new V
    if (grp < G + 2) {
        const bool is_q = grp < G, is_k = grp == G, is_v = grp == G + 1;
        if (is_q || ((is_k || is_v) && has_new)) {
            const uint16_t* src = is_q ? row + (g * G + grp) * HD
                                       : (is_k ? row + a.nq * HD + g * HD : row + (a.nq + a.nkv) * HD + g * HD);
            uint4 raw = *reinterpret_cast<const uint4*>(src + dl * 8);
            float x[8];
            {
                uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
                for (int j = 0; j < 4; j++) { x[2 * j] = bf_lo(w[j]); x[2 * j + 1] = bf_hi(w[j]); }
            }
            if (!is_v) {
                const uint16_t* nw = is_q ? a.q_norm : a.k_norm;
                if (nw) {   // qk_norm.cu:43-79 (per-head RMSNorm)
                    float ss = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; j++) ss += x[j] * x[j];
#pragma unroll
                    for (int off = LPT / 2; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
                    const float rms = sqrtf((ss / (float)HD) + a.eps);
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const float wv = bf2f(nw[dl * 8 + j]);
                        x[j] = hf ? rbf(wv * rbf(x[j] * (1.0f / rms))) : rbf((x[j] / rms) * wv);
                    }
                }
                // RoPE at position p (RoPE.cu:6-22 interleaved / HF rotate_half)
                const float* c = a.cs + (int64_t)p * (HD / 2);
                const float* sn = a.sn + (int64_t)p * (HD / 2);
                float y[8];
                if (hf) {
                    float o[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) o[j] = __shfl_xor(x[j], LPT / 2, 64);
                    const bool first = dl < LPT / 2;
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const int ti = (dl * 8 + j) % (HD / 2);
                        y[j] = first ? rbf(rbf(x[j] * c[ti]) + rbf(-o[j] * sn[ti]))
                                     : rbf(rbf(x[j] * c[ti]) + rbf(o[j] * sn[ti]));
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; j += 2) {
                        const int ti = dl * 4 + j / 2;
                        y[j] = rbf(x[j] * c[ti] - x[j + 1] * sn[ti]);
                        y[j + 1] = rbf(x[j + 1] * c[ti] + x[j] * sn[ti]);
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; j++) x[j] = y[j];
            }
            if (is_q) {
#pragma unroll
                for (int j = 0; j < 8; j++) q_s[grp][dl * 8 + j] = x[j];
            } else {
                const uint4 packed = make_uint4(pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]),
                                                pack2(x[6], x[7]));
                uint16_t* dst = (is_k ? kb : vb) + (int64_t)p * HD + dl * 8;
                *reinterpret_cast<uint4*>(dst) = packed;
                *reinterpret_cast<uint4*>(&kv_new[is_k ? 0 : 1][dl * 8]) = packed;
            }
        }
    }
    __syncthreads();

    // ---------------- K/V loads for this thread's NT keys (all issued up front)
    uint4 kr[NT], vr[NT];
    int tt[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) {
        const int t = t0 + grp + TPB * i;
        tt[i] = t;
        const int tc = t < t1 ? t : t0;   // masked slots re-read a written row (never garbage)
        if (tc == p) {
            kr[i] = *reinterpret_cast<const uint4*>(&kv_new[0][dl * 8]);
            vr[i] = *reinterpret_cast<const uint4*>(&kv_new[1][dl * 8]);
        } else {
            kr[i] = *reinterpret_cast<const uint4*>(kb + (int64_t)tc * HD + dl * 8);
            vr[i] = *reinterpret_cast<const uint4*>(vb + (int64_t)tc * HD + dl * 8);
        }
    }
    // ---------------- scores  s = dot(q, k) / sqrtf(hd)
    const float scale = sqrtf((float)HD);
    float sc[NT][kMaxGroup];
#pragma unroll
    for (int i = 0; i < NT; i++) {
        float kf[8];
        uint32_t w[4] = {kr[i].x, kr[i].y, kr[i].z, kr[i].w};
#pragma unroll
        for (int j = 0; j < 4; j++) { kf[2 * j] = bf_lo(w[j]); kf[2 * j + 1] = bf_hi(w[j]); }
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) { sc[i][gi] = -INFINITY; continue; }
            const float4 q0 = *reinterpret_cast<const float4*>(&q_s[gi][dl * 8]);
            const float4 q1 = *reinterpret_cast<const float4*>(&q_s[gi][dl * 8 + 4]);
            float d = 0.f;
            d = fmaf(q0.x, kf[0], d); d = fmaf(q0.y, kf[1], d); d = fmaf(q0.z, kf[2], d); d = fmaf(q0.w, kf[3], d);
            d = fmaf(q1.x, kf[4], d); d = fmaf(q1.y, kf[5], d); d = fmaf(q1.z, kf[6], d); d = fmaf(q1.w, kf[7], d);
#pragma unroll
            for (int off = LPT / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            sc[i][gi] = tt[i] < t1 ? d / scale : -INFINITY;
        }
    }
    // ---------------- block max per head
    float mx[kMaxGroup];
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++) {
        float v = -INFINITY;
#pragma unroll
        for (int i = 0; i < NT; i++) v = fmaxf(v, sc[i][gi]);
#pragma unroll
        for (int off = LPT; off < 64; off <<= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
        mx[gi] = v;
    }
    if (lane == 0)
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) red_m[wave][gi] = mx[gi];
    __syncthreads();
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++)
        mx[gi] = fmaxf(fmaxf(red_m[0][gi], red_m[1][gi]), fmaxf(red_m[2][gi], red_m[3][gi]));
    // ---------------- p = exp(s - max), l = sum p, o = sum p v
    float l[kMaxGroup], o[kMaxGroup][8];
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++) {
        l[gi] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) o[gi][j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < NT; i++) {
        float vf[8];
        uint32_t w[4] = {vr[i].x, vr[i].y, vr[i].z, vr[i].w};
#pragma unroll
        for (int j = 0; j < 4; j++) { vf[2 * j] = bf_lo(w[j]); vf[2 * j + 1] = bf_hi(w[j]); }
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) continue;
            const float e = tt[i] < t1 ? expf(sc[i][gi] - mx[gi]) : 0.f;
            l[gi] += e;
#pragma unroll
            for (int j = 0; j < 8; j++) o[gi][j] = fmaf(e, vf[j], o[gi][j]);
        }
    }
    // reduce over the key slots of the wave, then over waves via LDS
#pragma unroll
    for (int gi = 0; gi < kMaxGroup; gi++) {
        if (gi >= G) continue;
#pragma unroll
        for (int off = LPT; off < 64; off <<= 1) {
            l[gi] += __shfl_xor(l[gi], off, 64);
#pragma unroll
            for (int j = 0; j < 8; j++) o[gi][j] += __shfl_xor(o[gi][j], off, 64);
        }
    }
    if (lane < LPT) {
#pragma unroll
        for (int gi = 0; gi < kMaxGroup; gi++) {
            if (gi >= G) continue;
#pragma unroll
            for (int j = 0; j < 8; j++) red_o[wave][gi][dl * 8 + j] = o[gi][j];
            if (dl == 0) red_l[wave][gi] = l[gi];
        }
    }
    __syncthreads();
    const int nq = a.nq;
    if (nsplit == 1) {
        for (int idx = tid; idx < G * HD; idx += 256) {
            const int gi = idx / HD, d = idx % HD;
            const float ov = red_o[0][gi][d] + red_o[1][gi][d] + red_o[2][gi][d] + red_o[3][gi][d];
            const float lv = red_l[0][gi] + red_l[1][gi] + red_l[2][gi] + red_l[3][gi];
            a.out[m * (int64_t)nq * HD + (int64_t)(g * G + gi) * HD + d] = f2bf(ov / lv);
        }
        return;
    }
    for (int idx = tid; idx < G * HD; idx += 256) {
        const int gi = idx / HD, d = idx % HD;
        const int64_t pi = (m * nq + g * G + gi) * (int64_t)a.nsplit_max + s;
        a.part_o[pi * HD + d] = red_o[0][gi][d] + red_o[1][gi][d] + red_o[2][gi][d] + red_o[3][gi][d];
        if (d == 0) {
            a.part_ml[pi * 2] = mx[gi];
            a.part_ml[pi * 2 + 1] = red_l[0][gi] + red_l[1][gi] + red_l[2][gi] + red_l[3][gi];
        }
    }
    // ---------------- publish this split, last arriver combines (release / acquire)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* cnt = a.counters + m * a.nkv + g;
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_flag = (old == (unsigned)nsplit - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!last_flag) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int idx = tid; idx < G * HD; idx += 256) {
        const int gi = idx / HD, d = idx % HD;
        const int64_t base = (m * nq + g * G + gi) * (int64_t)a.nsplit_max;
        float mm = -INFINITY;
        for (int j = 0; j < nsplit; j++) mm = fmaxf(mm, a.part_ml[(base + j) * 2]);
        float lv = 0.f, ov = 0.f;
        for (int j = 0; j < nsplit; j++) {
            const float c = expf(a.part_ml[(base + j) * 2] - mm);
            lv += a.part_ml[(base + j) * 2 + 1] * c;
            ov += a.part_o[(base + j) * HD + d] * c;
        }
        a.out[m * (int64_t)nq * HD + (int64_t)(g * G + gi) * HD + d] = f2bf(ov / lv);
    }
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int attn_nsplit(int64_t M, int32_t max_ctx) {
    const char* e = getenv("QIE_ATTN_SPLIT_TOKENS");
    int per = e ? atoi(e) : 0;
    if (per <= 0) per = M > 8 ? 512 : 64;
    int ns = (max_ctx + per - 1) / per;
    const int cap = M > 8 ? 8 : 64;
    if (ns > cap) ns = cap;
    if (ns < 1) ns = 1;
    return ns;
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
    AttnParams a;
    a.q = (const uint16_t*)q;
    a.pos = pos;
    a.rows_per_seq = rows_per_seq;
    a.kc = (const uint16_t*)cache->k;
    a.vc = (const uint16_t*)cache->v;
    a.seq_stride = cache->seq_stride;
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
    if (cache->head_dim == 128) {
        hipLaunchKernelGGL(attn_split_kernel<128>, grid, dim3(256), 0, st, a);
        QIE_LAUNCH_CHECK();
        if (a.nsplit > 1) hipLaunchKernelGGL(attn_combine_kernel<128>, dim3(n_heads, (unsigned)M), dim3(128), 0, st, a);
    } else {
        hipLaunchKernelGGL(attn_split_kernel<64>, grid, dim3(256), 0, st, a);
        QIE_LAUNCH_CHECK();
        if (a.nsplit > 1) hipLaunchKernelGGL(attn_combine_kernel<64>, dim3(n_heads, (unsigned)M), dim3(64), 0, st, a);
    }
    QIE_LAUNCH_CHECK();
    return 0;
}

int64_t qie_attention_decode_workspace_bytes(int64_t B, int32_t n_heads, int32_t n_kv_heads, int32_t head_dim,
                                             int32_t max_ctx) {
    const int64_t ns = (max_ctx + kDecChunk - 1) / kDecChunk;
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
    a.qkv = (const uint16_t*)qkv;
    a.pos = pos;
    a.q_norm = (const uint16_t*)q_norm;
    a.k_norm = (const uint16_t*)k_norm;
    a.cs = rope_cos;
    a.sn = rope_sin;
    a.kc = (uint16_t*)cache->k;
    a.vc = (uint16_t*)cache->v;
    a.seq_stride = cache->seq_stride;
    a.layer = layer;
    a.nkv = cache->n_kv_heads;
    a.nq = n_heads;
    a.max_ctx = cache->max_ctx;
    a.nsplit_max = (cache->max_ctx + kDecChunk - 1) / kDecChunk;
    a.eps = eps;
    a.numerics = numerics;
    const int64_t cnt = ((B * a.nkv * 4 + 255) / 256) * 256;
    a.counters = (unsigned*)ws;
    a.part_o = (float*)((char*)ws + cnt);
    a.part_ml = a.part_o + B * n_heads * (int64_t)a.nsplit_max * cache->head_dim;
    a.out = (uint16_t*)out;
    dim3 grid((unsigned)(a.nkv * a.nsplit_max), (unsigned)B);
    if (cache->head_dim == 128)
        hipLaunchKernelGGL(attn_decode_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(attn_decode_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, a);
    QIE_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
