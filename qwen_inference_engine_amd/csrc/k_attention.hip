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

}  // extern "C"
