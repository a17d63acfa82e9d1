// k_sampling.hip — greedy arg-max and top-k / temperature / top-p sampling.
//
// Replaces topk_temperature_softmax_sampling_kernel_bf16 + blockArgMax/better
// (layers/src/logit_decode.cu:15-33, 149-274) and sample_topk_bf16
// (helpers.cuh:157-166).  The reference runs ONE 256-thread block that makes k
// full sweeps over V with an O(k) membership scan per element.  Here:
//   * every logit maps to a 64-bit selection key whose order IS the reference's
//     selection order (value, then bitrev8(idx mod 256), then -idx; see
//     qie_common.hpp sel_key) — greedy is a parallel max over keys (also fused
//     into the lm_head GEMV epilogue, k_gemv.hip);
//   * top-k = per-4096-slice bitonic sort (LDS) + a merge sort of the slice
//     winners; the sorted keys reproduce the reference's k rounds exactly;
//   * softmax + draw on one lane with the reference's sequential order and a
//     cuRAND-XORWOW restatement (curand_init(seed, 0, 0); curand_uniform).
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

namespace qie {

constexpr int kSlice = 4096;
constexpr int kMaxTopK = 256;

__global__ __launch_bounds__(256) void argmax_keys_kernel(const uint16_t* __restrict__ logits,
                                                          int64_t V, int64_t ld,
                                                          unsigned long long* keys) {
    __shared__ unsigned long long red[4];
    const int64_t m = blockIdx.y;
    const uint16_t* row = logits + m * ld;
    unsigned long long best = 0ull;
    const int64_t per = (V + gridDim.x - 1) / gridDim.x;
    const int64_t lo = blockIdx.x * per, hi = min(V, lo + per);
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        unsigned long long k = sel_key(bf2f(row[i]), (uint32_t)i);
        best = k > best ? k : best;
    }
    best = wave_max(best);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = red[0];
        for (int w = 1; w < 4; w++) b = red[w] > b ? red[w] : b;
        if (b) atomicMax(keys + m, b);
    }
}

__global__ void keys_to_ids_kernel(const unsigned long long* keys, int64_t M, int32_t* ids) {
    const int64_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m < M) ids[m] = key_idx(keys[m]);
}

// Bitonic sort, descending, of n (power of two) keys in LDS.
__device__ void bitonic_desc(unsigned long long* k, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int j = threadIdx.x; j < n / 2; j += blockDim.x) {
                const int i = (j / stride) * 2 * stride + (j % stride);
                const int q = i + stride;
                const bool desc = (i & size) == 0;
                unsigned long long a = k[i], b = k[q];
                if (desc ? (a < b) : (a > b)) {
                    k[i] = b;
                    k[q] = a;
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void topk_slice_kernel(const uint16_t* __restrict__ logits, int64_t V,
                                                         int64_t ld, int k,
                                                         unsigned long long* __restrict__ cand) {
    __shared__ unsigned long long keys[kSlice];
    const int64_t m = blockIdx.y;
    const int64_t base = (int64_t)blockIdx.x * kSlice;
    const uint16_t* row = logits + m * ld;
    for (int i = threadIdx.x; i < kSlice; i += 256) {
        const int64_t idx = base + i;
        keys[i] = idx < V ? sel_key(bf2f(row[idx]), (uint32_t)idx) : 0ull;
    }
    __syncthreads();
    bitonic_desc(keys, kSlice);
    unsigned long long* out = cand + (m * gridDim.x + blockIdx.x) * (int64_t)k;
    for (int i = threadIdx.x; i < k; i += 256) out[i] = keys[i];
}

// cuRAND XORWOW, curand_init(seed, subsequence = 0, offset = 0) (no skip-ahead)
// and curand_uniform — restated from the published curand_kernel.h.
__device__ __forceinline__ float xorwow_uniform_first(uint64_t seed) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    uint32_t d = 6615241u + t1 + t0;
    uint32_t v0 = 123456789u + t0, v4 = 5783321u + t0;
    uint32_t t = v0 ^ (v0 >> 2);
    uint32_t nv4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
    d += 362437u;
    uint32_t x = nv4 + d;
    return x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

__global__ __launch_bounds__(256) void topk_merge_sample_kernel(const unsigned long long* __restrict__ cand,
                                                                int nb, int k, int n2, float temperature,
                                                                float top_p, uint64_t seed,
                                                                const int32_t* step, int32_t* ids) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned long long sk[];
    const int64_t m = blockIdx.x;
    const int total = nb * k;
    for (int i = threadIdx.x; i < n2; i += 256) sk[i] = i < total ? cand[m * total + i] : 0ull;
    __syncthreads();
    bitonic_desc(sk, n2);
    if (threadIdx.x != 0) return;
    // logit_decode.cu:225-272 (thread 0): temperature, softmax, one draw.
    int n = 0;
    while (n < k && sk[n] != 0ull) n++;
    if (n == 0) { ids[m] = -1; return; }
    float vals[kMaxTopK];
    float T = temperature > 0.0f ? temperature : 1.0f;
    float max_val = key_val(sk[0]) / T;
    for (int i = 1; i < n; i++) {
        float v = key_val(sk[i]) / T;
        if (v > max_val) max_val = v;
        vals[i] = v;
    }
    vals[0] = key_val(sk[0]) / T;
    float sum = 0.0f;
    for (int i = 0; i < n; i++) {
        vals[i] = expf(vals[i] - max_val);
        sum += vals[i];
    }
    if (top_p > 0.0f && top_p < 1.0f) {
        float cum = 0.0f;
        int keep = n;
        for (int i = 0; i < n; i++) {
            cum += vals[i];
            if (cum >= top_p * sum) { keep = i + 1; break; }
        }
        n = keep;
        sum = 0.0f;
        for (int i = 0; i < n; i++) sum += vals[i];
    }
    const uint64_t sd = seed + (step ? (uint64_t)(int64_t)step[m] : 0ull);
    float u = xorwow_uniform_first(sd) * sum;
    float cum = 0.0f;
    int picked = key_idx(sk[n - 1]);
    for (int i = 0; i < n; i++) {
        cum += vals[i];
        if (u <= cum) { picked = key_idx(sk[i]); break; }
    }
    ids[m] = picked;
}

static int pow2_at_least(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace qie

using namespace qie;

extern "C" {

int64_t qie_sample_workspace_bytes(int64_t M, int64_t V) {
    const int64_t nb = (V + kSlice - 1) / kSlice;
    return M * nb * kMaxTopK * 8 + M * 8 + 64;
}

int qie_keys_to_ids(const uint64_t* keys, int64_t M, int32_t* out_ids, void* stream) {
    QIE_REQUIRE(keys && out_ids && M >= 0, "qie_keys_to_ids: bad arguments");
    if (M == 0) return 0;
    hipLaunchKernelGGL(keys_to_ids_kernel, dim3((unsigned)((M + 63) / 64)), dim3(64), 0,
                       (hipStream_t)stream, (const unsigned long long*)keys, M, out_ids);
    QIE_LAUNCH_CHECK();
    return 0;
}

int qie_sample(const void* logits, int64_t M, int64_t V, int64_t ld, const qie_sampling* s,
               const int32_t* step_dev, int32_t* out_ids, void* ws, void* stream) {
    QIE_REQUIRE(logits && s && out_ids && ws && M >= 0 && V > 0 && V < (1 << 24) && ld >= V,
                "qie_sample: bad arguments");
    if (M == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (s->top_k <= 1) {
        unsigned long long* keys = (unsigned long long*)ws;
        QIE_HIP(hipMemsetAsync(keys, 0, M * 8, st));
        hipLaunchKernelGGL(argmax_keys_kernel, dim3(64, (unsigned)M), dim3(256), 0, st,
                           (const uint16_t*)logits, V, ld, keys);
        QIE_LAUNCH_CHECK();
        return qie_keys_to_ids((const uint64_t*)keys, M, out_ids, stream);
    }
    int k = s->top_k;
    if (k > V) k = (int)V;
    if (k > kMaxTopK) k = kMaxTopK;
    const int nb = (int)((V + kSlice - 1) / kSlice);
    unsigned long long* cand = (unsigned long long*)ws;
    hipLaunchKernelGGL(topk_slice_kernel, dim3(nb, (unsigned)M), dim3(256), 0, st,
                       (const uint16_t*)logits, V, ld, k, cand);
    QIE_LAUNCH_CHECK();
    const int n2 = pow2_at_least(nb * k);
    const size_t shm = (size_t)n2 * 8;
    QIE_REQUIRE(shm <= 160 * 1024, "qie_sample: top-k merge exceeds LDS (V=%lld k=%d)", (long long)V, k);
    if (shm > 65536) {
        static bool raised = false;
        if (!raised) {
            QIE_HIP(hipFuncSetAttribute((const void*)topk_merge_sample_kernel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            raised = true;
        }
    }
    hipLaunchKernelGGL(topk_merge_sample_kernel, dim3((unsigned)M), dim3(256), shm, st, cand, nb, k, n2,
                       s->temperature, s->top_p, (uint64_t)s->seed, step_dev, out_ids);
    QIE_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
