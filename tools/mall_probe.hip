// mall_probe.hip — does a weight stream that was touched shortly before (so it sits in the
// 256 MiB Infinity Cache) read faster than a cold one, at the decode GEMVs' sizes?
// Per rep: [prefetch kernel reads the first X % of buffer i] -> event -> [stream kernel reads
// all of buffer i] -> event.  The buffers form a ring > 600 MB, so without the prefetch every
// read is cold.  Prints the stream kernel's avg time per X and prefetch policy.
//   hipcc --offload-arch=gfx950 -O3 -o mall_probe tools/mall_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int RPW, int U>
__global__ __launch_bounds__(1024) void stream_rows(const u32x4* __restrict__ w, int64_t rows, int64_t row_vec,
                                                     float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (int64_t r0 = wid * RPW; r0 < rows; r0 += nw * RPW) {
        float acc[RPW];
#pragma unroll
        for (int i = 0; i < RPW; i++) acc[i] = 0.f;
        for (int64_t k0 = lane; k0 < row_vec; k0 += 64 * U) {
            u32x4 v[U][RPW];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int i = 0; i < RPW; i++) {
                    const int64_t k = k0 + u * 64 < row_vec ? k0 + u * 64 : row_vec - 1;
                    const int64_t r = r0 + i < rows ? r0 + i : rows - 1;
                    v[u][i] = __builtin_nontemporal_load(w + r * row_vec + k);
                }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int i = 0; i < RPW; i++)
                    acc[i] += __uint_as_float(v[u][i].x ^ v[u][i].y) + __uint_as_float(v[u][i].z ^ v[u][i].w);
        }
#pragma unroll
        for (int i = 0; i < RPW; i++) {
            float a = acc[i];
            for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
            if (lane == 0 && r0 + i < rows) out[r0 + i] = a;
        }
    }
}

// touch n16 16-B vectors: each lane loads 8 in flight, xor-folds, one store per wave
template <bool NT>
__global__ __launch_bounds__(256) void touch(const u32x4* __restrict__ w, int64_t n16, unsigned* __restrict__ sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += 8 * stride) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t j = i + u * stride < n16 ? i + u * stride : n16 - 1;
            v[u] = NT ? __builtin_nontemporal_load(w + j) : w[j];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;   // practically never: keeps the loads
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct Shape { const char* name; int64_t rows, k; };
    const Shape shapes[] = {{"o(3584x3584)", 3584, 3584}, {"qkv(4608x3584)", 4608, 3584},
                            {"down(3584x18944)", 3584, 18944}, {"gate_up(37888x3584)", 37888, 3584}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float* out;
    unsigned* sink;
    CK(hipMalloc(&out, 64 << 20));
    CK(hipMalloc(&sink, 4096));
    const int reps = 24;
    std::vector<hipEvent_t> ev(2 * reps + 2);
    for (size_t i = 0; i < ev.size(); i++) CK(hipEventCreate(&ev[i]));
    for (const Shape& sh : shapes) {
        const int64_t bytes = sh.rows * sh.k * 2;
        const int nbuf = (int)std::max<int64_t>(2, (600ll << 20) / bytes + 1);
        std::vector<u32x4*> bufs(nbuf);
        for (auto& b : bufs) {
            CK(hipMalloc(&b, bytes));
            CK(hipMemset(b, 1, bytes));
        }
        const int64_t rv = sh.k / 8;
        const int64_t tasks = sh.rows / 2;
        int64_t nw = std::min<int64_t>(16, (tasks + cus - 1) / cus);
        const int threads = (int)(64 * nw), grid = (int)std::min<int64_t>(cus, (tasks + nw - 1) / nw);
        const int pcts[] = {0, 25, 50, 100};
        for (int pol = 0; pol < 2; pol++)
            for (int pct : pcts) {
                if (pol == 1 && pct == 0) continue;
                const int64_t n16 = bytes / 16 * pct / 100;
                double sum_s = 0, sum_p = 0;
                for (int it = 0; it < 2; it++) {   // first pass warms up
                    for (int i = 0; i < reps; i++) {
                        const u32x4* b = bufs[i % nbuf];
                        CK(hipEventRecord(ev[2 * i], s));
                        if (n16) {
                            if (pol == 0) hipLaunchKernelGGL(touch<false>, dim3(cus * 4), dim3(256), 0, s, b, n16, sink);
                            else hipLaunchKernelGGL(touch<true>, dim3(cus * 4), dim3(256), 0, s, b, n16, sink);
                        }
                        CK(hipEventRecord(ev[2 * i + 1], s));
                        hipLaunchKernelGGL((stream_rows<2, 7>), dim3(grid), dim3(threads), 0, s, b, sh.rows, rv, out);
                        CK(hipEventRecord(ev[2 * reps + (i & 1)], s));
                        CK(hipEventSynchronize(ev[2 * reps + (i & 1)]));
                        float ms_p = 0, ms_s = 0;
                        CK(hipEventElapsedTime(&ms_p, ev[2 * i], ev[2 * i + 1]));
                        CK(hipEventElapsedTime(&ms_s, ev[2 * i + 1], ev[2 * reps + (i & 1)]));
                        if (it == 1) { sum_s += ms_s; sum_p += ms_p; }
                    }
                }
                const double us = sum_s * 1e3 / reps, usp = sum_p * 1e3 / reps;
                printf("%-22s prefetch %3d%% %-7s  touch %8.2f us  stream %8.2f us  %7.1f GB/s\n", sh.name, pct,
                       pol ? "nt" : "default", usp, us, bytes / us / 1e3);
                fflush(stdout);
            }
        for (auto& b : bufs) CK(hipFree(b));
    }
    return 0;
}
