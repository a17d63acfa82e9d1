// stream_split_probe.hip — what a split-K form of the batch-1 down projection could stream at
// (DESIGN.md §13.8): the down projection's 135.8 MB (3,584 rows x 37,888 B) read as pure 16-B
// nt streams, (A) as the engine's grid does (one block of 7 waves per CU, two rows per wave,
// 14 row streams per CU), (B) with every row cut in two halves (14 waves per CU, 28 streams),
// (C) in four quarters (16 waves per CU, grid-stride, 56 streams).  Four rotating buffers
// (543 MB) keep the Infinity Cache out of it; 20 timed launches per case after 3 warm-up ones.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/stream_split_probe tools/stream_split_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

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

int main() {
    const int64_t bytes = 3584LL * 37888;   // the down projection's weights
    const int nbuf = 4;
    u32x4* buf[nbuf];
    float* out;
    for (int i = 0; i < nbuf; i++) {
        CK(hipMalloc((void**)&buf[i], bytes));
        CK(hipMemset(buf[i], 0x11 * (i + 1), bytes));
    }
    CK(hipMalloc((void**)&out, 1 << 20));
    CK(hipDeviceSynchronize());
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    struct Case { const char* name; int64_t rows; int threads; };
    const Case cases[] = {{"A: 3,584 rows x 37.9 KB, 7 waves/CU (the engine's down grid)", 3584, 448},
                          {"B: 7,168 half rows x 18.9 KB, 14 waves/CU", 7168, 896},
                          {"C: 14,336 quarter rows x 9.5 KB, 16 waves/CU, grid-stride", 14336, 1024}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Case& c : cases) {
        const int64_t row_vec = bytes / 16 / c.rows;
        auto launch = [&](int i) {
            hipLaunchKernelGGL((stream_rows<2, 8>), dim3(cus), dim3(c.threads), 0, 0, buf[i % nbuf], c.rows, row_vec, out);
        };
        for (int i = 0; i < 3; i++) launch(i);
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; i++) launch(i);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1000.0 / reps;
        printf("%-64s %8.2f us  %6.3f TB/s\n", c.name, us, bytes / us / 1e6);
    }
    return 0;
}
