// stream_probe.hip — what a pure weight stream costs on this MI355X, per launch, at the
// decode GEMVs' sizes (Qwen2-7B: O 25.7 MB, QKV 33.0 MB, down 135.8 MB, gate/up 271.6 MB),
// as the decode step runs it: back-to-back dependent launches on one stream, each reading
// a different buffer (a ring of buffers > 256 MiB so the Infinity Cache holds none of it).
// Every wave streams whole rows with 16-B loads, U loads in flight per row, RPW rows per
// wave, and reduces them (one dword stored per row) — the GEMV's memory shape without the
// arithmetic.  Variants: load policy (default / nt), rows per wave, loads in flight per row,
// waves per block, row length.  Prints one line per variant: avg us per launch and GB/s.
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int RPW, int U, bool NT>
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
                    const u32x4* p = w + r * row_vec + k;
                    v[u][i] = NT ? __builtin_nontemporal_load(p) : *p;
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

struct Variant { const char* name; int rpw, u; bool nt; int waves; int bpc; };

template <int RPW, int U, bool NT>
static void launch(int grid, int threads, const u32x4* w, int64_t rows, int64_t rv, float* out, hipStream_t s) {
    hipLaunchKernelGGL((stream_rows<RPW, U, NT>), dim3(grid), dim3(threads), 0, s, w, rows, rv, out);
}

static void dispatch(const Variant& v, int grid, int threads, const u32x4* w, int64_t rows, int64_t rv, float* out,
                     hipStream_t s) {
#define V(R, U_, N) if (v.rpw == R && v.u == U_ && v.nt == N) return launch<R, U_, N>(grid, threads, w, rows, rv, out, s);
    V(2, 7, true) V(2, 8, true) V(2, 7, false) V(2, 4, true) V(4, 4, true) V(1, 8, true) V(1, 16, true) V(2, 16, true)
    V(4, 8, true) V(1, 4, true)
#undef V
    printf("no instantiation\n");
    exit(1);
}

int main(int argc, char** argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct Shape { const char* name; int64_t rows, k; };
    const Shape shapes[] = {{"o(3584x3584)", 3584, 3584}, {"qkv(4608x3584)", 4608, 3584},
                            {"down(3584x18944)", 3584, 18944}, {"gate_up(37888x3584)", 37888, 3584}};
    const Variant vars[] = {
        {"rpw2 u7 nt, 1 blk/CU", 2, 7, true, 0, 1}, {"rpw2 u7 nt, grid-stride 4 waves x 4/CU", 2, 7, true, 4, 4},
        {"rpw2 u7 default", 2, 7, false, 0, 1},     {"rpw2 u8 nt, 1 blk/CU", 2, 8, true, 0, 1},
        {"rpw1 u8 nt, 1 blk/CU", 1, 8, true, 0, 1}, {"rpw1 u16 nt, 1 blk/CU", 1, 16, true, 0, 1},
        {"rpw2 u16 nt, 1 blk/CU", 2, 16, true, 0, 1}, {"rpw4 u4 nt, 1 blk/CU", 4, 4, true, 0, 1},
        {"rpw2 u4 nt, 1 blk/CU", 2, 4, true, 0, 1},  {"rpw2 u8 nt, 8 waves x 4/CU", 2, 8, true, 8, 4},
        {"rpw1 u8 nt, 16 waves x 2/CU", 1, 8, true, 16, 2}, {"rpw4 u8 nt, 1 blk/CU", 4, 8, true, 0, 1},
        {"rpw1 u4 nt, 16 waves x 2/CU", 1, 4, true, 16, 2},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float* out;
    CK(hipMalloc(&out, 64 << 20));
    for (const Shape& sh : shapes) {
        const int64_t bytes = sh.rows * sh.k * 2;
        const int nbuf = (int)std::max<int64_t>(2, (600ll << 20) / bytes + 1);   // ring > 256 MiB
        std::vector<u32x4*> bufs(nbuf);
        for (auto& b : bufs) {
            CK(hipMalloc(&b, bytes));
            CK(hipMemset(b, 1, bytes));
        }
        const int64_t rv = sh.k / 8;
        for (const Variant& v : vars) {
            const int64_t tasks = (sh.rows + v.rpw - 1) / v.rpw;
            int threads, grid;
            if (v.waves == 0) {   // one block per CU, ceil(tasks / CUs) waves (the engine's mid-size grid)
                int64_t nw = (tasks + cus - 1) / cus;
                if (nw > 16) nw = 16;
                threads = (int)(64 * nw);
                grid = (int)std::min<int64_t>(cus, (tasks + nw - 1) / nw);
            } else {
                threads = 64 * v.waves;
                grid = (int)std::min<int64_t>((int64_t)cus * v.bpc, (tasks + v.waves - 1) / v.waves);
            }
            const int reps = 60;   // captured in a hipGraph, replayed (as the decode step runs)
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < reps; i++) dispatch(v, grid, threads, bufs[i % nbuf], sh.rows, rv, out, s);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
            printf("%-22s %-40s grid %5d x %4d  %8.2f us  %7.1f GB/s\n", sh.name, v.name, grid, threads, us,
                   bytes / us / 1e3);
            fflush(stdout);
        }
        for (auto& b : bufs) CK(hipFree(b));
    }
    // empty-kernel chain: the per-launch floor on this stream
    {
        const int reps = 200;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < reps; i++) launch<2, 7, true>(256, 576, nullptr, 0, 448, out, s);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-22s %-40s grid %5d x %4d  %8.2f us\n", "empty", "rows=0", 256, 576, ms * 1e3 / reps);
    }
    return 0;
}
