// step_floor.hip — the floor of a 5-launch-per-layer decode step on this MI355X (verdict r04
// item 2): Qwen2-7B's decode step rebuilt from PURE streams at the engine's own grids and
// bytes, captured in one hipGraph as the engine captures its step (28 layers x [QKV, attention,
// O, gate/up, down] + lm_head + finalize), each launch reading its own buffer (14.3 GB in all,
// so nothing is served from the 256 MiB Infinity Cache).  Three measurements:
//   * the step of pure streams (every weight byte + ctx x 57,344 B of KV read once, each GEMV
//     as 16-B nt loads, 7-8 in flight per row, reduced to one dword per row; attention as the
//     engine's (kv head, split) blocks each streaming its 128-key K and V run);
//   * the same step with every launch EMPTY at the same grid (the launch / dependency floor);
//   * per launch kind, 28 back-to-back launches of it (in-graph average per launch).
// Engine grids (k_gemv.hip launch_gemv_t, k_attention.hip): QKV 2,304 two-row tasks on one
// block of 9 waves per CU; O 3,584 one-row tasks, 14 waves per CU; down 1,792 two-row tasks,
// 7 waves per CU; gate/up and lm_head grid-stride, 4 four-wave blocks per CU; attention
// 4 kv heads x 18 splits of 128 keys (ctx 2,304, the mid timed context), 4 waves per block.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/step_floor tools/step_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

// attention floor: block (kv head h, split s) streams keys [128 s, 128 s + 128) of K and V
// (256 B per key and head), 4 waves x 32 keys, one dword per block out
__global__ __launch_bounds__(256) void stream_kv(const u32x4* __restrict__ k, const u32x4* __restrict__ v, int ctx,
                                                 int max_ctx, int splits, float* __restrict__ out) {
    const int h = blockIdx.x / splits, s = blockIdx.x % splits, t = threadIdx.x;
    const int key0 = 128 * s;
    if (key0 >= ctx) return;
    const u32x4* kb = k + ((int64_t)h * max_ctx + key0) * 16;   // 16 x 16 B per key row
    const u32x4* vb = v + ((int64_t)h * max_ctx + key0) * 16;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) {   // 128 keys x 16 vectors = 2,048 per operand, 8 per thread
        const u32x4 x = __builtin_nontemporal_load(kb + t + 256 * i);
        const u32x4 y = __builtin_nontemporal_load(vb + t + 256 * i);
        a += __uint_as_float(x.x ^ y.y) + __uint_as_float(x.z ^ y.w);
    }
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if ((t & 63) == 0) out[blockIdx.x * 4 + (t >> 6)] = a;
}

__global__ void empty_kernel(float*) {}

struct Gemv { const char* name; int64_t rows, k; int rpw, u, grid, threads; };

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int L = 28, ctx = 2304, max_ctx = 2560, nkv = 4;
    // gate/up and lm_head grids: blocks per CU as the engine launches them (round 5: 6 and 2;
    // GU_BPC / LM_BPC override, e.g. 4 and 4 for the round-4 grids)
    const int gu_bpc = getenv("GU_BPC") ? atoi(getenv("GU_BPC")) : 6;
    const int lm_bpc = getenv("LM_BPC") ? atoi(getenv("LM_BPC")) : 2;
    const Gemv qkv{"qkv", 4608, 3584, 2, 7, cus, 576}, o{"o", 3584, 3584, 1, 7, cus, 896},
        gu{"gate_up", 37888, 3584, 2, 7, gu_bpc * cus, 256}, down{"down", 3584, 18944, 2, 7, cus, 448},
        head{"lm_head", 152064, 3584, 2, 8, lm_bpc * cus, 256};
    const Gemv* per_layer[4] = {&qkv, &o, &gu, &down};
    std::vector<u32x4*> wl[4];
    for (int j = 0; j < 4; j++)
        for (int l = 0; l < L; l++) {
            u32x4* p;
            CK(hipMalloc(&p, per_layer[j]->rows * per_layer[j]->k * 2));
            CK(hipMemset(p, 1, per_layer[j]->rows * per_layer[j]->k * 2));
            wl[j].push_back(p);
        }
    u32x4 *wh, *kc, *vc;
    CK(hipMalloc(&wh, head.rows * head.k * 2));
    CK(hipMemset(wh, 1, head.rows * head.k * 2));
    const int64_t kv_bytes = (int64_t)L * nkv * max_ctx * 256;
    CK(hipMalloc(&kc, kv_bytes));
    CK(hipMalloc(&vc, kv_bytes));
    CK(hipMemset(kc, 1, kv_bytes));
    CK(hipMemset(vc, 1, kv_bytes));
    float* out;
    CK(hipMalloc(&out, 64 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int splits = (ctx + 127) / 128, att_grid = nkv * splits;

    auto gemv = [&](const Gemv& g, const u32x4* w, bool empty) {
        if (empty) {
            hipLaunchKernelGGL(empty_kernel, dim3(g.grid), dim3(g.threads), 0, s, out);
            return;
        }
        const int64_t rv = g.k / 8;
        if (g.rpw == 1) hipLaunchKernelGGL((stream_rows<1, 7>), dim3(g.grid), dim3(g.threads), 0, s, w, g.rows, rv, out);
        else if (g.u == 8) hipLaunchKernelGGL((stream_rows<2, 8>), dim3(g.grid), dim3(g.threads), 0, s, w, g.rows, rv, out);
        else hipLaunchKernelGGL((stream_rows<2, 7>), dim3(g.grid), dim3(g.threads), 0, s, w, g.rows, rv, out);
    };
    auto attn = [&](int l, bool empty) {
        if (empty) {
            hipLaunchKernelGGL(empty_kernel, dim3(nkv * splits), dim3(256), 0, s, out);
            return;
        }
        hipLaunchKernelGGL(stream_kv, dim3(att_grid), dim3(256), 0, s, kc + (int64_t)l * nkv * max_ctx * 16,
                           vc + (int64_t)l * nkv * max_ctx * 16, ctx, max_ctx, splits, out);
    };
    auto timed = [&](auto body, int reps) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        body();
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return (double)ms / reps;
    };
    auto step = [&](bool empty) {
        for (int l = 0; l < L; l++) {
            gemv(qkv, wl[0][l], empty);
            attn(l, empty);
            gemv(o, wl[1][l], empty);
            gemv(gu, wl[2][l], empty);
            gemv(down, wl[3][l], empty);
        }
        gemv(head, wh, empty);
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, out);   // finalize
    };
    const double bytes = 14.1412e9 + (double)ctx * 57344;
    const double ms_s = timed([&] { step(false); }, 20);
    const double ms_e = timed([&] { step(true); }, 20);
    printf("step of pure streams    : %.4f ms  (%.1f tok/s, %.1f GB/s)\n", ms_s, 1e3 / ms_s, bytes / ms_s / 1e6);
    printf("step of empty launches  : %.4f ms  (%d launches: %.2f us each)\n", ms_e, 5 * L + 2,
           ms_e * 1e3 / (5 * L + 2));
    struct Kind { const char* name; int j; };
    const Kind kinds[] = {{"qkv", 0}, {"attention", -1}, {"o", 1}, {"gate_up", 2}, {"down", 3}};
    for (const Kind& k : kinds) {
        for (int empty = 0; empty < 2; empty++) {
            const double ms = timed([&] {
                for (int l = 0; l < L; l++) {
                    if (k.j < 0) attn(l, empty);
                    else gemv(*per_layer[k.j], wl[k.j][l], empty);
                }
            }, 20);
            printf("%-10s %-6s : %7.2f us per launch (28 back to back, in a graph)\n", k.name,
                   empty ? "empty" : "stream", ms * 1e3 / L);
        }
    }
    const double ms_h = timed([&] { gemv(head, wh, false); }, 50);
    printf("lm_head    stream : %7.2f us\n", ms_h * 1e3);
    return 0;
}
