// comm.hip — tensor-parallel collectives (qie_comm_* of qie_engine.h).
//
// The engine shards Megatron-style: QKV and gate/up column-parallel,
// O and down row-parallel, lm_head vocab-parallel.  Per decode layer that needs two
// all-reduces of the fp32 [B, H] partial sums (after O and after down), and per step
// one max-all-reduce of the u64 arg-max keys (greedy) or an all-gather of the logit
// shards (sampling).  RCCL is called from here, on the engine stream — never through
// torch.distributed, whose wheel brings a second HIP runtime into the process.
#include "qie_common.hpp"
#include "qie_comm.hpp"
#include "../../include/qie/qie_engine.h"
#include "../../include/qie/qie_ops.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <type_traits>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace qie {

#define QIE_NCCL(expr)                                                                  \
    do {                                                                                \
        ncclResult_t _r = (expr);                                                       \
        if (_r != ncclSuccess)                                                          \
            return ::qie::fail(-100 - (int)_r, "%s:%d %s -> %s", __FILE__, __LINE__, #expr, \
                               ncclGetErrorString(_r));                                 \
    } while (0)

#define QIE_TRY_C(expr)           \
    do {                          \
        int _rc = (expr);         \
        if (_rc != 0) return _rc; \
    } while (0)

struct RcclComm : qie_comm {
    ncclComm_t c = nullptr;
    ~RcclComm() override {
        if (c) ncclCommDestroy(c);
    }
    int allreduce_sum_f32(float* buf, int64_t n, hipStream_t st) override {
        QIE_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c, st));
        return 0;
    }
    int allreduce_max_u64(uint64_t* buf, int64_t n, hipStream_t st) override {
        QIE_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclUint64, ncclMax, c, st));
        return 0;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st) override {
        QIE_NCCL(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c, st));
        return 0;
    }
    bool graph_capturable() const override { return true; }
};

// ------------------------------------------------------------- local backend
constexpr int kLocalMaxWorld = 8;
struct PtrSet {
    const void* p[kLocalMaxWorld];
};

__global__ void local_sum_f32_kernel(PtrSet in, int world, float* out, int64_t n) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float s = reinterpret_cast<const float*>(in.p[0])[i];
        for (int r = 1; r < world; r++) s += reinterpret_cast<const float*>(in.p[r])[i];
        out[i] = s;
    }
}

__global__ void local_max_u64_kernel(PtrSet in, int world, uint64_t* out, int64_t n) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        uint64_t s = reinterpret_cast<const uint64_t*>(in.p[0])[i];
        for (int r = 1; r < world; r++) {
            const uint64_t v = reinterpret_cast<const uint64_t*>(in.p[r])[i];
            s = v > s ? v : s;
        }
        out[i] = s;
    }
}

struct LocalGroup {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t gen = 0;
    std::vector<const void*> ptr;
    std::vector<hipEvent_t> ready, done;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const int64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
    ~LocalGroup() {
        for (auto e : ready) hipEventDestroy(e);
        for (auto e : done) hipEventDestroy(e);
    }
};

struct LocalComm : qie_comm {
    std::shared_ptr<LocalGroup> g;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    ~LocalComm() override {
        if (tmp) hipFree(tmp);
    }
    int ensure_tmp(size_t bytes) {
        if (bytes <= tmp_bytes) return 0;
        if (tmp) hipFree(tmp);
        tmp = nullptr;
        tmp_bytes = 0;
        QIE_HIP(hipMalloc(&tmp, bytes));
        tmp_bytes = bytes;
        return 0;
    }
    // publish `p` (ready on st), wait for every rank's, run body, then hold every
    // rank until all have consumed the published buffers
    template <class Body>
    int exchange(const void* p, hipStream_t st, Body body) {
        g->ptr[rank] = p;
        QIE_HIP(hipEventRecord(g->ready[rank], st));
        g->barrier();
        for (int r = 0; r < world; r++)
            if (r != rank) QIE_HIP(hipStreamWaitEvent(st, g->ready[r], 0));
        PtrSet ps{};
        for (int r = 0; r < world; r++) ps.p[r] = g->ptr[r];
        int rc = body(ps);
        QIE_HIP(hipEventRecord(g->done[rank], st));
        g->barrier();
        for (int r = 0; r < world; r++)
            if (r != rank) QIE_HIP(hipStreamWaitEvent(st, g->done[r], 0));
        return rc;
    }
    int allreduce_sum_f32(float* buf, int64_t n, hipStream_t st) override {
        QIE_TRY_C(ensure_tmp((size_t)n * 4));
        QIE_TRY_C(exchange(buf, st, [&](const PtrSet& ps) -> int {
            const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
            hipLaunchKernelGGL(local_sum_f32_kernel, dim3(grid), dim3(256), 0, st, ps, world, (float*)tmp, n);
            QIE_LAUNCH_CHECK();
            return 0;
        }));
        QIE_HIP(hipMemcpyAsync(buf, tmp, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    int allreduce_max_u64(uint64_t* buf, int64_t n, hipStream_t st) override {
        QIE_TRY_C(ensure_tmp((size_t)n * 8));
        QIE_TRY_C(exchange(buf, st, [&](const PtrSet& ps) -> int {
            const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
            hipLaunchKernelGGL(local_max_u64_kernel, dim3(grid), dim3(256), 0, st, ps, world, (uint64_t*)tmp, n);
            QIE_LAUNCH_CHECK();
            return 0;
        }));
        QIE_HIP(hipMemcpyAsync(buf, tmp, (size_t)n * 8, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st) override {
        return exchange(send, st, [&](const PtrSet& ps) -> int {
            for (int r = 0; r < world; r++)
                QIE_HIP(hipMemcpyAsync((char*)recv + (int64_t)r * bytes, ps.p[r], (size_t)bytes,
                                       hipMemcpyDeviceToDevice, st));
            return 0;
        });
    }
    bool graph_capturable() const override { return false; }
};

// ------------------------------------------------------------- peer backend
// One-shot exchange through every rank's buffer mapped into every other rank (HIP IPC across
// processes; plain pointers for ranks of one process): each collective is ONE kernel that
// pushes this rank's slice into slot [parity][rank] of EVERY rank's buffer, raises a
// per-block flag (the generation) in every buffer, waits for the W flags of its block in its
// own buffer, and reduces the W slots in rank order 0..W-1 (the local backend's order: the
// results are bit-identical to it).  The all-reduce after the row-parallel projections
// fuses the residual add, x = bf16(x + bf16(sum)) (qie_residual_add_f32), so a layer's
// exchange is one graph node instead of RCCL's collective + a residual launch.
//   * buffers are uncached device memory (hipDeviceMallocUncached): another device's stores
//     and this device's loads meet in memory, never in a stale L2 line;
//   * generation e lives in device memory (graph replays advance it): every block reads it
//     first, the last block to finish (ticket) stores e + 1; data and flags alternate
//     between two parities, and a rank can only reach generation e + 2 after every peer
//     raised its e + 1 flags, i.e. after every peer finished reading generation e;
//   * the wait is bounded (~10 s of s_memrealtime): a peer that never arrives sets the error
//     word and the kernel ends without storing a result or advancing the generation (no
//     hang, no silently wrong residual); the communicator is then poisoned (every later
//     exchange returns at once) and the engine fails its next synchronising call
//     (qie_decode / qie_decode_step / prefill with ids / logits); qie_comm_peer_error()
//     reads the word directly.  Every rank's
//     collective must be able to run while another waits: one process per GPU, or (ranks of
//     one process on one device) at most 2 ranks — a process gets 4 hardware queues, and two
//     ranks' streams sharing one queue would serialise a waiting kernel before its peer.
constexpr int kPeerMaxWorld = 8;
constexpr int kPeerBlocks = 16;
constexpr int64_t kPeerFlagBytes = 4096;             // [2][8][16] uint32 flags, padded
constexpr int64_t kPeerCap = 2 << 20;                // data bytes per (parity, rank) slot
// the tagged slots (peer_tag_kernel) follow the flagged ones: [2][8] x kPeerTagCap bytes
constexpr int64_t kPeerTagOff = kPeerFlagBytes + 2 * kPeerMaxWorld * kPeerCap;
static_assert(kPeerMaxWorld == kPeerTagMaxWorld, "tagged slots cover every rank");

struct PeerArgs {
    char* buf[kPeerMaxWorld];   // every rank's exchange buffer (this rank's own included)
    int world, rank;
    unsigned* ctl;              // this rank's [0] generation, [1] ticket, [2] error
};

enum { kPeerSumF32 = 0, kPeerSumResid = 1, kPeerMaxU64 = 2, kPeerGather = 3, kPeerGatherB = 4 };

__device__ __forceinline__ unsigned* peer_flag(char* b, int par, int src, int blk) {
    return reinterpret_cast<unsigned*>(b) + (par * kPeerMaxWorld + src) * kPeerBlocks + blk;
}
__device__ __forceinline__ char* peer_slot(char* b, int par, int src) {
    return b + kPeerFlagBytes + (int64_t)(par * kPeerMaxWorld + src) * kPeerCap;
}

// n elements of 4 (f32 / gather words) or 8 (u64) bytes; dst: f32 sum, u64 max, gathered
// words [world][n], or (kPeerSumResid) the bf16 residual stream x updated in place
template <int OP>
__global__ __launch_bounds__(256) void peer_kernel(PeerArgs A, const void* src, void* dst, int64_t n) {
    using T = typename std::conditional<OP == kPeerMaxU64, uint64_t,
                                        typename std::conditional<OP == kPeerGatherB, uint8_t, uint32_t>::type>::type;
    __shared__ unsigned e_s, err_s;
    const int blk = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) {
        e_s = __hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        err_s = __hip_atomic_load(A.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // a communicator whose exchange once timed out is poisoned: the ranks are out of step
    // (this rank's generation moved on without the late one), so later exchanges neither
    // push, wait nor store; the engine reports the error word at its next sync point
    if (err_s) return;
    const unsigned e = e_s;
    const int par = e & 1;
    // this block's slice (resid: whole groups of 8 so the bf16 row is read in 16-B pieces)
    const int64_t gran = OP == kPeerSumResid ? 8 : 1;
    const int64_t ng = (n + gran - 1) / gran;
    const int64_t i0 = (ng * blk / kPeerBlocks) * gran, i1 = (ng * (blk + 1) / kPeerBlocks) * gran;
    const int64_t e1 = i1 < n ? i1 : n;
    const T* in = reinterpret_cast<const T*>(src);
    for (int q = 0; q < A.world; q++) {
        T* slot = reinterpret_cast<T*>(peer_slot(A.buf[q], par, A.rank));
        for (int64_t i = i0 + tid; i < e1; i += 256) slot[i] = in[i];
    }
    __threadfence_system();
    __syncthreads();
    if (tid < A.world)
        __hip_atomic_store(peer_flag(A.buf[tid], par, A.rank, blk), e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid < A.world) {   // wait for rank tid's push of this block's slice
        const unsigned* f = peer_flag(A.buf[A.rank], par, tid, blk);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != e + 1) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {   // ~10 s at 100 MHz
                __hip_atomic_store(A.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                err_s = 1;
                break;
            }
        }
    }
    __syncthreads();
    // timed out: the slots may hold a stale generation — store nothing, and never take the
    // ticket, so the generation does not advance past the late rank
    if (err_s) return;
    __threadfence_system();
    char* mine = A.buf[A.rank];
    if constexpr (OP == kPeerGather || OP == kPeerGatherB) {
        for (int q = 0; q < A.world; q++) {
            const T* sl = reinterpret_cast<const T*>(peer_slot(mine, par, q));
            T* out = reinterpret_cast<T*>(dst) + (int64_t)q * n;
            for (int64_t i = i0 + tid; i < e1; i += 256) out[i] = sl[i];
        }
    } else if constexpr (OP == kPeerSumResid) {
        uint16_t* x = reinterpret_cast<uint16_t*>(dst);
        for (int64_t i = i0 + tid; i < e1; i += 256) {
            float s = reinterpret_cast<const float*>(peer_slot(mine, par, 0))[i];
            for (int q = 1; q < A.world; q++) s += reinterpret_cast<const float*>(peer_slot(mine, par, q))[i];
            x[i] = f2bf(bf2f(x[i]) + rbf(s));
        }
    } else {
        for (int64_t i = i0 + tid; i < e1; i += 256) {
            if constexpr (OP == kPeerSumF32) {
                float s = reinterpret_cast<const float*>(peer_slot(mine, par, 0))[i];
                for (int q = 1; q < A.world; q++) s += reinterpret_cast<const float*>(peer_slot(mine, par, q))[i];
                reinterpret_cast<float*>(dst)[i] = s;
            } else {
                uint64_t s = reinterpret_cast<const uint64_t*>(peer_slot(mine, par, 0))[i];
                for (int q = 1; q < A.world; q++) {
                    const uint64_t v = reinterpret_cast<const uint64_t*>(peer_slot(mine, par, q))[i];
                    s = v > s ? v : s;
                }
                reinterpret_cast<uint64_t*>(dst)[i] = s;
            }
        }
    }
    __syncthreads();
    if (tid == 0) {   // the last block of this generation advances it
        const unsigned old = __hip_atomic_fetch_add(A.ctl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == kPeerBlocks - 1) {
            __hip_atomic_store(A.ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(A.ctl, e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Exchange buffers are uncached device memory.  A freed one goes to a process-wide pool and is
// handed to the next communicator instead of back to the allocator: physical pages that were
// mapped uncached are never recycled into ordinary (cached) allocations of the process — a
// weight arena placed on them after the peer tests read back 40 whole 128-B lines of a
// freshly written tensor as stale zeros (test_tp_weights_bin_equals_synthetic, r06).
static std::mutex g_peer_pool_mu;
static std::vector<char*> g_peer_pool;
static char* peer_pool_get() {
    std::lock_guard<std::mutex> lk(g_peer_pool_mu);
    if (g_peer_pool.empty()) return nullptr;
    char* p = g_peer_pool.back();
    g_peer_pool.pop_back();
    return p;
}
static void peer_pool_put(char* p) {
    std::lock_guard<std::mutex> lk(g_peer_pool_mu);
    g_peer_pool.push_back(p);
}

// Tagged row-parallel exchange (decode sizes, n <= kPeerTagCap / 8): x = bf16(x + bf16(sum of
// the W partials)), the same rank-ordered sum as kPeerSumResid, bit for bit.  Each partial is
// written as 8-byte words {e + 1, f32} by relaxed SYSTEM-scope atomic stores (write-through to
// the owner's uncached buffer, single-copy atomic), and the reader polls the words themselves:
// no system fence before a flag, no flag round trip, no fence after it.  PUSHED: the producer
// GEMV already wrote this rank's words from its epilogue (set_gemv_push), so the kernel only
// waits, reduces and advances the generation.  A word of generation e - 2 (the other value
// the slot can hold: parity reuse, as above) carries tag e - 1, never e + 1.
template <bool PUSHED>
__global__ __launch_bounds__(256) void peer_tag_kernel(PeerArgs A, const float* part, uint16_t* x, int64_t n) {
    __shared__ unsigned e_s, err_s;
    const int blk = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) {
        e_s = __hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        err_s = __hip_atomic_load(A.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (err_s) return;   // poisoned communicator (see peer_kernel)
    const unsigned e = e_s;
    const uint64_t tag = (uint64_t)(e + 1);
    const int64_t i0 = n * blk / gridDim.x, i1 = n * (blk + 1) / gridDim.x;
    if constexpr (!PUSHED) {
        for (int64_t i = i0 + tid; i < i1; i += 256) {
            const uint64_t w = tag | ((uint64_t)__float_as_uint(part[i]) << 32);
#pragma unroll
            for (int q = 0; q < kPeerTagMaxWorld; q++)
                if (q < A.world)
                    __hip_atomic_store(peer_tag_slot(A.buf[q] + kPeerTagOff, e, A.rank) + i, w, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    char* mine = A.buf[A.rank] + kPeerTagOff;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool late = false;
    for (int64_t i = i0 + tid; i < i1 && !late; i += 256) {
        uint64_t w[kPeerTagMaxWorld];
#pragma unroll
        for (int q = 0; q < kPeerTagMaxWorld; q++)
            w[q] = q < A.world ? __hip_atomic_load(peer_tag_slot(mine, e, q) + i, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM)
                               : tag;
        for (;;) {
            bool ready = true;
#pragma unroll
            for (int q = 0; q < kPeerTagMaxWorld; q++) ready &= (uint32_t)w[q] == (uint32_t)tag;
            if (ready) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {   // ~10 s at 100 MHz
                late = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int q = 0; q < kPeerTagMaxWorld; q++)
                if ((uint32_t)w[q] != (uint32_t)tag)
                    w[q] = __hip_atomic_load(peer_tag_slot(mine, e, q) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (late) break;
        float s = __uint_as_float((uint32_t)(w[0] >> 32));
#pragma unroll
        for (int q = 1; q < kPeerTagMaxWorld; q++)
            if (q < A.world) s += __uint_as_float((uint32_t)(w[q] >> 32));
        x[i] = f2bf(bf2f(x[i]) + rbf(s));
    }
    if (late) {
        __hip_atomic_store(A.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        err_s = 1;
    }
    __syncthreads();
    // timed out: x may be partly updated (the communicator is poisoned and the engine fails
    // its next synchronising call); the generation does not advance past the late rank
    if (err_s) return;
    if (tid == 0) {   // the last block of this generation advances it
        const unsigned old = __hip_atomic_fetch_add(A.ctl + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(A.ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(A.ctl, e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

struct PeerComm : qie_comm {
    char* own = nullptr;          // this rank's exchange buffer (uncached)
    unsigned* ctl = nullptr;      // generation, ticket, error
    char* peer[kPeerMaxWorld] = {};
    bool opened[kPeerMaxWorld] = {};   // IPC-mapped (closed on destroy)
    float* tmp = nullptr;
    size_t tmp_bytes = 0;
    ~PeerComm() override {
        for (int r = 0; r < kPeerMaxWorld; r++)
            if (opened[r] && peer[r]) hipIpcCloseMemHandle(peer[r]);
        if (own_alloc && own) peer_pool_put(own);
        if (ctl) hipFree(ctl);
        if (tmp) hipFree(tmp);
    }
    bool own_alloc = true;
    PeerArgs args() const {
        PeerArgs a{};
        for (int r = 0; r < world; r++) a.buf[r] = peer[r];
        a.world = world;
        a.rank = rank;
        a.ctl = ctl;
        return a;
    }
    template <int OP>
    int run(const void* src, void* dst, int64_t n, hipStream_t st) {
        hipLaunchKernelGGL((peer_kernel<OP>), dim3(kPeerBlocks), dim3(256), 0, st, args(), src, dst, n);
        QIE_LAUNCH_CHECK();
        return 0;
    }
    // large exchanges (prefill rows) go through in slot-sized chunks, one generation each
    int allreduce_sum_f32(float* buf, int64_t n, hipStream_t st) override {
        const int64_t per = kPeerCap / 4;
        for (int64_t o = 0; o < n; o += per) QIE_TRY_C(run<kPeerSumF32>(buf + o, buf + o, std::min(per, n - o), st));
        return 0;
    }
    // tagged form for decode-sized exchanges, producer-side push (qie_comm_peer_set_mode; env
    // defaults QIE_PEER_TAGGED / QIE_PEER_PUSH, 1 each)
    int tagged = dev_env("QIE_PEER_TAGGED", 1);
    int push = dev_env("QIE_PEER_PUSH", 1);
    bool tagged_on() const { return tagged != 0; }
    static unsigned tag_blocks() {
        static const int v = dev_env("QIE_PEER_TAG_BLOCKS", kPeerBlocks);
        return (unsigned)std::max(1, std::min(v, 256));
    }
    template <bool PUSHED>
    int run_tagged(const float* part, uint16_t* x, int64_t n, hipStream_t st) {
        hipLaunchKernelGGL((peer_tag_kernel<PUSHED>), dim3(tag_blocks()), dim3(256), 0, st, args(), part, x, n);
        QIE_LAUNCH_CHECK();
        return 0;
    }
    bool peer_push(PeerPush* out, int64_t n) const override {
        if (!push || !tagged_on() || n <= 0 || n * 8 > kPeerTagCap) return false;
        for (int r = 0; r < kPeerTagMaxWorld; r++) out->tb[r] = r < world ? peer[r] + kPeerTagOff : nullptr;
        out->gen = ctl;
        out->world = world;
        out->rank = rank;
        return true;
    }
    int allreduce_residual_pushed(uint16_t* x, int64_t n, hipStream_t st) override {
        QIE_REQUIRE(n > 0 && n * 8 <= kPeerTagCap, "peer exchange: pushed exchange of %lld elements exceeds a slot",
                    (long long)n);
        return run_tagged<true>(nullptr, x, n, st);
    }
    int allreduce_residual_bf16(const float* part, uint16_t* x, int64_t n, hipStream_t st) override {
        if (n > 0 && n * 8 <= kPeerTagCap && tagged_on()) return run_tagged<false>(part, x, n, st);
        const int64_t per = kPeerCap / 4;   // a multiple of 8
        for (int64_t o = 0; o < n; o += per)
            QIE_TRY_C(run<kPeerSumResid>(part + o, x + o, std::min(per, n - o), st));
        return 0;
    }
    int allreduce_max_u64(uint64_t* buf, int64_t n, hipStream_t st) override {
        const int64_t per = kPeerCap / 8;
        for (int64_t o = 0; o < n; o += per) QIE_TRY_C(run<kPeerMaxU64>(buf + o, buf + o, std::min(per, n - o), st));
        return 0;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st) override {
        // byte-granular form for odd sizes (a vocab shard of 777 bf16 logits), small by construction
        if (bytes % 4 != 0) {
            QIE_REQUIRE(bytes <= kPeerCap, "peer allgather: %lld bytes (not a multiple of 4) exceed a slot",
                        (long long)bytes);
            return run<kPeerGatherB>(send, recv, bytes, st);
        }
        const int64_t words = bytes / 4, per = kPeerCap / 4;
        if (words <= per) return run<kPeerGather>(send, recv, words, st);
        // chunked: gather each chunk into tmp [world][chunk], then scatter into recv rows
        if ((size_t)(world * per * 4) > tmp_bytes) {
            if (tmp) hipFree(tmp);
            tmp = nullptr;
            QIE_HIP(hipMalloc((void**)&tmp, (size_t)world * per * 4));
            tmp_bytes = (size_t)world * per * 4;
        }
        for (int64_t o = 0; o < words; o += per) {
            const int64_t c = std::min(per, words - o);
            QIE_TRY_C(run<kPeerGather>((const uint32_t*)send + o, tmp, c, st));
            for (int r = 0; r < world; r++)
                QIE_HIP(hipMemcpyAsync((char*)recv + (int64_t)r * bytes + o * 4, (char*)tmp + (int64_t)r * c * 4,
                                       (size_t)c * 4, hipMemcpyDeviceToDevice, st));
        }
        return 0;
    }
    bool graph_capturable() const override { return true; }
    const unsigned* error_word() const override { return ctl + 2; }
    int error_state(void* stream) const override {   // stream-ordered (never the null stream)
        unsigned v = 0;
        if (hipMemcpyAsync(&v, ctl + 2, sizeof(v), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return -1;
        return (int)v;
    }
};

static int peer_alloc(PeerComm* c) {
    const size_t tag_bytes = (size_t)2 * kPeerMaxWorld * kPeerTagCap;
    const size_t bytes = (size_t)kPeerTagOff + tag_bytes;
    c->own = peer_pool_get();
    if (!c->own) QIE_HIP(hipExtMallocWithFlags((void**)&c->own, bytes, hipDeviceMallocUncached));
    QIE_HIP(hipMemset(c->own, 0, kPeerFlagBytes));
    QIE_HIP(hipMemset(c->own + kPeerTagOff, 0, tag_bytes));   // tag 0: no generation's
    QIE_HIP(hipMalloc((void**)&c->ctl, 64));
    QIE_HIP(hipMemset(c->ctl, 0, 64));
    QIE_HIP(hipDeviceSynchronize());   // zeroed before any stream's exchange kernel can run
    return 0;
}

}  // namespace qie

int qie_comm::allreduce_residual_bf16(const float* part, uint16_t* x, int64_t n, hipStream_t st) {
    const int rc = allreduce_sum_f32(const_cast<float*>(part), n, st);   // the engine's own scratch
    if (rc) return rc;
    return qie_residual_add_f32(x, part, n, st);
}

using namespace qie;

extern "C" {

int qie_comm_unique_id(void* id_out) {
    QIE_REQUIRE(id_out, "qie_comm_unique_id: null output");
    ncclUniqueId id;
    QIE_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int qie_comm_create_rccl(const void* id, int32_t world, int32_t rank, int32_t device, qie_comm** out) {
    QIE_REQUIRE(id && out && world >= 1 && rank >= 0 && rank < world, "qie_comm_create_rccl: bad arguments");
    QIE_HIP(hipSetDevice(device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    auto* c = new RcclComm();
    c->world = world;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->c, world, uid, rank);
    if (r != ncclSuccess) {
        c->c = nullptr;
        delete c;
        return fail(-100 - (int)r, "ncclCommInitRank(world %d, rank %d): %s", world, rank, ncclGetErrorString(r));
    }
    *out = c;
    return 0;
}

int qie_comm_create_local(int32_t world, qie_comm** out) {
    QIE_REQUIRE(out && world >= 1 && world <= kLocalMaxWorld, "qie_comm_create_local: world must be 1..%d",
                kLocalMaxWorld);
    auto g = std::make_shared<LocalGroup>();
    g->world = world;
    g->ptr.assign(world, nullptr);
    g->ready.assign(world, nullptr);
    g->done.assign(world, nullptr);
    for (int r = 0; r < world; r++) {
        QIE_HIP(hipEventCreateWithFlags(&g->ready[r], hipEventDisableTiming));
        QIE_HIP(hipEventCreateWithFlags(&g->done[r], hipEventDisableTiming));
    }
    for (int r = 0; r < world; r++) {
        auto* c = new LocalComm();
        c->world = world;
        c->rank = r;
        c->g = g;
        out[r] = c;
    }
    return 0;
}

int qie_comm_create_peer(int32_t world, int32_t rank, int32_t device, qie_comm** out, void* handle_out) {
    QIE_REQUIRE(out && handle_out && world >= 1 && world <= kPeerMaxWorld && rank >= 0 && rank < world,
                "qie_comm_create_peer: bad arguments (world 1..%d)", kPeerMaxWorld);
    QIE_HIP(hipSetDevice(device));
    auto* c = new PeerComm();
    c->world = world;
    c->rank = rank;
    const int rc = peer_alloc(c);
    if (rc) {
        delete c;
        return rc;
    }
    c->peer[rank] = c->own;
    hipIpcMemHandle_t h;
    const hipError_t he = hipIpcGetMemHandle(&h, c->own);
    if (he != hipSuccess) {
        delete c;
        return fail((int)he, "qie_comm_create_peer: hipIpcGetMemHandle: %s", hipGetErrorString(he));
    }
    static_assert(sizeof(hipIpcMemHandle_t) <= QIE_COMM_PEER_HANDLE_BYTES, "IPC handle size");
    std::memset(handle_out, 0, QIE_COMM_PEER_HANDLE_BYTES);
    std::memcpy(handle_out, &h, sizeof(h));
    *out = c;
    return 0;
}

int qie_comm_peer_connect(qie_comm* comm, const void* handles) {
    auto* c = dynamic_cast<PeerComm*>(comm);
    QIE_REQUIRE(c && handles, "qie_comm_peer_connect: not a peer communicator");
    for (int r = 0; r < c->world; r++) {
        if (r == c->rank) continue;
        hipIpcMemHandle_t h;
        std::memcpy(&h, (const char*)handles + (int64_t)r * QIE_COMM_PEER_HANDLE_BYTES, sizeof(h));
        void* p = nullptr;
        const hipError_t he = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (he != hipSuccess)
            return fail((int)he, "qie_comm_peer_connect: rank %d: hipIpcOpenMemHandle: %s", r, hipGetErrorString(he));
        c->peer[r] = (char*)p;
        c->opened[r] = true;
    }
    return 0;
}

int qie_comm_create_peer_local(int32_t world, qie_comm** out) {
    // ranks of one process share its hardware queues (4): beyond 2 ranks two of them can land
    // on one queue, where a waiting exchange kernel blocks its own peer (see the kernel's notes)
    QIE_REQUIRE(out && world >= 1 && world <= 2, "qie_comm_create_peer_local: world must be 1 or 2");
    std::vector<PeerComm*> cs;
    for (int r = 0; r < world; r++) {
        auto* c = new PeerComm();
        c->world = world;
        c->rank = r;
        const int rc = peer_alloc(c);
        if (rc) {
            delete c;
            for (auto* d : cs) delete d;
            return rc;
        }
        cs.push_back(c);
    }
    for (auto* c : cs)
        for (int r = 0; r < world; r++) c->peer[r] = cs[r]->own;
    for (int r = 0; r < world; r++) out[r] = cs[r];
    return 0;
}

int qie_comm_peer_error(const qie_comm* comm, int32_t* err) {
    auto* c = dynamic_cast<const PeerComm*>(comm);
    QIE_REQUIRE(c && err, "qie_comm_peer_error: not a peer communicator");
    unsigned v[3] = {0, 0, 0};
    QIE_HIP(hipMemcpy(v, c->ctl, sizeof(v), hipMemcpyDeviceToHost));
    *err = (int32_t)v[2];
    return 0;
}

int qie_comm_allreduce_residual_bf16(qie_comm* c, const float* part, void* x, int64_t n, void* stream) {
    QIE_REQUIRE(c && part && x && n >= 0, "qie_comm_allreduce_residual_bf16: bad arguments");
    return c->allreduce_residual_bf16(part, (uint16_t*)x, n, (hipStream_t)stream);
}

int qie_comm_peer_set_mode(qie_comm* comm, int32_t tagged, int32_t push) {
    auto* c = dynamic_cast<PeerComm*>(comm);
    QIE_REQUIRE(c && (tagged == 0 || tagged == 1) && (push == 0 || push == 1),
                "qie_comm_peer_set_mode: a peer communicator and 0/1 flags");
    c->tagged = tagged;
    c->push = push;
    return 0;
}

int qie_comm_time_exchange(qie_comm* c, const float* part, void* x, int64_t n, int32_t count, int32_t reps,
                           int32_t form, void* stream, float* us_out) {
    QIE_REQUIRE(c && part && x && n >= 0 && count >= 1 && reps >= 1 && form >= 0 && form <= 2 && us_out && stream,
                "qie_comm_time_exchange: bad arguments");
    auto* pc = dynamic_cast<PeerComm*>(c);
    QIE_REQUIRE(form == 0 || pc, "qie_comm_time_exchange: forms 1 and 2 are the peer backend's");
    QIE_REQUIRE(c->graph_capturable(), "qie_comm_time_exchange: backend is not graph-capturable");
    hipStream_t st = (hipStream_t)stream;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    QIE_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < count && rc == 0; i++) {
        if (form == 0) rc = c->allreduce_residual_bf16(part, (uint16_t*)x, n, st);
        else rc = pc->run<kPeerSumResid>(part, x, form == 2 ? 0 : n, st);
    }
    const hipError_t ce = hipStreamEndCapture(st, &g);
    if (rc || ce != hipSuccess) {
        if (g) hipGraphDestroy(g);
        return rc ? rc : fail((int)ce, "qie_comm_time_exchange: capture: %s", hipGetErrorString(ce));
    }
    float ms = 0.f;
    auto run = [&]() -> int {
        QIE_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        QIE_HIP(hipEventCreate(&e0));
        QIE_HIP(hipEventCreate(&e1));
        QIE_HIP(hipGraphLaunch(ge, st));
        QIE_HIP(hipStreamSynchronize(st));
        QIE_HIP(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) QIE_HIP(hipGraphLaunch(ge, st));
        QIE_HIP(hipEventRecord(e1, st));
        QIE_HIP(hipEventSynchronize(e1));
        QIE_HIP(hipEventElapsedTime(&ms, e0, e1));
        return 0;
    };
    rc = run();
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (ge) hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    if (rc) return rc;
    *us_out = ms * 1000.f / ((float)count * (float)reps);
    return 0;
}

int qie_comm_rank(const qie_comm* c, int32_t* world, int32_t* rank) {
    QIE_REQUIRE(c, "qie_comm_rank: null communicator");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    return 0;
}

int qie_comm_allreduce_sum_f32(qie_comm* c, float* buf, int64_t n, void* stream) {
    QIE_REQUIRE(c && buf && n >= 0, "qie_comm_allreduce_sum_f32: bad arguments");
    return c->allreduce_sum_f32(buf, n, (hipStream_t)stream);
}

int qie_comm_allreduce_max_u64(qie_comm* c, uint64_t* buf, int64_t n, void* stream) {
    QIE_REQUIRE(c && buf && n >= 0, "qie_comm_allreduce_max_u64: bad arguments");
    return c->allreduce_max_u64(buf, n, (hipStream_t)stream);
}

void qie_comm_destroy(qie_comm* c) { delete c; }

}  // extern "C"
