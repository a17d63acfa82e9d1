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

#include <rccl/rccl.h>

#include <condition_variable>
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

}  // namespace qie

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

void qie_comm_destroy(qie_comm* c) { delete c; }

}  // extern "C"
