// qie_comm.hpp — internal definition of the tensor-parallel communicator behind the
// opaque qie_comm handle of qie_engine.h.
//
// Three backends (the peer one in comm.hip's header comment):
//   * RCCL (one process per GPU, xGMI): ncclAllReduce / ncclAllGather enqueued on the
//     engine stream, so they are captured into the decode hipGraph;
//   * local (test backend): `world` ranks driven by host threads of ONE process, all
//     on one device; collectives are event waits + a host barrier + a reduction kernel.
//     Not graph-capturable (host barriers) — engines on it run eagerly.  It exists so
//     the sharded forward can be checked against the oracle on a one-GPU box, where
//     RCCL refuses two ranks on one device.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace qie { struct PeerPush; }

struct qie_comm {
    int world = 1, rank = 0;
    virtual ~qie_comm() = default;
    // in place; every rank ends with the identical sum (ranks summed in order 0..world-1
    // by the local backend; RCCL's ring gives one reduced value per element to all)
    virtual int allreduce_sum_f32(float* buf, int64_t n, hipStream_t st) = 0;
    virtual int allreduce_max_u64(uint64_t* buf, int64_t n, hipStream_t st) = 0;
    // recv = [world][bytes], rank r's send at offset r * bytes
    virtual int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st) = 0;
    virtual bool graph_capturable() const = 0;
    // x (bf16 [n]) = bf16(x + bf16(all-reduced sum of part)): the row-parallel exchange; the
    // peer backend does it in one kernel, the others all-reduce `part` in place and add
    virtual int allreduce_residual_bf16(const float* part, uint16_t* x, int64_t n, hipStream_t st);
    // non-zero once an exchange failed on the device (the peer backend's bounded wait timed
    // out); read after the stream synchronised — a blocking copy of one word
    virtual int error_state(void* stream) const { (void)stream; return 0; }
    // device word error_state reads (nullptr: the backend has none), so a caller that already
    // copies results back can read it in the same stream-ordered batch, one synchronisation
    virtual const unsigned* error_word() const { return nullptr; }
    // Producer-side push (peer backend, tagged form): true when an n-element row-parallel
    // exchange may take its partials from the producer's epilogue (*out filled); the
    // exchange is then allreduce_residual_pushed — wait on the tagged words, reduce, add.
    virtual bool peer_push(qie::PeerPush* out, int64_t n) const { (void)out; (void)n; return false; }
    virtual int allreduce_residual_pushed(uint16_t* x, int64_t n, hipStream_t st) {
        (void)x; (void)n; (void)st;
        return -1;
    }
};
