#!/usr/bin/env python3
"""One rank of tests/test_gpu_tp.py::test_peer_two_processes_one_gpu (run as a child process,
never collected by pytest): a peer communicator across processes (HIP IPC handles exchanged
through files in DIR), one fused all-reduce + residual add and one fp32 all-reduce on seeded
data, the results written to DIR/out<rank>.npz.  Exit 5 (message on stderr) when the IPC
mapping itself is refused, so the test can report that as a skip."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    rank, world, d = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 60000
    import gpu_util as G
    import qwen_inference_engine_amd as Q

    def exchange(h):
        with open(os.path.join(d, f"h{rank}.tmp"), "wb") as f:
            f.write(h)
        os.replace(os.path.join(d, f"h{rank}.tmp"), os.path.join(d, f"h{rank}"))
        t0 = time.time()
        out = []
        for r in range(world):
            p = os.path.join(d, f"h{r}")
            while not os.path.exists(p):
                if time.time() - t0 > 60:
                    raise TimeoutError(f"rank {r} never published its handle")
                time.sleep(0.05)
            out.append(open(p, "rb").read())
        return out
    try:
        comm = Q.Comm.peer(world, rank, 0, exchange)
    except Exception as ex:   # the IPC mapping refused on this box
        print(f"peer_worker: {ex}", file=sys.stderr)
        return 5
    lib = Q._lib.load()
    part = np.random.default_rng(10 + rank).standard_normal(n).astype(np.float32)
    x0 = G.to_bf16(np.random.default_rng(5).standard_normal(n).astype(np.float32))
    pb, xb, sb = G.dev(part), G.dev(x0), G.dev(part)
    st = G.stream()
    G.check(lib.qie_comm_allreduce_residual_bf16(comm.h, G.p(pb), G.p(xb), n, st))
    G.check(lib.qie_comm_allreduce_sum_f32(comm.h, G.p(sb), n, st))
    G.check(lib.qie_stream_synchronize(st))
    err = comm.peer_error()
    np.savez(os.path.join(d, f"out{rank}.npz"), x=G.host_bf16(xb), s=G.host(sb), err=np.int32(err))
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
