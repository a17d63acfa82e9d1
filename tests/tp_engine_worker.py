#!/usr/bin/env python3
"""One rank of tests/test_gpu_tp.py::test_engine_tp_two_processes_peer_forced_decisions (run
as a child process, never collected by pytest): the ENGINE's tensor-parallel forward across
processes — a peer communicator over HIP IPC (handles exchanged through files in DIR), a
Qwen2-7B-width model (N_LAYERS layers, peaked synthetic head) sharded over WORLD ranks, decode
steps replayed from a captured hipGraph — driven through the teacher-forced protocol of
tests/parity.py forced_decisions (same forced continuation seed).  Every decision's gathered
logits and greedy id go to DIR/out<rank>.npz; the parent test checks them against the oracle.
Exit 5 (message on stderr) when the IPC mapping itself is refused."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

FORCED_SEED = 77     # tests/parity.py forced_decisions' default


def file_exchange(d, rank, world, tag):
    def exchange(h):
        tmp = os.path.join(d, f"{tag}{rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(h)
        os.replace(tmp, os.path.join(d, f"{tag}{rank}"))
        t0 = time.time()
        out = []
        for r in range(world):
            p = os.path.join(d, f"{tag}{r}")
            while not os.path.exists(p):
                if time.time() - t0 > 120:
                    raise TimeoutError(f"rank {r} never published its handle")
                time.sleep(0.05)
            out.append(open(p, "rb").read())
        return out
    return exchange


def main():
    rank, world, d = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    n_layers, P, n = int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
    import qwen_inference_engine_amd as Q
    from qwen_inference_engine_amd import spec as S, weights as W
    from parity import PEAKED
    try:
        comm = Q.Comm.peer(world, rank, 0, file_exchange(d, rank, world, "h"))
    except Exception as ex:   # the IPC mapping refused on this box
        print(f"tp_engine_worker: {ex}", file=sys.stderr)
        return 5
    spec = S.QWEN2_7B.replace(n_layers=n_layers)
    max_ctx = P + n + 16
    eng = Q.Engine(spec, max_ctx=max_ctx, use_graph=True, comm=comm).init_synthetic(W.SynthParams(seed=0, **PEAKED))
    b = eng.batch(1, max_ctx)
    prompt = [int(t) for t in np.random.default_rng(P).integers(0, spec.vocab, P)]
    forced = [int(t) for t in np.random.default_rng(FORCED_SEED).integers(0, spec.vocab, max(n - 1, 0))]
    ids, logits = [], []
    t = b.prefill(0, prompt)
    for i in range(n):
        ids.append(int(t))
        logits.append(b.logits()[0].copy())       # collective: both ranks gather the vocab shards
        if i + 1 < n:
            b.set_position(0, P + i, forced[i])
            t = b.decode_step()[0]                # graph replay (captured at the first step)
    err = comm.peer_error()
    np.savez(os.path.join(d, f"out{rank}.npz"), ids=np.array(ids, np.int32), logits=np.stack(logits),
             prompt=np.array(prompt, np.int32), err=np.int32(err))
    b.close()
    eng.close()
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
