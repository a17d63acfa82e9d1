#!/usr/bin/env python3
"""Probe for test_tp_weights_bin_equals_synthetic's intermittent logit mismatch: the same
scenario (Qwen3-style tiny model, TP2 on the local backend, synthetic vs weights.bin engines)
repeated, with device memory poisoned (allocated, filled with a byte pattern, freed) before
each engine so that a read of memory nothing wrote shows up.  Prints, per iteration and rank,
whether ids / logits agree and the first differing logit columns."""
import ctypes as C
import os
import sys
import tempfile
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import _lib, spec as S, weights as W  # noqa: E402

SYN = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
spec = S.tiny("t-q3", n_layers=2, hidden=512, n_heads=8, n_kv_heads=2, head_dim=128, ffn=768, vocab=1536, bias=False,
              qk_norm=True)
world = 2
lib = _lib.load()


def poison(nbytes, byte):
    p = C.c_void_p()
    _lib.check(lib.qie_malloc(C.byref(p), nbytes), "malloc")
    _lib.check(lib.qie_memset(p, byte, nbytes), "memset")
    _lib.check(lib.qie_synchronize(), "sync")
    lib.qie_free(p)


def run(binp, meta, pat):
    comms = Q.Comm.local(world)
    out, err = [None] * world, [None] * world

    def fn(r):
        try:
            res = []
            for src in ("syn", "bin"):
                e = Q.Engine(spec, max_ctx=64, comm=comms[r])
                e = e.init_synthetic(SYN) if src == "syn" else e.load_weights_bin(binp, meta)
                b = e.batch(1, 64)
                ids = [b.prefill(0, [5, 9, 2, 7, 1, 3])] + list(b.decode(6)[:, 0])
                res.append((ids, b.logits()))
                b.close()
                e.close()
            out[r] = res
        except BaseException as ex:  # noqa: BLE001
            err[r] = ex
    ts = [threading.Thread(target=fn, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    for c in comms:
        c.close()
    for e in err:
        if e is not None:
            raise e
    for r in range(world):
        (i1, l1), (i2, l2) = out[r]
        d = np.nonzero(l1[0] != l2[0])[0]
        print(f"pattern {pat:#04x} rank {r}: ids {'==' if i1 == i2 else '!='} logits diff at {len(d)} cols "
              f"{d[:12].tolist()}", flush=True)


def main():
    hw = W.HostWeights.synthetic(spec, SYN)
    d = tempfile.mkdtemp()
    binp, meta = os.path.join(d, "weights.bin"), os.path.join(d, "meta_data.txt")
    hw.write_weights_bin(binp, meta)
    for it in range(int(os.environ.get("FT_ITERS", "6"))):
        pat = [0x00, 0x7f, 0xff, 0x3c, 0xc1, 0x55][it % 6]
        poison(1 << 30, pat)
        run(binp, meta, pat)


if __name__ == "__main__":
    main()
