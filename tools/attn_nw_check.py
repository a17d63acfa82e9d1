#!/usr/bin/env python3
"""Development A/B check (dev build, QIE_LIB=lib/dev/libqie.so): the causal prefill attention
with 4- and 8-wave workgroups (QIE_ATTN_PF_NW) must give bit-identical outputs (a row group's
arithmetic does not depend on which workgroup owns it).  Cases: P = 2048 / 1000 (ragged),
hd 128 (28 / 4 heads) and hd 64 (14 / 2 heads), two sequences of the ragged length."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gpu_util as G  # noqa: E402
from qwen_inference_engine_amd import _lib  # noqa: E402
from qwen_inference_engine_amd._lib import KvCacheC  # noqa: E402


def rnd(shape, seed):
    a = np.random.default_rng(seed).standard_normal(shape).astype(np.float32)
    return (a.view(np.uint32) >> 16).astype(np.uint16)


def run(R, nseq, nq, nkv, hd, nw):
    lib = _lib.load()
    os.environ["QIE_ATTN_PF_NW"] = str(nw)
    M = R * nseq
    kc, vc = G.dev(rnd((nseq, 1, nkv, R, hd), 8)), G.dev(rnd((nseq, 1, nkv, R, hd), 9))
    q = G.dev(rnd((M, nq * hd), 11))
    pos = G.dev(np.tile(np.arange(R, dtype=np.int32), nseq))
    out = G.zeros_bf16(M, nq * hd)
    c = KvCacheC()
    c.k, c.v, c.seq_stride = G.p(kc), G.p(vc), nkv * R * hd
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = 1, nkv, hd, R
    G.check(lib.qie_attention(G.p(q), M, G.p(pos), R, C.byref(c), 0, nq, G.p(out), None, None))
    G.check(lib.qie_synchronize())
    res = G.host(out).copy()
    G.release_all()
    return res


def main():
    bad = 0
    for R, nseq, nq, nkv, hd in ((2048, 1, 28, 4, 128), (1000, 2, 28, 4, 128), (2048, 1, 14, 2, 64), (333, 2, 14, 2, 64)):
        a, b = run(R, nseq, nq, nkv, hd, 4), run(R, nseq, nq, nkv, hd, 8)
        same = np.array_equal(a, b)
        bad += not same
        print(f"R={R} seqs={nseq} hd={hd}: nw4 == nw8 {same} (rows differing {int((a != b).any(axis=1).sum())})", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
