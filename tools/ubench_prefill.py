#!/usr/bin/env python3
"""Prefill kernel micro-benchmark at the headline shapes (Qwen2-7B, P = 2048): the four
projection GEMMs through qie_linear's real dispatch and the causal flash attention through
qie_attention, each launched UB_ITERS times back to back on the null stream and timed on
the host around a device synchronise (every case runs >= 50 us, so launch cost hides).
Variants: UB_ENVS="NAME=v1,NAME=v2" re-runs every case with that environment variable set
(development A/B only).  One JSON line per case and variant."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gpu_util as G  # noqa: E402
from qwen_inference_engine_amd import _lib  # noqa: E402
from qwen_inference_engine_amd._lib import LinearArgsC, KvCacheC  # noqa: E402

M, H, I, NQ, NKV, HD = 2048, 3584, 18944, 28, 4, 128
ITERS = int(os.environ.get("UB_ITERS", "20"))


def rnd(shape, scale, seed):
    a = (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)
    return (a.view(np.uint32) >> 16).astype(np.uint16)


def linear_args(x, segs, M, K, N, y, epi, biases=()):
    a = LinearArgsC()
    a.x, a.ldx = G.p(x), K
    for i, (w, r) in enumerate(segs):
        a.w[i] = G.p(w)
        a.seg_rows[i] = r
    for i, b in enumerate(biases):
        a.bias[i] = G.p(b)
    a.M, a.K, a.N = M, K, N
    a.y, a.ldy = G.p(y), N
    a.epilogue = epi
    return a


def timed(fn, flops):
    lib = _lib.load()
    fn()
    G.check(lib.qie_synchronize())
    t0 = time.perf_counter()
    for _ in range(ITERS):
        fn()
    G.check(lib.qie_synchronize())
    us = (time.perf_counter() - t0) * 1e6 / ITERS
    return {"us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}


def cases():
    lib = _lib.load()
    xh = G.dev(rnd((M, H), 1.0, 1))
    xi = G.dev(rnd((M, I), 1.0, 2))
    wq = [G.dev(rnd((r, H), 0.02, 10 + i)) for i, r in enumerate((NQ * HD, NKV * HD, NKV * HD))]
    bq = [G.dev(rnd((r,), 0.1, 20 + i)) for i, r in enumerate((NQ * HD, NKV * HD, NKV * HD))]
    wo = G.dev(rnd((H, NQ * HD), 0.02, 3))
    wg, wu = G.dev(rnd((I, H), 0.02, 4)), G.dev(rnd((I, H), 0.02, 5))
    wd = G.dev(rnd((H, I), 0.02, 6))
    yq = G.zeros_bf16(M, (NQ + 2 * NKV) * HD)
    yh = G.dev(rnd((M, H), 1.0, 7))
    yi = G.zeros_bf16(M, I)
    out = {}
    nqkv = (NQ + 2 * NKV) * HD
    aq = linear_args(xh, list(zip(wq, (NQ * HD, NKV * HD, NKV * HD))), M, H, nqkv, yq, _lib.QIE_EPI_STORE, bq)
    ao = linear_args(xh, [(wo, H)], M, H, H, yh, _lib.QIE_EPI_RESIDUAL)
    agu = linear_args(xh, [(wg, I), (wu, I)], M, H, I, yi, _lib.QIE_EPI_SWIGLU)
    ad = linear_args(xi, [(wd, H)], M, I, H, yh, _lib.QIE_EPI_RESIDUAL)
    for name, a, fl in (("qkv", aq, 2.0 * M * nqkv * H), ("o", ao, 2.0 * M * H * H),
                        ("gate_up", agu, 4.0 * M * I * H), ("down", ad, 2.0 * M * I * H)):
        out[name] = timed(lambda a=a: G.check(lib.qie_linear(C.byref(a), None)), fl)
    # causal prefill attention, one layer of the headline cache
    maxc = M
    kc, vc = G.dev(rnd((1, 1, NKV, maxc, HD), 1.0, 8)), G.dev(rnd((1, 1, NKV, maxc, HD), 1.0, 9))
    q = G.dev(rnd((M, NQ * HD), 1.0, 11))
    pos = G.dev(np.arange(M, dtype=np.int32))
    ao_ = G.zeros_bf16(M, NQ * HD)
    ws = G.zeros_bytes(max(1, lib.qie_attention_workspace_bytes(M, NQ, HD, maxc)))
    c = KvCacheC()
    c.k, c.v, c.seq_stride = G.p(kc), G.p(vc), NKV * maxc * HD
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = 1, NKV, HD, maxc
    fl = 4.0 * NQ * HD * M * (M + 1) / 2
    out["attention"] = timed(lambda: G.check(lib.qie_attention(G.p(q), M, G.p(pos), M, C.byref(c), 0, NQ, G.p(ao_),
                                                                   G.p(ws), None)), fl)
    return out


def main():
    envs = [e for e in os.environ.get("UB_ENVS", "").split(",") if e]
    for var in [None] + envs:
        if var:
            k, v = var.split("=", 1)
            os.environ[k] = v
        print(json.dumps({"variant": var or "default", **cases()}), flush=True)
        if var:
            del os.environ[k]
        G.release_all()


if __name__ == "__main__":
    main()
