#!/usr/bin/env python3
"""A/B of the prefill projection GEMMs (Qwen2-7B at P = AB_M rows) over development-build knobs:
every variant's output is compared bit for bit with the first variant's (a kernel change that
keeps the k-order of the fp32 sums must reproduce it exactly), and timed in interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  O and down use the STORE epilogue here (the engine's
residual epilogue reads one more bf16 per output).  One JSON line per (GEMM, variant).

  QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so AB_GEMM_VARIANTS='[{}, {"QIE_GEMM8": "1"}]' \\
      python tools/ab_gemm.py"""
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
from qwen_inference_engine_amd._lib import LinearArgsC  # noqa: E402

M = int(os.environ.get("AB_M", "2048"))
H, I, NQ, NKV, HD = 3584, 18944, 28, 4, 128
ITERS = int(os.environ.get("AB_ITERS", "10"))
ROUNDS = int(os.environ.get("AB_ROUNDS", "3"))


def rnd(shape, scale, seed):
    a = (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)
    return (a.view(np.uint32) >> 16).astype(np.uint16)


def linear_args(x, segs, K, N, y, epi, biases=()):
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


def main():
    lib = _lib.load()
    variants = json.loads(os.environ.get("AB_GEMM_VARIANTS", "[{}]"))
    xh = G.dev(rnd((M, H), 1.0, 1))
    xi = G.dev(rnd((M, I), 1.0, 2))
    nq = (NQ * HD, NKV * HD, NKV * HD)
    wq = [G.dev(rnd((r, H), 0.02, 10 + i)) for i, r in enumerate(nq)]
    bq = [G.dev(rnd((r,), 0.1, 20 + i)) for i, r in enumerate(nq)]
    wo = G.dev(rnd((H, NQ * HD), 0.02, 3))
    wg, wu = G.dev(rnd((I, H), 0.02, 4)), G.dev(rnd((I, H), 0.02, 5))
    wd = G.dev(rnd((H, I), 0.02, 6))
    nqkv = sum(nq)
    gemms = {
        "qkv": (lambda y: linear_args(xh, list(zip(wq, nq)), H, nqkv, y, _lib.QIE_EPI_STORE, bq), nqkv,
                2.0 * M * nqkv * H),
        "o": (lambda y: linear_args(xh, [(wo, H)], H, H, y, _lib.QIE_EPI_STORE), H, 2.0 * M * H * H),
        "gate_up": (lambda y: linear_args(xh, [(wg, I), (wu, I)], H, I, y, _lib.QIE_EPI_SWIGLU), I,
                    4.0 * M * I * H),
        "down": (lambda y: linear_args(xi, [(wd, H)], I, H, y, _lib.QIE_EPI_STORE), H, 2.0 * M * I * H),
    }
    only = os.environ.get("AB_GEMMS")
    if only:
        gemms = {k: v for k, v in gemms.items() if k in only.split(",")}
    ys = {name: G.zeros_bf16(M, N) for name, (mk, N, fl) in gemms.items()}
    ref = {}
    res = {}
    for rnd_i in range(ROUNDS):
        for vi, env in enumerate(variants):
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update({k: str(v) for k, v in env.items()})
            try:
                for name, (mk, N, fl) in gemms.items():
                    y = ys[name]
                    G.check(lib.qie_memset(G.p(y), 0, y.nbytes))
                    a = mk(y)
                    G.check(lib.qie_linear(C.byref(a), None))
                    G.check(lib.qie_synchronize())
                    if rnd_i == 0:
                        out = G.host_bf16(y)
                        if name not in ref:
                            ref[name] = out
                        res.setdefault((name, vi), {})["bit_equal"] = bool(np.array_equal(out, ref[name]))
                        res[(name, vi)]["max_ulp"] = int(G.ulp_diff(out, ref[name]).max())
                    t0 = time.perf_counter()
                    for _ in range(ITERS):
                        G.check(lib.qie_linear(C.byref(a), None))
                    G.check(lib.qie_synchronize())
                    us = (time.perf_counter() - t0) * 1e6 / ITERS
                    res[(name, vi)].setdefault("us", []).append(us)
                    res[(name, vi)]["flops"] = fl
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        print(f"ab_gemm: round {rnd_i + 1}/{ROUNDS}", file=sys.stderr, flush=True)
    for (name, vi), r in res.items():
        us = float(np.median(r["us"]))
        print(json.dumps({"gemm": name, "env": variants[vi], "us_median": round(us, 2),
                          "us": [round(u, 1) for u in r["us"]], "tflops": round(r["flops"] / us / 1e6, 1),
                          "bit_equal": r["bit_equal"], "max_ulp": r["max_ulp"]}), flush=True)


if __name__ == "__main__":
    main()
