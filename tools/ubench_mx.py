#!/usr/bin/env python3
"""Block-scaled fp8 prefill GEMM (QIE_LINEAR_ACT_FP8) vs the bf16 LDS-DMA GEMM at the
headline / config-4 shapes (Qwen2-7B, M = 2048 and 8192 rows): the four projections through
qie_linear's real dispatch, UB_ITERS launches back to back, host-timed around a synchronise
(every case >= 50 us).  fp8 weights in the engine's 16-row tiled layout; plus the per-row
activation quantiser.  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes as C  # noqa: E402
import gpu_util as G  # noqa: E402
from qwen_inference_engine_amd import _lib  # noqa: E402
from qwen_inference_engine_amd._lib import LinearArgsC  # noqa: E402

H, I, QKV = 3584, 18944, 4608
ITERS = int(os.environ.get("UB_ITERS", "20"))


def rnd(shape, scale, seed):
    a = (np.random.default_rng(seed).standard_normal(shape) * scale).astype(np.float32)
    return (a.view(np.uint32) >> 16).astype(np.uint16)


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


def main():
    lib = _lib.load()
    shapes = [("qkv", H, QKV, 0), ("o", H, H, 1), ("gate_up", H, I, 2), ("down", I, H, 1)]
    for M in (2048, 8192):
        for name, K, N, epi in shapes:
            rows = 2 * N if epi == 2 else N
            wb = G.dev(rnd((rows, K), 0.02, 3))
            w8 = G.zeros((int(lib.qie_fp8_weight_bytes(rows, K)),), np.uint8)
            G.check(lib.qie_quantize_fp8(G.p(wb), rows, K, G.p(w8), None))
            wt = G.zeros((w8.nbytes,), np.uint8)
            G.check(lib.qie_fp8_tile16(G.p(w8), rows, K, G.p(wt), None))
            x = G.dev(rnd((M, K), 1.0, 1))
            q = G.zeros((M * K,), np.uint8)
            e = G.zeros((M,), np.uint8)
            y = G.zeros_bf16(M, N)
            flops = 2.0 * M * K * rows

            # separate gate / up segments: first and second half of the weight rows
            def seg_args(xp, base, fl, exps=None, fp8=False):
                a = LinearArgsC()
                a.x, a.ldx = G.p(xp), K
                if epi == 2:
                    w1 = G.zeros((int(lib.qie_fp8_weight_bytes(N, K)) if fp8 else N * K * 2,), np.uint8)
                    a.w[0], a.w[1] = G.p(base), G.p(w1)
                    a.seg_rows[0] = a.seg_rows[1] = N
                else:
                    a.w[0], a.seg_rows[0] = G.p(base), N
                a.M, a.K, a.N, a.y, a.ldy, a.flags = M, K, N, G.p(y), N, fl
                a.epilogue = {0: _lib.QIE_EPI_STORE, 1: _lib.QIE_EPI_RESIDUAL, 2: _lib.QIE_EPI_SWIGLU}[epi]
                if exps is not None:
                    a.x_exps = G.p(exps)
                return a
            ab = seg_args(x, wb, 0)
            am = seg_args(q, wt, _lib.QIE_LINEAR_FP8 | _lib.QIE_LINEAR_FP8_T16 | _lib.QIE_LINEAR_ACT_FP8, e, True)
            rb = timed(lambda: G.check(lib.qie_linear(C.byref(ab), None)), flops)
            rm = timed(lambda: G.check(lib.qie_linear(C.byref(am), None)), flops)
            rq = timed(lambda: G.check(lib.qie_quantize_rows_fp8(G.p(x), K, M, K, G.p(q), K, G.p(e), None)), 0)
            print(json.dumps({"M": M, "gemm": name, "K": K, "N": N, "bf16": rb, "fp8_mx": rm, "quant_us": rq["us"],
                              "speedup": round(rb["us"] / rm["us"], 3)}), flush=True)
            G.release_all()


if __name__ == "__main__":
    main()
