#!/usr/bin/env python3
"""Debug probe (dev): where are the fp8-activation GEMM's wrong elements?  Runs a gate-only
STORE three times (determinism), prints error statistics by row / column / 16x16 subtile
position, and the same with all exponents forced to 127 (scale 1) and integer-valued codes."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
import gpu_util as G  # noqa: E402
from qwen_inference_engine_amd import _lib, weights as W  # noqa: E402
from test_gpu_fp8_mx import _quant_dev, _fp8w, _mx_linear  # noqa: E402
from test_gpu_ops import rand_bf16, _abs_scale  # noqa: E402


def main():
    lib = _lib.load()
    M, K, N = 300, 3584, 2048
    x = rand_bf16(O, (M, K), seed=6)
    dg, qg = _fp8w(lib, rand_bf16(O, (N, K), 0.08, seed=7), False)
    dqx, _ = O.quant_rows_fp8(x)
    q, e = _quant_dev(lib, x)
    want = G.bf(O.matmul(dqx, qg)).astype(np.float64)
    sc = _abs_scale(O, dqx, qg)
    outs = []
    for rep in range(3):
        y = G.zeros_bf16(M, N)
        _mx_linear(lib, q, e, [(dg, N)], [None], M, K, N, y, _lib.QIE_EPI_STORE, False)
        outs.append(G.bf(G.host_bf16(y)).astype(np.float64))
    print("deterministic:", all(np.array_equal(outs[0], o) for o in outs[1:]))
    err = np.abs(outs[0] - want) / sc
    bad = err > 3e-5
    print(f"bad {bad.sum()} of {bad.size}; max {err.max():.3e}")
    r, c = np.nonzero(bad)
    if len(r):
        print("rows mod 16:", np.bincount(r % 16, minlength=16).tolist())
        print("rows mod 256 // 16:", np.bincount((r % 256) // 16, minlength=16).tolist())
        print("cols mod 16:", np.bincount(c % 16, minlength=16).tolist())
        print("cols mod 256 // 16:", np.bincount((c % 256) // 16, minlength=16).tolist())
        print("row tile:", np.bincount(r // 256).tolist(), "col tile:", np.bincount(c // 256).tolist())
        i = np.argmax(err)
        print("worst", np.unravel_index(i, err.shape), outs[0].flat[i], want.flat[i], sc.flat[i])
        # per-row exact float64 with the oracle's dequantised operands: is the oracle right?
        rr, cc = np.unravel_index(i, err.shape)
        ex = O.bf16_to_f32(dqx[rr]).astype(np.float64) @ O.bf16_to_f32(qg[cc]).astype(np.float64)
        print("float64 exact", ex)
        # which k-blocks: recompute with each 128-k tile dropped, find the tile whose omission explains it
        a = O.bf16_to_f32(dqx[rr]).astype(np.float64)
        w = O.bf16_to_f32(qg[cc]).astype(np.float64)
        parts = (a * w).reshape(-1, 32).sum(1)
        d = outs[0].flat[i] - ex
        cand = np.argsort(np.abs(parts - (-d)))[:5]
        print("delta", d, "closest 32-blocks to -delta:", [(int(k), parts[k]) for k in cand])
        parts128 = (a * w).reshape(-1, 128).sum(1)
        cand = np.argsort(np.abs(parts128 - (-d)))[:5]
        print("closest 128-tiles:", [(int(k), parts128[k]) for k in cand])


if __name__ == "__main__":
    main()
