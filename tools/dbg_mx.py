#!/usr/bin/env python3
"""Debug probe for the fp8-activation prefill (dev only): tiny-model engine with
prefill_fp8 (single and batched prefill) against the oracle in act_fp8 and bf16-activation
modes, and the SWIGLU op's worst elements."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import ctypes as C  # noqa: E402
import oracle as O  # noqa: E402
import gpu_util as G  # noqa: E402
from parity import norm_rel  # noqa: E402
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import _lib, spec as S, weights as W  # noqa: E402


def engine_probe():
    spec = S.tiny("t-mx", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=1024,
                  bias=True)
    syn = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
    hw = W.HostWeights.synthetic(spec, syn).fp8_dequantized()
    prompts = [[int(t) for t in np.random.default_rng(50 + i).integers(0, spec.vocab, 70)] for i in range(4)]
    want_q = [O.Model(hw, 96, prefill_act_fp8=True).forward(p, 0) for p in prompts]
    want_b = [O.Model(hw, 96).forward(p, 0) for p in prompts]
    for pf8 in (False, True):
        eng = Q.Engine(spec, max_ctx=96, weight_fp8=True, prefill_fp8=pf8).init_synthetic(syn)
        for batched in (False, True):
            b = eng.batch(4, 96)
            if batched:
                b.prefill_batch(0, prompts)
            else:
                for i, p in enumerate(prompts):
                    b.prefill(i, p)
            lg = b.logits()
            print(f"prefill_fp8={pf8} batched={batched}: vs act-oracle",
                  [f"{norm_rel(lg[i], want_q[i]):.2e}" for i in range(4)], " vs bf16-oracle",
                  [f"{norm_rel(lg[i], want_b[i]):.2e}" for i in range(4)], flush=True)
            b.close()
        eng.close()


def swiglu_probe():
    lib = _lib.load()
    from test_gpu_fp8_mx import _quant_dev, _fp8w, _mx_linear
    from test_gpu_ops import rand_bf16, _abs_scale
    for M, K, I in ((40, 896, 640), (40, 3584, 640), (300, 3584, 18944)):
        x = rand_bf16(O, (M, K), seed=6)
        (dg, qg), (du, qu) = _fp8w(lib, rand_bf16(O, (I, K), 0.08, seed=7), False), \
            _fp8w(lib, rand_bf16(O, (I, K), 0.08, seed=8), False)
        dqx, _ = O.quant_rows_fp8(x)
        q, e = _quant_dev(lib, x)
        for epi, name in ((_lib.QIE_EPI_STORE, "gate-only STORE"),):
            y = G.zeros_bf16(M, I)
            _mx_linear(lib, q, e, [(dg, I)], [None], M, K, I, y, epi, False)
            want = O.matmul(dqx, qg)
            got = G.bf(G.host_bf16(y)).astype(np.float64)
            w = G.bf(want).astype(np.float64)
            sc = _abs_scale(O, dqx, qg)
            err = np.abs(got - w) / sc
            print(f"{name} M={M} K={K} N={I}: max |err| / sum|a w| = {err.max():.3e}, ulps>1 frac "
                  f"{(G.ulp_diff(G.host_bf16(y), want) > 1).mean():.4f}", flush=True)
        y = G.zeros_bf16(M, I)
        _mx_linear(lib, q, e, [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU, False)
        want = O.silu_mul(O.matmul(dqx, qg), O.matmul(dqx, qu))
        d = G.ulp_diff(G.host_bf16(y), want)
        gs = G.bf(O.matmul(dqx, qg)).astype(np.float64)
        i = np.unravel_index(np.argmax(d), d.shape)
        print(f"SWIGLU M={M} K={K}: exact {(d == 0).mean():.4f}, max ulps {d.max()} at {i}, g {gs[i]:.4e}, "
              f"scale {_abs_scale(O, dqx, qg)[i]:.4e}", flush=True)
        G.release_all()


if __name__ == "__main__":
    swiglu_probe()
    engine_probe()
