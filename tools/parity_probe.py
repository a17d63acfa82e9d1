#!/usr/bin/env python3
"""Localise where the engine's numerics leave the oracle's (GPU box; test tooling).

Runs a model teacher-forced on the engine and on the oracle (order 0) and, after the
prefill and after every decode step, compares the cached K and V rows of every layer at
every position written so far.  Layer l's K/V rows are a function of the residual stream
entering layer l only, so the first (step, layer, kind) whose rows differ localises the
first diverging op to layer l - 1's attention / O / MLP (or layer l's QKV + RoPE when
V matches and K does not).  Prints one line per step with the first mismatch and the
logit norm-relative error.

    python tools/parity_probe.py [--fp8] [--model tiny|7b2] [--steps N] [--prompt P]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402
from parity import norm_rel  # noqa: E402


def ulps(a, b):
    def key(x):
        x = x.astype(np.int32)
        return np.where(x & 0x8000, -(x & 0x7FFF), x & 0x7FFF)
    return np.abs(key(a) - key(b))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--model", default="tiny")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--prompt", type=int, default=5)
    ap.add_argument("--env", default="", help="VAR=VAL,... set before the engine is built (A/B variants)")
    a = ap.parse_args()
    for kv in filter(None, a.env.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    if a.model == "tiny":
        spec = S.tiny("t-q2", n_layers=3, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=1000,
                      bias=True)
        syn = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
    else:
        spec = S.QWEN2_7B.replace(n_layers=2)
        syn = W.SynthParams(seed=0)
    max_ctx = a.prompt + a.steps + 8
    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=a.fp8).init_synthetic(syn)
    hw = W.HostWeights.synthetic(spec, syn)
    if a.fp8:
        hw = hw.fp8_dequantized()
    om = O.Model(hw, max_ctx)
    b = eng.batch(1, max_ctx)
    prompt = [int(t) for t in np.random.default_rng(a.prompt).integers(0, spec.vocab, a.prompt)]
    lg = om.forward(prompt, 0)
    t_e = b.prefill(0, prompt)
    n = a.prompt
    for step in range(a.steps):
        first = None
        for layer in range(spec.n_layers):
            kg, vg = b.kv_rows(0, layer, n)
            for kind, g, o in (("V", vg, om.v[layer][:, :n]), ("K", kg, om.k[layer][:, :n])):
                d = ulps(g, o)
                if d.any() and first is None:
                    hs, ps, _ = np.nonzero(d)
                    first = f"layer {layer} {kind}: pos {int(ps.min())}, {int((d > 0).sum())} elems, max {int(d.max())} ulp"
        t_o = O.argmax(lg)
        print(f"step {step:2d} ctx {n:4d}  logits norm-rel {norm_rel(b.logits()[0], lg):.2e}  "
              f"id {'=' if t_e == t_o else 'FLIP'}  first KV mismatch: {first or 'none'}", flush=True)
        if t_e != t_o:
            b.set_position(0, n, t_o)
        t_e = b.decode_step()[0]
        lg = om.forward([t_o])
        n += 1


if __name__ == "__main__":
    main()
