"""Shared by tests/test_hf_golden.py (oracle, CPU) and tests/test_gpu_hf.py (engine, GPU):
the transformers fixtures of tools/make_hf_golden.py and the rule they are checked with.

Rule (the repository's end-to-end parity rule, tests/parity.py, with transformers in the
place of oracle order 0): teacher-forced on the fixture's greedy continuation, every
decision's bf16 logits within max(1e-3, 2 x the run's max norm-relative spread between
oracle summation orders 0 and 2 in hf numerics) of transformers', and every greedy id equal
to transformers' except near-ties whose transformers top-2 gap is within max(2 bf16 ulps
of max|logit|, the run's max absolute order-0 / order-2 logit spread), at most
max_flips(decisions) of them."""
import json
import os

import numpy as np

import gpu_util as G
from parity import NORM_REL, SPREAD_FACTOR, max_flips, norm_rel

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["hf_qwen2_tiny", "hf_qwen3_tiny", "hf_qwen2_tied"]


def load(name):
    from qwen_inference_engine_amd import spec as S, weights as W
    z = np.load(os.path.join(GOLD, name + ".npz"))
    cfg = json.loads(str(z["config"]))
    spec = S.ModelSpec.from_hf_config(cfg, name=name, numerics="hf")
    syn = W.SynthParams(**json.loads(str(z["synth"])))
    return spec, syn, [int(t) for t in z["prompt"]], [int(t) for t in z["ids"]], z["logits"]


def oracle_spread(oracle, hw, prompt, ids):
    """Orders 0 and 2 of the oracle (hf numerics, transformers' eager attention form — the
    fixtures') teacher-forced on `ids`: (order-0 logits per step, max norm-relative spread,
    max absolute spread)."""
    n = len(ids)
    outs = {}
    for o in (0, 2):
        oracle.set_sum_order(o)
        oracle.set_hf_eager(1)   # the fixtures' attention form (transformers eager)
        try:
            m = oracle.Model(hw, len(prompt) + n + 2)
            lg = [m.forward(prompt, 0)]
            for t in ids[:-1]:
                lg.append(m.forward([t]))
        finally:
            oracle.set_sum_order(0)
            oracle.set_hf_eager(0)
        outs[o] = lg
    rel = max(norm_rel(a, b) for a, b in zip(outs[2], outs[0]))
    ab = max(float(np.abs(G.bf(a).astype(np.float64) - G.bf(b)).max()) for a, b in zip(outs[2], outs[0]))
    return outs[0], rel, ab


def check(got_logits, got_ids, hf_ids, hf_logits, spread_rel, spread_abs, what):
    """Applies the rule; returns the report dict (report["ok"])."""
    bar = max(NORM_REL, SPREAD_FACTOR * spread_rel)
    rels, flips, hard = [], 0, 0
    for i, (lg, t) in enumerate(zip(got_logits, got_ids)):
        rels.append(norm_rel(lg, hf_logits[i]))
        if t != hf_ids[i]:
            f = G.bf(hf_logits[i]).astype(np.float64)
            gap = abs(f[hf_ids[i]] - f[t])
            if gap <= max(2 * 2.0 ** -7 * np.abs(f).max(), spread_abs):
                flips += 1
            else:
                hard += 1
    rep = {"what": what, "max_norm_rel_vs_transformers": round(max(rels), 6), "bar": round(bar, 6),
           "oracle_o2_spread": round(spread_rel, 6), "id_flips": flips, "hard_mismatches": hard,
           "decisions": len(got_ids)}
    rep["ok"] = bool(max(rels) <= bar and hard == 0 and flips <= max_flips(len(got_ids)))
    return rep
