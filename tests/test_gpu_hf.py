"""GPU: the engine's HF numerics mode against transformers (tests/golden/hf_*.npz, made by
tools/make_hf_golden.py from the local transformers' Qwen2ForCausalLM / Qwen3ForCausalLM
on the same synthetic weights the engine generates on the device).  Prefill, then hipGraph
decode steps teacher-forced on transformers' greedy continuation; rule: tests/hf_golden.py
(logits within max(1e-3, 2 x the oracle's own order-0 / order-2 spread in hf numerics) of
transformers', ids equal except bounded near-ties)."""
import pytest

import hf_golden as H

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import weights as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", H.CASES)
@pytest.mark.parametrize("graph", [True, False])
def test_engine_hf_mode_matches_transformers(oracle, name, graph):
    spec, syn, prompt, ids, logits = H.load(name)
    max_ctx = len(prompt) + len(ids) + 8
    eng = Q.Engine(spec, max_ctx=max_ctx, use_graph=graph).init_synthetic(syn)
    b = eng.batch(1, max_ctx)
    got_ids, got_lg = [b.prefill(0, prompt)], []
    for i in range(len(ids)):
        got_lg.append(b.logits()[0].copy())
        if i + 1 < len(ids):
            if got_ids[-1] != ids[i]:
                b.set_position(0, len(prompt) + i, ids[i])
            got_ids.append(b.decode_step()[0])
    b.close()
    eng.close()
    hw = W.HostWeights.synthetic(spec, syn)
    _, rel, ab = H.oracle_spread(oracle, hw, prompt, ids)
    rep = H.check(got_lg, got_ids, ids, logits, rel, ab, f"engine hf vs transformers, {name}, graph={graph}")
    print(rep)
    assert rep["ok"], rep
