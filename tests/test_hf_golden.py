"""CPU: the oracle's HF numerics mode pinned to transformers (tests/golden/hf_*.npz, made by
tools/make_hf_golden.py from the local transformers' Qwen2ForCausalLM / Qwen3ForCausalLM on
the repository's synthetic weights).  Rule: tests/hf_golden.py."""
import pytest

import hf_golden as H


@pytest.mark.parametrize("name", H.CASES)
def test_oracle_hf_mode_matches_transformers(oracle, name):
    from qwen_inference_engine_amd import weights as W
    spec, syn, prompt, ids, logits = H.load(name)
    hw = W.HostWeights.synthetic(spec, syn)
    lg0, rel, ab = H.oracle_spread(oracle, hw, prompt, ids)
    rep = H.check(lg0, [oracle.argmax(x) for x in lg0], ids, logits, rel, ab, f"oracle hf vs transformers, {name}")
    print(rep)
    assert rep["ok"], rep


def test_hf_fixture_configs_map_to_specs():
    """The fixtures' HF configs go through ModelSpec.from_hf_config, the converter's path."""
    for name in H.CASES:
        spec, _, prompt, ids, logits = H.load(name)
        assert spec.numerics == "hf" and logits.shape == (len(ids), spec.vocab)
    assert H.load("hf_qwen3_tiny")[0].qk_norm and not H.load("hf_qwen3_tiny")[0].qkv_bias
    assert H.load("hf_qwen2_tied")[0].tie_embeddings
