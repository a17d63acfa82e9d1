"""CPU check of the forced-decision parity protocol (tests/parity.py forced_decisions) that
bench.py's full-depth gpu_parity and the 2-layer P = 2048 GPU twin use: an "engine" made of
the oracle itself in another summation order must pass the rule, and a wrong one (a
corrupted lm_head row block) must fail it.  The host logic only — no GPU."""
import numpy as np

from parity import PEAKED, forced_decisions

from qwen_inference_engine_amd import spec as S, weights as W


class OracleBatch:
    """The Batch calls forced_decisions makes, served by an oracle model in `order`."""

    def __init__(self, oracle, hw, max_ctx, order):
        self.O, self.order = oracle, order
        self.m = oracle.Model(hw, max_ctx)
        self.next = None

    def _fwd(self, ids, start):
        self.O.set_sum_order(self.order)
        try:
            self.lg = self.m.forward(ids, start)
        finally:
            self.O.set_sum_order(0)
        return self.O.argmax(self.lg)

    def prefill(self, seq, ids):
        return self._fwd(ids, 0)

    def logits(self):
        return self.lg[None, :]

    def set_position(self, seq, pos, tok):
        self.next = (pos, tok)

    def decode_step(self):
        pos, tok = self.next
        return [self._fwd([tok], pos)]


def _model(peaked=True):
    spec = S.tiny("proto", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=8192)
    syn = W.SynthParams(seed=4, **(PEAKED if peaked else {}))
    return spec, W.HostWeights.synthetic(spec, syn)


def test_boost_is_exact_power_of_two():
    spec, hw = _model(peaked=False)
    _, hb = _model(peaked=True)
    a, b = W.HostWeights.lm_head.fget(hw), W.HostWeights.lm_head.fget(hb)
    fa = (a.astype(np.uint32) << 16).view(np.float32)
    fb = (b.astype(np.uint32) << 16).view(np.float32)
    rows = np.arange(a.shape[0]) % PEAKED["head_boost_every"] == 0
    assert np.array_equal(fb[rows], fa[rows] * 2.0 ** PEAKED["head_boost_log2"])
    assert np.array_equal(fb[~rows], fa[~rows])


def test_another_summation_order_passes(oracle):
    spec, hw = _model()
    prompt = [int(t) for t in np.random.default_rng(3).integers(0, spec.vocab, 12)]
    rep = forced_decisions(oracle, hw, OracleBatch(oracle, hw, 96, order=2), prompt, 24)
    assert rep["ok"], rep
    assert rep["decisions"] == 24 and rep["hard_mismatches"] == 0
    # the engine here IS oracle order 2: its id disagreements are the oracle's own
    assert rep["gpu_vs_o0_id_disagreements"] == rep["oracle_o2_vs_o0_id_disagreements"]


def test_corrupted_head_fails(oracle):
    spec, hw = _model()
    bad = W.HostWeights(spec, dict(hw.tensors))
    name = "model.embed_tokens.weight" if spec.tie_embeddings else "lm_head.weight"
    w = bad.tensors[name].copy()
    w[::4096] = 0        # the boosted rows lost: the engine's picks move off them
    bad.tensors[name] = w
    prompt = [int(t) for t in np.random.default_rng(3).integers(0, spec.vocab, 12)]
    rep = forced_decisions(oracle, hw, OracleBatch(oracle, bad, 96, order=0), prompt, 12)
    assert not rep["ok"] and (rep["hard_mismatches"] > 0 or rep["max_norm_rel"] > rep["bar"]), rep
