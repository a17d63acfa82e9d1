"""GPU: the persistent decode step (qie_batch_set_decode_mode(b, 1), k_persist.hip) against the
five-launch step it replaces (mode 0), BIT FOR BIT, and against the oracle.

Mode 1 runs every layer of a batch-1 decode step in ONE launch: each CU streams its rows of
every projection with the launch path's exact per-lane fp32 order, the RMSNorms in the launch
path's orders, the attention as the stand-alone kernel's body (8 waves at head_dim 128, 4 at 64),
and hands activations
between CUs as tagged granules.  Every output is therefore the same bytes as mode 0's — ids and
logits are compared for equality, not within a tolerance.  Contexts cover one split (ctx <=
256), the 1 -> 3 split change at 257, and 16 -> 17 splits around 2,048 (the headline's range);
numerics REF and HF; Qwen2 (q/k/v bias) and Qwen3 (qk-norm) forms.  Mode 0 itself is pinned to
the oracle by test_gpu_engine.py / test_gpu_headline.py; one run here is also checked against
the oracle directly (tests/parity.py forced_decisions).

Reference loop replaced: llm()'s decode branch, layers/src/qwen_main.cu:271-359."""
import numpy as np
import pytest

from conftest import rng
from parity import PEAKED, forced_decisions

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W

pytestmark = pytest.mark.gpu

QWEN3_T = S.tiny("t-q3-128", n_layers=3, hidden=1024, n_heads=8, n_kv_heads=2, head_dim=128, ffn=2048, vocab=4096,
                 bias=False, qk_norm=True)
SYN = W.SynthParams(seed=5, w_scale=0.05, norm_scale=0.25, bias_scale=0.05)


def _gen(b, prompt, steps, mode):
    b.set_decode_mode(mode)
    assert b.decode_mode == mode
    ids = [b.prefill(0, prompt)]
    lgs = [b.logits()]
    for _ in range(steps):
        ids.append(int(b.decode_step()[0]))
        lgs.append(b.logits())
    return ids, np.stack(lgs)


@pytest.mark.parametrize("spec,P,steps", [
    (S.QWEN2_7B.replace(n_layers=2), 20, 260),      # one split -> three splits at ctx 257
    (S.QWEN2_7B.replace(n_layers=2), 2040, 24),     # 16 -> 17 splits at ctx 2,049
    (QWEN3_T, 100, 170),                            # qk-norm, no bias, 4 q heads per kv head
    (QWEN3_T.replace(numerics="hf"), 60, 80),       # HF numerics (rotate_half RoPE, HF norms)
    (S.QWEN2_0_5B.replace(n_layers=3), 128, 140),   # hd 64 (4-wave workgroups), config 2's ctx 129..
], ids=["qwen2-7b-short", "qwen2-7b-2k", "qwen3-qknorm", "qwen3-hf", "qwen2-0.5b"])
def test_persistent_equals_launches(spec, P, steps):
    syn = SYN if spec.hidden < 2048 else W.SynthParams(seed=0)
    max_ctx = P + steps + 8
    eng = Q.Engine(spec, max_ctx=max_ctx).init_synthetic(syn)
    prompt = [int(t) for t in rng(P).integers(0, spec.vocab, P)]
    a = _gen(eng.batch(1, max_ctx), prompt, steps, 0)
    b = _gen(eng.batch(1, max_ctx), prompt, steps, 1)
    assert a[0] == b[0]
    bad = [i for i in range(len(a[1])) if not np.array_equal(a[1][i], b[1][i])]
    assert not bad, f"logits differ at steps {bad[:8]} (of {len(bad)})"


def test_persistent_mode_switch_and_refusals():
    """Switching modes mid-sequence continues the same sequence bit for bit (the graph is
    re-captured); batches the persistent step does not cover are refused with a reason."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    eng = Q.Engine(spec, max_ctx=512).init_synthetic(W.SynthParams(seed=0))
    prompt = [int(t) for t in rng(3).integers(0, spec.vocab, 77)]
    ref = eng.batch(1, 512)
    want = [ref.prefill(0, prompt)] + [int(t) for t in ref.decode(40)[:, 0]]
    b = eng.batch(1, 512)
    got = [b.prefill(0, prompt)]
    for i in range(40):
        b.set_decode_mode(1 if (i // 7) % 2 == 0 else 0)
        got.append(int(b.decode_step()[0]))
    assert got == want
    with pytest.raises(_lib.QieError, match="batch != 1"):
        eng.batch(2, 512).set_decode_mode(1)
    with pytest.raises(_lib.QieError, match="paged"):
        eng.batch(1, 512, page_tokens=128).set_decode_mode(1)
    small = Q.Engine(S.tiny("t32", n_layers=1, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512,
                            vocab=512), max_ctx=64).init_synthetic(SYN)
    with pytest.raises(_lib.QieError, match="hidden / 2 < CUs"):
        small.batch(1, 64).set_decode_mode(1)


def test_persistent_forced_decisions_vs_oracle(oracle):
    """Mode 1 against the oracle directly (tests/parity.py forced_decisions: orders 0/1/2,
    peaked head), Qwen2-7B widths, 2 layers, a 300-token prompt, 48 teacher-forced decisions."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    syn = W.SynthParams(seed=0, **PEAKED)
    eng = Q.Engine(spec, max_ctx=400).init_synthetic(syn)
    b = eng.batch(1, 400)
    b.set_decode_mode(1)
    prompt = [int(t) for t in rng(300).integers(0, spec.vocab, 300)]
    rep = forced_decisions(oracle, W.HostWeights.synthetic(spec, syn), b, prompt, 48)
    print("persistent forced decisions:", rep)
    assert rep["ok"], rep
