"""GPU parity at the BASELINE configurations' real shapes, against the CPU oracle.

* Config 3 (headline, Qwen2-7B bf16, B = 1, P = 2048): the engine's real dispatch —
  2048-row LDS-DMA GEMMs with their XCD remap, flash prefill attention over 2048 keys,
  then 63 hipGraph decode steps at ctx 2049..2111 whose fused attention runs 17+ live
  splits — on Qwen2-7B widths (2 layers): 64 greedy decisions on a forced continuation
  against or_forward in summation orders 0 / 1 / 2 (tests/parity.py forced_decisions, the
  2-layer twin of bench.py's full-depth gpu_parity; qwen_main.cu:74-247 prefill,
  :250-405 decode).
* Decode attention at ctx 1500 / 2560 / 4097 / 8192 (up to 32 splits, 2-step splits).
* Prefill attention at P = 2048; the big GEMMs at M = 2048 with Qwen2-7B's K / N.
* Config 4 (Qwen2-7B fp8 weights, B = 8, P = 1024): 8 prompts of 1024 tokens, batched
  graph decode, against the oracle on the dequantised weights.

Bars (written per check): end-to-end, tests/parity.py — logits within max(1e-3,
2 x the oracle's own order-0 vs order-2 norm-relative spread on the same input), greedy
ids equal (teacher-forced) except near-ties within the oracle's own order spread
(counted, bounded).  Ops: the tolerances of tests/test_gpu_ops.py."""
import ctypes as C

import numpy as np
import pytest

import gpu_util as G
from conftest import rng
from test_gpu_ops import _cache, _linear, _abs_scale, rand_bf16
from parity import PEAKED, OrderPair, check_step, forced_decisions, max_flips, oracle_trace

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W

pytestmark = pytest.mark.gpu

def test_headline_forced_decisions_2layers_p2048(oracle):
    """The 2-layer twin of bench.py's full-depth gpu_parity (tests/parity.py
    forced_decisions, same rule): Qwen2-7B widths, peaked head, a 2048-token prompt
    (LDS-DMA GEMMs, flash prefill attention) then 63 graph decode steps at ctx 2049..2111
    on a seeded random continuation — 64 greedy decisions against oracle orders 0 / 1 / 2."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    syn = W.SynthParams(seed=0, **PEAKED)
    P, n, max_ctx = 2048, 64, 2176
    eng = Q.Engine(spec, max_ctx=max_ctx, use_graph=True).init_synthetic(syn)
    b = eng.batch(1, max_ctx)
    prompt = [int(t) for t in rng(2048).integers(0, spec.vocab, P)]
    rep = forced_decisions(oracle, W.HostWeights.synthetic(spec, syn), b, prompt, n, progress=True)
    print("forced decisions (2 layers, P 2048):", rep)
    assert rep["ok"], rep


@pytest.mark.parametrize("hd,nq,nkv", [(128, 28, 4), (64, 14, 2)])
@pytest.mark.parametrize("qkn", [False, True])
def test_attention_decode_fused_long_context(oracle, qlib, hd, nq, nkv, qkn):
    """Fused decode attention at long context: ctx 1500 / 2560 (17-20 splits of 128
    keys), 4097 and 8192 (capped splits, several 128-key steps per split)."""
    ctxs = [1500, 2560, 4097, 8192]
    L, layer, maxc, num = 2, 1, 8200, "ref"
    B = len(ctxs)
    QD, KD = nq * hd, nkv * hd
    seq_stride = L * nkv * maxc * hd
    kc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq)
    vc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq + 1)
    qkv = rand_bf16(oracle, (B, QD + 2 * KD), seed=5)
    pos = np.array(ctxs, np.int32) - 1
    eps = 1e-4
    qn = oracle.f32_to_bf16((1 + 0.3 * rng(1).standard_normal(hd)).astype(np.float32)) if qkn else None
    kn = oracle.f32_to_bf16((1 + 0.3 * rng(2).standard_normal(hd)).astype(np.float32)) if qkn else None
    cs, sn = oracle.rope_table(maxc, hd, 1e6, num)
    q, k, v = qkv[:, :QD].copy(), qkv[:, QD:QD + KD].copy(), qkv[:, QD + KD:].copy()
    if qkn:
        q = oracle.qknorm(q, qn, nq, hd, eps, num)
        k = oracle.qknorm(k, kn, nkv, hd, eps, num)
    q = oracle.rope(q, cs, sn, pos, nq, hd, num)
    k = oracle.rope(k, cs, sn, pos, nkv, hd, num)
    ws = G.zeros_bytes(qlib.qie_attention_decode_workspace_bytes(B, nq, nkv, hd, maxc))
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    out = G.zeros_bf16(B, QD)
    c = _cache(kc, vc, L, nkv, hd, maxc, seq_stride)
    dqn, dkn = (G.dev(qn), G.dev(kn)) if qkn else (None, None)
    G.check(qlib.qie_attention_decode(G.p(G.dev(qkv)), B, G.p(G.dev(pos)), G.p(dqn), G.p(dkn), G.p(G.dev(cs)),
                                      G.p(G.dev(sn)), nq, C.byref(c), layer, eps, 0, G.p(out), G.p(ws), None))
    got = G.host_bf16(out)
    for i in range(B):
        p = pos[i]
        kk = kc_h[i, layer, :, :p + 1].copy()
        vv = vc_h[i, layer, :, :p + 1].copy()
        kk[:, p] = k[i].reshape(nkv, hd)
        vv[:, p] = v[i].reshape(nkv, hd)
        want = oracle.attention(q[i:i + 1], kk, vv, nq, nkv, hd, False, 0)
        d = np.abs(G.bf(got[i]) - G.bf(want[0]))
        assert d.max() <= 2 ** -7 * max(1.0, np.abs(G.bf(want[0])).max()) * 2, f"ctx {ctxs[i]}: {d.max()}"
    assert not G.host(ws)[:B * nkv * 4].any()   # split tickets left zeroed


@pytest.mark.parametrize("hd,nq,nkv", [(128, 28, 4), (64, 14, 2)])
def test_attention_prefill_causal_2048(oracle, qlib, hd, nq, nkv):
    P, L, layer, maxc = 2048, 1, 0, 2048
    seq_stride = L * nkv * maxc * hd
    kc_h = rand_bf16(oracle, (1, L, nkv, maxc, hd), seed=11)
    vc_h = rand_bf16(oracle, (1, L, nkv, maxc, hd), seed=12)
    q = rand_bf16(oracle, (P, nq * hd), seed=13)
    pos = np.arange(P, dtype=np.int32)
    ws = G.zeros_bytes(qlib.qie_attention_workspace_bytes(P, nq, hd, maxc))
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    out = G.zeros_bf16(P, nq * hd)
    c = _cache(kc, vc, L, nkv, hd, maxc, seq_stride)
    G.check(qlib.qie_attention(G.p(G.dev(q)), P, G.p(G.dev(pos)), P, C.byref(c), layer, nq, G.p(out), G.p(ws), None))
    want = oracle.attention(q, kc_h[0, layer], vc_h[0, layer], nq, nkv, hd, True, 0)
    d = np.abs(G.bf(G.host_bf16(out)) - G.bf(want))
    assert d.max() <= 2 ** -6, d.max()


@pytest.mark.parametrize("what", ["qkv", "o", "gate_up", "down"])
def test_linear_at_prefill_2048(oracle, qlib, what):
    """The prefill GEMMs of Qwen2-7B at M = 2048 through qie_linear's real dispatch."""
    M, H, I = 2048, 3584, 18944
    x = rand_bf16(oracle, (M, I if what == "down" else H), seed=21)
    K = x.shape[1]
    if what == "qkv":
        n = (3584, 512, 512)
        ws = [rand_bf16(oracle, (r, K), 0.02, seed=30 + i) for i, r in enumerate(n)]
        bs = [rand_bf16(oracle, (r,), 0.1, seed=40 + i) for i, r in enumerate(n)]
        want = np.concatenate([oracle.matmul(x, w, b) for w, b in zip(ws, bs)], axis=1)
        y = G.zeros_bf16(M, sum(n))
        _linear(qlib, G.dev(x), list(zip([G.dev(w) for w in ws], n)), [G.dev(b) for b in bs], M, K, sum(n), y,
                _lib.QIE_EPI_STORE)
        scale = np.concatenate([_abs_scale(oracle, x, w) for w in ws], axis=1)
        G.assert_sum_close(G.host_bf16(y), want, scale, what="qkv M=2048")
    elif what == "gate_up":
        wg = rand_bf16(oracle, (I, K), 0.02, seed=7)
        wu = rand_bf16(oracle, (I, K), 0.02, seed=8)
        want = oracle.silu_mul(oracle.matmul(x, wg), oracle.matmul(x, wu))
        y = G.zeros_bf16(M, I)
        _linear(qlib, G.dev(x), [(G.dev(wg), I), (G.dev(wu), I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU)
        d = G.ulp_diff(G.host_bf16(y), want)
        assert (d == 0).mean() > 0.97 and (d <= 2).mean() > 0.999, f"exact {(d == 0).mean():.4f}"
    else:
        N = H
        w = rand_bf16(oracle, (N, K), 0.02, seed=4)
        res = rand_bf16(oracle, (M, N), seed=5)
        acc_b = oracle.matmul(x, w)
        want = oracle.resadd(res, acc_b)
        y = G.dev(res)
        _linear(qlib, G.dev(x), [(G.dev(w), N)], [], M, K, N, y, _lib.QIE_EPI_RESIDUAL)
        got = G.host_bf16(y)
        acc = G.bf(acc_b).astype(np.float64)
        tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, x, w)
        err = np.abs(G.bf(got).astype(np.float64) - G.bf(want))
        assert (err <= tol).all(), f"worst {(err - tol).max()}"


def test_config4_fp8_batch8_prompt1024(oracle):
    """BASELINE config 4 shape: Qwen2-7B widths (2 layers), e4m3 weights, 8 sequences of
    1024-token prompts, batched hipGraph decode (skinny MFMA kernel over fp8 weights)."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    syn = W.SynthParams(seed=0)
    B, P, n_new, max_ctx = 8, 1024, 4, 1040
    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=True).init_synthetic(syn)
    b = eng.batch(B, max_ctx)
    hw = W.HostWeights.synthetic(spec, syn).fp8_dequantized()
    prompts = [[int(t) for t in rng(300 + i).integers(0, spec.vocab, P)] for i in range(B)]
    # order-2 spread measured on sequence 0 (same model and depth) sizes every row's bar
    oms = [OrderPair(oracle, hw, max_ctx, with_spread=(i == 0)) for i in range(B)]
    traces = [oracle_trace(oracle, om, pr, n_new) for om, pr in zip(oms, prompts)]
    bar_pair = oms[0]
    t_e = [b.prefill(i, pr) for i, pr in enumerate(prompts)]
    flips = 0
    for step in range(n_new):
        lg_e = b.logits()
        for i in range(B):
            ids, outs = traces[i]
            lg0 = outs[step][0]
            flips += check_step(lg_e[i], lg0, None, t_e[i], ids[step], f"seq {i} step {step}", bar_pair.bars(lg0))
            if t_e[i] != ids[step]:
                b.set_position(i, P + step, ids[step])
        if step + 1 < n_new:
            t_e = b.decode_step()
    assert flips <= max_flips(B * n_new)


def test_fp8_tiled_batch1_short_prompt(oracle):
    """Qwen2-7B widths (2 layers), e4m3 weights at batch 1 with a 12-token prompt: every
    projection runs the batched-decode kernel on the engine's 16-row tiled weights (prefill
    of <= 16 rows and the M = 1 decode), against the oracle on the dequantised model."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    syn = W.SynthParams(seed=0)
    P, n_new, max_ctx = 12, 6, 32
    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=True).init_synthetic(syn)
    b = eng.batch(1, max_ctx)
    hw = W.HostWeights.synthetic(spec, syn).fp8_dequantized()
    prompt = [int(t) for t in rng(77).integers(0, spec.vocab, P)]
    om = OrderPair(oracle, hw, max_ctx)
    ids, outs = oracle_trace(oracle, om, prompt, n_new)
    t = b.prefill(0, prompt)
    flips = 0
    for step in range(n_new):
        lg0 = outs[step][0]
        flips += check_step(b.logits()[0], lg0, om, t, ids[step], f"step {step}")
        if t != ids[step]:
            b.set_position(0, P + step, ids[step])
        if step + 1 < n_new:
            t = b.decode_step()[0]
    assert flips <= max_flips(n_new)


# ---------------------------------------------------------------------------------------
# The exact config-4 path bench.py's configs.config4 times (verdict r05 item 1): fp8 weights,
# PAGED KV with 128-token pages, B = 8, 1,024-token prompts through qie_prefill_batch, graph
# decode at ctx 1,025.. — the B >= 8 split rule (splits target 8: two-step 256-key splits
# from ctx 1,025 on, k_attention.hip qie_attention_decode) on the paged kernel instance.
C4_SPEC = S.QWEN2_7B.replace(n_layers=2)
C4_B, C4_P, C4_STEPS = 8, 1024, 16
C4_MAXC = C4_P + 256 + 16   # bench.py config 4's max_ctx (P + G + 16)


def _c4_prompts():
    return [[int(t) for t in rng(400 + i).integers(0, C4_SPEC.vocab, C4_P)] for i in range(C4_B)]


def test_config4_paged_equals_contiguous_batch8():
    """Paged (128-token pages) == contiguous, bit for bit, at B = 8 over the page boundary
    at 1,024: the same batched prefill, then 16 free-running greedy graph steps (ctx 1,025 ..
    1,040); ids and every step's logits identical."""
    eng = Q.Engine(C4_SPEC, max_ctx=C4_MAXC, weight_fp8=True).init_synthetic(W.SynthParams(seed=0))
    prompts = _c4_prompts()
    runs = []
    for pt in (None, 128):
        b = eng.batch(C4_B, C4_MAXC, page_tokens=pt)
        ids = [b.prefill_batch(0, prompts)]
        lgs = [b.logits()]
        for _ in range(C4_STEPS):
            ids.append(list(b.decode_step()))
            lgs.append(b.logits())
        assert b.positions().tolist() == [C4_P + C4_STEPS] * C4_B
        runs.append((ids, np.stack(lgs)))
        b.close()
    assert runs[0][0] == runs[1][0]
    assert np.array_equal(runs[0][1], runs[1][1])


def test_config4_paged128_fp8_batch8_prompt1024_matches_oracle(oracle):
    """The bench's config-4 path against the oracle on the dequantised weights
    (tests/parity.py check_step, bar from the order-0 vs order-2 spread of sequence 0 on the
    same model): 8 prompts of 1,024 tokens in one batched prefill, then 16 teacher-forced
    graph decode steps per sequence (ctx 1,025 .. 1,040)."""
    syn = W.SynthParams(seed=0)
    eng = Q.Engine(C4_SPEC, max_ctx=C4_MAXC, weight_fp8=True).init_synthetic(syn)
    b = eng.batch(C4_B, C4_MAXC, page_tokens=128)
    hw = W.HostWeights.synthetic(C4_SPEC, syn).fp8_dequantized()
    prompts = _c4_prompts()
    oms = [OrderPair(oracle, hw, C4_MAXC, with_spread=(i == 0)) for i in range(C4_B)]
    traces = [oracle_trace(oracle, om, pr, C4_STEPS) for om, pr in zip(oms, prompts)]
    bar_pair = oms[0]
    t_e = b.prefill_batch(0, prompts)
    flips = 0
    for step in range(C4_STEPS):
        lg_e = b.logits()
        for i in range(C4_B):
            ids, outs = traces[i]
            lg0 = outs[step][0]
            flips += check_step(lg_e[i], lg0, None, t_e[i], ids[step], f"paged c4 seq {i} step {step}",
                                bar_pair.bars(lg0))
            if t_e[i] != ids[step]:
                b.set_position(i, C4_P + step, ids[step])
        if step + 1 < C4_STEPS:
            t_e = b.decode_step()
    assert flips <= max_flips(C4_B * C4_STEPS)
    assert b.page_stats()[2] == 128
