"""GPU: the block-scaled fp8 MFMA prefill path — BASELINE config 4's "CDNA4 fp8 MFMA"
(qie_ops.h QIE_LINEAR_ACT_FP8, the engine's prefill_fp8 numerics flag; replaced op
matrix_mul.cu:165-288) — against the oracle's fp8-activation mode (or_set_act_fp8):

* qie_quantize_rows_fp8 == or_quant_rows_fp8 bit for bit (exponents and dequantised values);
* qie_linear with fp8 activations (plain and 16-row tiled fp8 weights; STORE + bias over three
  segments, SWIGLU, RESIDUAL, F32; split-K and full-chip grids) == the oracle's matmul of the
  dequantised operands within MX_ACC_REL of sum|a w| (every e4m3 x e4m3 product is exact; the
  instruction's internal sum is not fp32-exact, tools/mx_mfma_probe.hip);
* the engine (Qwen2-7B widths, 2 layers, fp8 weights, prefill_fp8) teacher-forced against the
  oracle with the same activation quantisation in its prefill (tests/parity.py's bar, whose
  second evaluation is then oracle order 8: order 2 + the MFMA accumulation model).
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as G
from conftest import rng
from parity import OrderPair, check_step, max_flips, oracle_trace
from test_gpu_ops import _abs_scale, rand_bf16

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W
from qwen_inference_engine_amd._lib import LinearArgsC

pytestmark = pytest.mark.gpu

# The fp8 MFMA's own accumulation is not fp32-exact: tools/mx_mfma_probe.hip measures one
# v_mfma_scale_f32_16x16x128_f8f6f4 at up to 1.5e-4 of sum|p| from the exact sum of its 128
# (exact) products on random e4m3 data.  The op bar is therefore this fraction of sum|a w|
# (besides one bf16 ulp), not the 1e-5 of the bf16 GEMMs.
MX_ACC_REL = 5e-4


def _quant_dev(qlib, x):
    """x bf16 [M, K] on the device -> (codes, e8m0 exps) device buffers."""
    M, K = x.shape
    q = G.zeros((M * K,), np.uint8)
    e = G.zeros((max(M, 16),), np.uint8)
    G.check(qlib.qie_quantize_rows_fp8(G.p(G.dev(x)), K, M, K, G.p(q), K, G.p(e), None), "quantize_rows_fp8")
    return q, e


def _fp8w(qlib, w, tiled):
    rows, cols = w.shape
    d = G.zeros((int(qlib.qie_fp8_weight_bytes(rows, cols)),), np.uint8)
    G.check(qlib.qie_quantize_fp8(G.p(G.dev(w)), rows, cols, G.p(d), None))
    if tiled:
        t = G.zeros((d.nbytes,), np.uint8)
        G.check(qlib.qie_fp8_tile16(G.p(d), rows, cols, G.p(t), None))
        d = t
    return d, W.dequantize_fp8(*W.quantize_fp8(w))


def _mx_linear(qlib, q, e, segs, biases, M, K, N, y, epi, tiled, ldy=None):
    a = LinearArgsC()
    a.x, a.ldx, a.x_exps = G.p(q), K, G.p(e)
    for i, s in enumerate(segs):
        a.w[i] = G.p(s[0])
        a.seg_rows[i] = s[1]
    for i, b in enumerate(biases):
        a.bias[i] = G.p(b) if b is not None else None
    a.M, a.K, a.N = M, K, N
    a.y, a.ldy = G.p(y), ldy or N
    a.epilogue = epi
    a.flags = _lib.QIE_LINEAR_FP8 | _lib.QIE_LINEAR_ACT_FP8 | (_lib.QIE_LINEAR_FP8_T16 if tiled else 0)
    G.check(qlib.qie_linear(C.byref(a), None), "qie_linear act_fp8")


@pytest.mark.parametrize("M,K", [(37, 3584), (5, 18944), (300, 896)])
def test_quantize_rows_fp8_matches_oracle(oracle, qlib, M, K):
    x = rand_bf16(oracle, (M, K), seed=M)
    xf = oracle.bf16_to_f32(x) * np.logspace(-20, 20, M, base=2.0).astype(np.float32)[:, None]
    x = oracle.f32_to_bf16(xf.astype(np.float32))
    x[M // 2] = 0                       # an all-zero row: scale 1, zero codes
    # a tiny-amax row: its scale would be a subnormal float below 2^-126 (exponent field 0);
    # clamped to 2^-126 on both sides
    x[1] = oracle.f32_to_bf16((oracle.bf16_to_f32(rand_bf16(oracle, (K,), seed=3)) * 2.0 ** -121).astype(np.float32))
    q, e = _quant_dev(qlib, x)
    codes = G.host(q).reshape(M, K)
    ex = G.host(e)[:M].astype(np.int64) - 127
    dq_or, e_or = oracle.quant_rows_fp8(x)
    assert np.array_equal(ex, e_or)
    assert ex.min() >= -126 and e_or[1] == -126
    got = W.e4m3_table()[codes].astype(np.float64) * np.exp2(ex.astype(np.float64))[:, None]
    assert np.array_equal(got, oracle.bf16_to_f32(dq_or).astype(np.float64))


@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("M,K,n", [(5, 256, (64, 32, 32)), (256, 3584, (512, 128, 128)),
                                   (700, 3584, (3584, 512, 512)), (300, 18944, (3584, 0, 0))])
def test_linear_act_fp8_store_bias(oracle, qlib, tiled, M, K, n):
    n = tuple(r for r in n if r)
    x = rand_bf16(oracle, (M, K), seed=M + K)
    ws = [rand_bf16(oracle, (r, K), 0.05, seed=10 + i) for i, r in enumerate(n)]
    bs = [rand_bf16(oracle, (r,), 0.1, seed=20 + i) for i, r in enumerate(n)]
    qw = [_fp8w(qlib, w, tiled) for w in ws]
    N = sum(n)
    dqx, _ = oracle.quant_rows_fp8(x)
    want = np.concatenate([oracle.matmul(dqx, dq, b) for (_, dq), b in zip(qw, bs)], axis=1)
    q, e = _quant_dev(qlib, x)
    y = G.zeros_bf16(M, N)
    _mx_linear(qlib, q, e, [(d, r) for (d, _), r in zip(qw, n)], [G.dev(b) for b in bs], M, K, N, y,
               _lib.QIE_EPI_STORE, tiled)
    scale = np.concatenate([_abs_scale(oracle, dqx, dq) for _, dq in qw], axis=1)
    G.assert_sum_close(G.host_bf16(y), want, scale, rel=MX_ACC_REL, what=f"act_fp8 M={M} K={K} tiled={tiled}")


@pytest.mark.parametrize("tiled", [False, True])
def test_linear_act_fp8_full_chip_grid(oracle, qlib, tiled):
    """2,048 rows x 8,192 columns: 256 tiles of 256x256, one round, no split — checked on a
    sample of rows (the per-row quantisation makes a row's result independent of the others)."""
    M, K, N = 2048, 3584, 8192
    x = rand_bf16(oracle, (M, K), seed=5)
    d, dq = _fp8w(qlib, rand_bf16(oracle, (N, K), 0.05, seed=6), tiled)
    q, e = _quant_dev(qlib, x)
    y = G.zeros_bf16(M, N)
    _mx_linear(qlib, q, e, [(d, N)], [None], M, K, N, y, _lib.QIE_EPI_STORE, tiled)
    rows = np.array([0, 1, 255, 256, 1000, 1023, 1777, 2047])
    dqx, _ = oracle.quant_rows_fp8(x[rows])
    want = oracle.matmul(dqx, dq)
    G.assert_sum_close(G.host_bf16(y)[rows], want, _abs_scale(oracle, dqx, dq), rel=MX_ACC_REL,
                       what="act_fp8 full grid")


@pytest.mark.parametrize("M", [40, 600])
@pytest.mark.parametrize("tiled", [False, True])
def test_linear_act_fp8_swiglu_residual_f32(oracle, qlib, M, tiled):
    """SWIGLU: the epilogue on the kernel's own accumulators — the gate and up halves run as
    STORE launches of the same kernel (K = 896: 7 k-tiles, no split in either launch, so every
    accumulator sees the same MFMA sequence) and the SWIGLU output must equal the oracle's
    silu_mul of those bf16 halves (within one ulp: device vs host expf); the halves against
    the oracle's matmul under MX_ACC_REL.  RESIDUAL and F32 (the down projection's two
    epilogues) against the oracle under the same accumulation bar."""
    K, I = 896, 640
    x = rand_bf16(oracle, (M, K), seed=6)
    (dg, qg), (du, qu) = _fp8w(qlib, rand_bf16(oracle, (I, K), 0.08, seed=7), tiled), \
        _fp8w(qlib, rand_bf16(oracle, (I, K), 0.08, seed=8), tiled)
    dqx, _ = oracle.quant_rows_fp8(x)
    q, e = _quant_dev(qlib, x)
    halves = []
    for d_, q_ in ((dg, qg), (du, qu)):
        yh = G.zeros_bf16(M, I)
        _mx_linear(qlib, q, e, [(d_, I)], [None], M, K, I, yh, _lib.QIE_EPI_STORE, tiled)
        halves.append(G.host_bf16(yh))
        G.assert_sum_close(halves[-1], oracle.matmul(dqx, q_), _abs_scale(oracle, dqx, q_), rel=MX_ACC_REL,
                           what="act_fp8 gate/up half")
    y = G.zeros_bf16(M, I)
    _mx_linear(qlib, q, e, [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU, tiled)
    d = G.ulp_diff(G.host_bf16(y), oracle.silu_mul(halves[0], halves[1]))
    assert d.max() <= 1 and (d == 0).mean() > 0.99, f"SWIGLU epilogue: max {d.max()} ulps"
    # residual and fp32 partial epilogues (the down projection; K = I)
    dw, qw = _fp8w(qlib, rand_bf16(oracle, (K, I), 0.02, seed=4), tiled)
    h = rand_bf16(oracle, (M, I), seed=3)
    res = rand_bf16(oracle, (M, K), seed=5)
    dqh, _ = oracle.quant_rows_fp8(h)
    want = oracle.resadd(res, oracle.matmul(dqh, qw))
    hq, he = _quant_dev(qlib, h)
    yr = G.dev(res)
    _mx_linear(qlib, hq, he, [(dw, K)], [], M, I, K, yr, _lib.QIE_EPI_RESIDUAL, tiled)
    acc = G.bf(oracle.matmul(dqh, qw)).astype(np.float64)
    sc = _abs_scale(oracle, dqh, qw)
    tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + MX_ACC_REL * sc
    assert (np.abs(G.bf(G.host_bf16(yr)).astype(np.float64) - G.bf(want)) <= tol).all()
    yf = G.zeros((M, K), np.float32)
    _mx_linear(qlib, hq, he, [(dw, K)], [], M, I, K, yf, _lib.QIE_EPI_F32, tiled)
    exact = oracle.bf16_to_f32(dqh).astype(np.float64) @ oracle.bf16_to_f32(qw).astype(np.float64).T
    assert (np.abs(G.host(yf) - exact) <= MX_ACC_REL * sc + 1e-6).all()


def test_linear_act_fp8_rejects_bad_shapes(qlib):
    """K not a multiple of 128, or bf16 weights: refused, nothing launched."""
    M, K, N = 64, 896 + 64, 128
    x, y = G.zeros((M * K,), np.uint8), G.zeros_bf16(M, N)
    e = G.zeros((M,), np.uint8)
    w = G.zeros((int(qlib.qie_fp8_weight_bytes(N, K)),), np.uint8)
    with pytest.raises(_lib.QieError):
        _mx_linear(qlib, x, e, [(w, N)], [], M, K, N, y, _lib.QIE_EPI_STORE, False)
    a = LinearArgsC()
    a.x, a.ldx, a.x_exps = G.p(x), 896, G.p(e)
    a.w[0], a.seg_rows[0] = G.p(w), N
    a.M, a.K, a.N, a.y, a.ldy = M, 896, N, G.p(y), N
    a.flags = _lib.QIE_LINEAR_ACT_FP8   # bf16 weights
    assert qlib.qie_linear(C.byref(a), None) != 0


def _engine_vs_oracle(oracle, spec, syn, prompts, n_new, max_ctx, batched):
    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=True, prefill_fp8=True).init_synthetic(syn)
    B = len(prompts)
    b = eng.batch(B, max_ctx)
    hw = W.HostWeights.synthetic(spec, syn).fp8_dequantized()
    oms = [OrderPair(oracle, hw, max_ctx, with_spread=(i == 0), act_fp8=True) for i in range(B)]
    traces = [oracle_trace(oracle, om, pr, n_new) for om, pr in zip(oms, prompts)]
    t_e = b.prefill_batch(0, prompts) if batched else [b.prefill(i, pr) for i, pr in enumerate(prompts)]
    flips = 0
    first = None
    for step in range(n_new):
        lg_e = b.logits()
        if step == 0:
            first = lg_e.copy()
        for i in range(B):
            ids, outs = traces[i]
            lg0 = outs[step][0]
            flips += check_step(lg_e[i], lg0, None, t_e[i], ids[step], f"seq {i} step {step}", oms[0].bars(lg0))
            if t_e[i] != ids[step]:
                b.set_position(i, len(prompts[i]) + step, ids[step])
        if step + 1 < n_new:
            t_e = b.decode_step()
    assert flips <= max_flips(B * n_new)
    b.close()
    eng.close()
    return hw, first


def test_engine_prefill_fp8_qwen2_7b_widths_p1024(oracle):
    """Config 4's shape at batch 1: Qwen2-7B widths (2 layers), e4m3 weights (tiled decode
    layout, read by the fp8 GEMM too), a 1,024-token prompt through the block-scaled fp8 prefill,
    then graph decode — against the oracle with the same activation quantisation.  Also
    prints the model change the flag makes: the first decision's logits against the
    bf16-activation oracle (dequantised weights), the number DESIGN.md §3 quotes."""
    spec = S.QWEN2_7B.replace(n_layers=2)
    syn = W.SynthParams(seed=0)
    P, n_new, max_ctx = 1024, 6, 1040
    prompt = [int(t) for t in rng(1024).integers(0, spec.vocab, P)]
    hw, first = _engine_vs_oracle(oracle, spec, syn, [prompt], n_new, max_ctx, False)
    from parity import norm_rel
    lg_bf16 = oracle.Model(hw, max_ctx).forward(prompt, 0)
    print(f"prefill_fp8 vs bf16-activation oracle (first decision): norm-rel {norm_rel(first[0], lg_bf16):.4e}")


def test_engine_prefill_fp8_batched_tiny(oracle):
    """qie_prefill_batch with fp8 activations (4 equal-length prompts in one pass, per-row
    quantisation) == each sequence against its own oracle trace."""
    spec = S.tiny("t-mx", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=1024,
                  bias=True)
    syn = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
    prompts = [[int(t) for t in rng(50 + i).integers(0, spec.vocab, 70)] for i in range(4)]
    _engine_vs_oracle(oracle, spec, syn, prompts, 6, 96, True)
