"""fp8 weights (BASELINE config "Qwen2-7B fp8 weights, batch 8"): OCP e4m3 codes with
power-of-two row scales, so each dequantised weight is exactly a bf16 and the fp8 engine
must compute what the oracle computes on the dequantised bf16 weights.

Bar: the device decode of all 256 codes equals the e4m3fn table bit-exactly; device
quantisation equals the host quantiser bit-exactly; fp8 GEMV / GEMM results meet the same
tolerances as the bf16 linear tests against oracle.matmul on the dequantised weights;
the fp8 engine's teacher-forced greedy run matches the oracle on the dequantised model
under tests/test_gpu_engine.py's bar.
"""
import numpy as np
import pytest

import gpu_util as G
from conftest import rng
from test_gpu_ops import _linear, _abs_scale, rand_bf16
from test_gpu_engine import forced_compare

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W

pytestmark = pytest.mark.gpu

SYN = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)


def test_fp8_decode_all_codes(qlib):
    out = G.zeros((256,), np.float32)
    G.check(qlib.qie_debug_fp8_decode(G.p(out)))
    got, want = G.host(out), W.e4m3_table()
    ok = ~np.isnan(want)
    assert np.array_equal(got[ok].view(np.uint32), want[ok].view(np.uint32))
    assert np.isnan(got[~ok]).all()


def test_fp8_decode_bf16_all_codes(qlib):
    """The MFMA GEMV's one-instruction decode (v_cvt_scalef32_pk_bf16_fp8, scale 1.0) gives
    the bf16 of every finite e4m3fn code bit-exactly (each is exactly a bf16), NaN for NaN."""
    out = G.zeros((256,), np.uint16)
    G.check(qlib.qie_debug_fp8_decode_bf16(G.p(out)))
    got, want = G.host(out), W.e4m3_table()
    ok = ~np.isnan(want)
    assert np.array_equal(got[ok], (want[ok].view(np.uint32) >> 16).astype(np.uint16))
    assert (want[ok].view(np.uint32) & 0xffff == 0).all()
    nan = got[~ok]
    assert ((nan & 0x7f80) == 0x7f80).all() and ((nan & 0x7f) != 0).all()


@pytest.mark.parametrize("rows,cols", [(7, 64), (33, 896), (5, 18944)])
def test_quantize_device_equals_host(oracle, qlib, rows, cols):
    w = rand_bf16(oracle, (rows, cols), 0.05, seed=rows)
    w[0] = 0                                                 # all-zero row: scale 1
    w[1 % rows, :3] = oracle.f32_to_bf16(np.array([1e4, -3e-3, 7.0], np.float32))
    nbytes = int(qlib.qie_fp8_weight_bytes(rows, cols))
    out = G.zeros((nbytes,), np.uint8)
    G.check(qlib.qie_quantize_fp8(G.p(G.dev(w)), rows, cols, G.p(out), None))
    G.check(qlib.qie_synchronize())
    codes, scales = W.quantize_fp8(w)
    got = G.host(out)
    assert np.array_equal(got[:rows * cols].reshape(rows, cols), codes)
    assert np.array_equal(got[rows * cols:].view(np.float32), scales)


@pytest.mark.parametrize("rows,cols", [(7, 64), (33, 896), (5, 18944)])
def test_dequantize_device_exact(oracle, qlib, rows, cols):
    """qie_dequantize_fp8 (the fp8 prefill's weight expansion) == the host dequantisation
    of the same codes, bit for bit (every e4m3 x power-of-two value is a bf16)."""
    w = rand_bf16(oracle, (rows, cols), 0.05, seed=rows + 1)
    w[0] = 0
    q = G.zeros((int(qlib.qie_fp8_weight_bytes(rows, cols)),), np.uint8)
    G.check(qlib.qie_quantize_fp8(G.p(G.dev(w)), rows, cols, G.p(q), None))
    out = G.zeros_bf16(rows, cols)
    G.check(qlib.qie_dequantize_fp8(G.p(q), rows, cols, G.p(out), None))
    assert np.array_equal(G.host_bf16(out), W.dequantize_fp8(*W.quantize_fp8(w)))


def _fp8_dev(qlib, w):
    rows, cols = w.shape
    out = G.zeros((int(qlib.qie_fp8_weight_bytes(rows, cols)),), np.uint8)
    G.check(qlib.qie_quantize_fp8(G.p(G.dev(w)), rows, cols, G.p(out), None))
    return out, W.dequantize_fp8(*W.quantize_fp8(w))


def _linear_fp8(qlib, x, segs, biases, M, K, N, y, epi, **kw):
    import ctypes as C
    from qwen_inference_engine_amd._lib import LinearArgsC
    a = LinearArgsC()
    a.x, a.ldx = G.p(x), K
    for i, s in enumerate(segs):
        a.w[i] = G.p(s[0])
        a.seg_rows[i] = s[1]
    for i, b in enumerate(biases):
        a.bias[i] = G.p(b) if b is not None else None
    a.M, a.K, a.N = M, K, N
    a.y, a.ldy = G.p(y), N
    a.epilogue = epi
    a.flags = _lib.QIE_LINEAR_FP8
    if kw.get("keys") is not None:
        a.argmax_keys = G.p(kw["keys"])
    G.check(qlib.qie_linear(C.byref(a), None), "qie_linear fp8")


@pytest.mark.parametrize("M", [1, 3, 8, 40, 300])
@pytest.mark.parametrize("K,n", [(128, (64, 32, 32)), (3584, (512, 128, 128))])
def test_fp8_linear_store_bias(oracle, qlib, M, K, n):
    x = rand_bf16(oracle, (M, K), seed=M)
    ws = [rand_bf16(oracle, (r, K), 0.05, seed=10 + i) for i, r in enumerate(n)]
    bs = [rand_bf16(oracle, (r,), 0.1, seed=20 + i) for i, r in enumerate(n)]
    q = [_fp8_dev(qlib, w) for w in ws]
    N = sum(n)
    want = np.concatenate([oracle.matmul(x, dq, b) for (_, dq), b in zip(q, bs)], axis=1)
    y = G.zeros_bf16(M, N)
    _linear_fp8(qlib, G.dev(x), [(d, r) for (d, _), r in zip(q, n)], [G.dev(b) for b in bs], M, K, N, y,
                _lib.QIE_EPI_STORE)
    scale = np.concatenate([_abs_scale(oracle, x, dq) for _, dq in q], axis=1)
    G.assert_sum_close(G.host_bf16(y), want, scale, what=f"fp8 linear M={M} K={K}")


@pytest.mark.parametrize("M", [1, 8, 64])
def test_fp8_linear_swiglu_and_residual(oracle, qlib, M):
    K, I = 896, 640
    x = rand_bf16(oracle, (M, K), seed=6)
    (dg, qg), (du, qu) = _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=7)), \
        _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=8))
    want = oracle.silu_mul(oracle.matmul(x, qg), oracle.matmul(x, qu))
    y = G.zeros_bf16(M, I)
    _linear_fp8(qlib, G.dev(x), [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU)
    d = G.ulp_diff(G.host_bf16(y), want)
    assert (d == 0).mean() > 0.97
    gs = G.bf(oracle.matmul(x, qg)).astype(np.float64)
    u = np.abs(G.bf(oracle.matmul(x, qu)).astype(np.float64))
    ill = (np.abs(gs) < 1e-2 * _abs_scale(oracle, x, qg)) | (u < 1e-2 * _abs_scale(oracle, x, qu)) | (gs < -4)
    assert not ((d > 2) & ~ill).any()
    # residual: y = bf16(res + bf16(x W^T))
    dw, qw = _fp8_dev(qlib, rand_bf16(oracle, (K, I), 0.02, seed=4))
    h = rand_bf16(oracle, (M, I), seed=3)
    res = rand_bf16(oracle, (M, K), seed=5)
    want = oracle.resadd(res, oracle.matmul(h, qw))
    yr = G.dev(res)
    _linear_fp8(qlib, G.dev(h), [(dw, K)], [], M, I, K, yr, _lib.QIE_EPI_RESIDUAL)
    acc = G.bf(oracle.matmul(h, qw)).astype(np.float64)
    tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, h, qw)
    assert (np.abs(G.bf(G.host_bf16(yr)).astype(np.float64) - G.bf(want)) <= tol).all()


CONFIGS = {
    "qwen2-bias-hd64": S.tiny("t-q2", n_layers=3, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512,
                              vocab=1000, bias=True),
    "tied-g7": S.tiny("t-tied", n_layers=2, hidden=448, n_heads=7, n_kv_heads=1, head_dim=64, ffn=640,
                      vocab=777 * 2, tie=True, bias=True),
}


@pytest.mark.parametrize("name", list(CONFIGS))
@pytest.mark.parametrize("P", [5, 23])
def test_fp8_engine_matches_oracle_on_dequantised_model(oracle, name, P):
    spec = CONFIGS[name]
    eng = Q.Engine(spec, max_ctx=128, weight_fp8=True).init_synthetic(SYN)
    hw = W.HostWeights.synthetic(spec, SYN).fp8_dequantized()
    from parity import OrderPair
    prompt = list(rng(P).integers(0, spec.vocab, P))
    ids, flips = forced_compare(oracle, eng.batch(1, 128), OrderPair(oracle, hw, 128), prompt, 12)
    assert flips <= 2


def test_fp8_batch8_equals_single(oracle):
    """B = 8 (skinny MFMA kernel) vs one sequence at a time (GEMV): the bar of
    tests/test_gpu_engine.py::test_graph_equals_eager_and_batch_equals_single."""
    from test_gpu_engine import _teacher_forced_trace, logits_close, logit_tol
    spec = CONFIGS["qwen2-bias-hd64"]
    eng = Q.Engine(spec, max_ctx=96, weight_fp8=True).init_synthetic(SYN)
    prompts = [list(rng(40 + i).integers(0, spec.vocab, 4 + 3 * i)) for i in range(8)]
    singles = [_teacher_forced_trace(eng.batch(1, 96), [pr], 7) for pr in prompts]
    s_ids = [r[0][0] for r in singles]
    s_lgs = [r[1][0] for r in singles]
    raw, lgs = _teacher_forced_trace(eng.batch(8, 96), prompts, 7, forced=s_ids)
    flips = 0
    for i in range(8):
        for t in range(7):
            logits_close(lgs[i][t], s_lgs[i][t], f"seq {i} step {t}")
            if raw[i][t] != s_ids[i][t]:
                gap = abs(float(G.bf(s_lgs[i][t][s_ids[i][t]])) - float(G.bf(s_lgs[i][t][raw[i][t]])))
                assert gap <= logit_tol(s_lgs[i][t])
                flips += 1
    assert flips <= 3


@pytest.mark.parametrize("M", [2, 8, 16])
@pytest.mark.parametrize("K", [896, 3584])
@pytest.mark.parametrize("num", ["ref", "hf"])
def test_fp8_batched_decode_kernel(oracle, qlib, M, K, num):
    """k_decode_fp8.hip (fp8 weights, 2..16 rows, K = 7 wave slices): the fused RMSNorm with
    the 3-segment QKV-shaped STORE (+bias, arg-max keys), SwiGLU with the norm, the residual
    and the fp32 epilogue, each against the oracle on the dequantised weights (the bar of
    test_linear_fused_norm_and_argmax / test_linear_swiglu / test_linear_residual)."""
    eps = 1e-4 if num == "ref" else 1e-6
    nf = 0 if num == "ref" else 1
    x = rand_bf16(oracle, (M, K), seed=M + K)
    nw = oracle.f32_to_bf16((1 + 0.2 * rng(12).standard_normal(K)).astype(np.float32))
    # the fused norm itself: identity weights make the STORE output the kernel's normalised
    # rows; they may round an element 1 ulp away from the oracle's (sum order of the squares,
    # test_rmsnorm's bar) — the projections below are then checked on the kernel's own rows
    eye = oracle.f32_to_bf16(np.eye(K, dtype=np.float32))
    de, _ = _fp8_dev(qlib, eye)
    ye = G.zeros_bf16(M, K)
    _linear(qlib, G.dev(x), [(de, K)], [], M, K, K, ye, _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=eps, num=nf,
            flags=_lib.QIE_LINEAR_FP8)
    xn = G.host_bf16(ye)
    G.assert_bf16_close(xn, oracle.rmsnorm(x, nw, eps, num), max_ulp=1 if num == "ref" else 2, min_exact=0.98,
                        what="fused norm")
    # QKV-shaped: 3 segments with biases, norm fused, arg-max keys
    n = (512, 128, 128)
    q = [_fp8_dev(qlib, rand_bf16(oracle, (r, K), 0.05, seed=30 + i)) for i, r in enumerate(n)]
    bs = [rand_bf16(oracle, (r,), 0.1, seed=40 + i) for i, r in enumerate(n)]
    N = sum(n)
    want = np.concatenate([oracle.matmul(xn, dq, b) for (_, dq), b in zip(q, bs)], axis=1)
    y = G.zeros_bf16(M, N)
    keys = G.dev(np.zeros(M, np.uint64))
    _linear(qlib, G.dev(x), [(d, r) for (d, _), r in zip(q, n)], [G.dev(b) for b in bs], M, K, N, y,
            _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=eps, num=nf, keys=keys, flags=_lib.QIE_LINEAR_FP8)
    got = G.host_bf16(y)
    scale = np.concatenate([_abs_scale(oracle, xn, dq) for _, dq in q], axis=1)
    G.assert_sum_close(got, want, scale, what=f"fp8 dec8 store M={M}")
    ids = G.zeros((M,), np.int32)
    G.check(qlib.qie_keys_to_ids(G.p(keys), M, G.p(ids), None))
    for m in range(M):
        assert G.host(ids)[m] == oracle.argmax(got[m])
    # SwiGLU with the fused norm
    I = 640
    (dg, qg), (du, qu) = _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=7)), \
        _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=8))
    want = oracle.silu_mul(oracle.matmul(xn, qg), oracle.matmul(xn, qu))
    y = G.zeros_bf16(M, I)
    _linear(qlib, G.dev(x), [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU, norm_w=G.dev(nw), eps=eps,
            num=nf, flags=_lib.QIE_LINEAR_FP8)
    d = G.ulp_diff(G.host_bf16(y), want)
    assert (d == 0).mean() > 0.97
    gs = G.bf(oracle.matmul(xn, qg)).astype(np.float64)
    u = np.abs(G.bf(oracle.matmul(xn, qu)).astype(np.float64))
    ill = (np.abs(gs) < 1e-2 * _abs_scale(oracle, xn, qg)) | (u < 1e-2 * _abs_scale(oracle, xn, qu)) | (gs < -4)
    assert not ((d > 2) & ~ill).any()
    # residual (O-shaped: N = K) and fp32 partial sums, no norm
    h = rand_bf16(oracle, (M, K), seed=3)
    dw, qw = _fp8_dev(qlib, rand_bf16(oracle, (K, K), 0.02, seed=4))
    res = rand_bf16(oracle, (M, K), seed=5)
    want = oracle.resadd(res, oracle.matmul(h, qw))
    yr = G.dev(res)
    _linear(qlib, G.dev(h), [(dw, K)], [], M, K, K, yr, _lib.QIE_EPI_RESIDUAL, flags=_lib.QIE_LINEAR_FP8)
    acc = G.bf(oracle.matmul(h, qw)).astype(np.float64)
    tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, h, qw)
    assert (np.abs(G.bf(G.host_bf16(yr)).astype(np.float64) - G.bf(want)) <= tol).all()
    yf = G.zeros((M, K), np.float32)
    _linear(qlib, G.dev(h), [(dw, K)], [], M, K, K, yf, _lib.QIE_EPI_F32, flags=_lib.QIE_LINEAR_FP8)
    want = oracle.bf16_to_f32(h).astype(np.float64) @ oracle.bf16_to_f32(qw).astype(np.float64).T
    assert np.abs(G.host(yf) - want).max() <= 1e-5 * _abs_scale(oracle, h, qw).max() + 1e-6


@pytest.mark.parametrize("M", [2, 8, 16])
@pytest.mark.parametrize("K,N", [(4864, 896), (18944, 3584)])
def test_fp8_batched_decode_long_k(oracle, qlib, M, K, N):
    """fp8, 2..16 rows, long K without a norm (the down projection): k_decode_fp8.hip's
    split-K form (parts of 8 waves x 4 units, the last one ragged: 3 parts at K = 4,864, 10 at
    18,944; the last arriving part sums them in part order): residual, STORE + bias and fp32
    against the oracle on the dequantised weights; a second launch reproduces the first bit
    for bit (the tickets are back at zero, the part order does not depend on arrival)."""
    h = rand_bf16(oracle, (M, K), seed=K + M)
    dw, qw = _fp8_dev(qlib, rand_bf16(oracle, (N, K), 0.02, seed=4))
    res = rand_bf16(oracle, (M, N), seed=5)
    want = oracle.resadd(res, oracle.matmul(h, qw))
    yr = G.dev(res)
    _linear(qlib, G.dev(h), [(dw, N)], [], M, K, N, yr, _lib.QIE_EPI_RESIDUAL, flags=_lib.QIE_LINEAR_FP8)
    acc = G.bf(oracle.matmul(h, qw)).astype(np.float64)
    tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, h, qw)
    got = G.host_bf16(yr)
    assert (np.abs(G.bf(got).astype(np.float64) - G.bf(want)) <= tol).all()
    assert (G.ulp_diff(got, want) == 0).mean() > 0.99
    yr2 = G.dev(res)
    _linear(qlib, G.dev(h), [(dw, N)], [], M, K, N, yr2, _lib.QIE_EPI_RESIDUAL, flags=_lib.QIE_LINEAR_FP8)
    assert np.array_equal(G.host_bf16(yr2), got)
    # STORE + bias (the bench's live timing of this launch uses it)
    b = rand_bf16(oracle, (N,), 0.1, seed=6)
    ys = G.zeros_bf16(M, N)
    _linear(qlib, G.dev(h), [(dw, N)], [G.dev(b)], M, K, N, ys, _lib.QIE_EPI_STORE, flags=_lib.QIE_LINEAR_FP8)
    G.assert_sum_close(G.host_bf16(ys), oracle.matmul(h, qw, b), _abs_scale(oracle, h, qw), what="long-K store")
    if M == 8:
        yf = G.zeros((M, N), np.float32)
        _linear(qlib, G.dev(h), [(dw, N)], [], M, K, N, yf, _lib.QIE_EPI_F32, flags=_lib.QIE_LINEAR_FP8)
        want = oracle.bf16_to_f32(h).astype(np.float64) @ oracle.bf16_to_f32(qw).astype(np.float64).T
        assert np.abs(G.host(yf) - want).max() <= 1e-5 * _abs_scale(oracle, h, qw).max() + 1e-6


def _tile16_host(codes, rows, cols):
    """qie_ops.h's 16-row tiled layout restated on the host: block (t, j) piece l = row
    16 t + l % 16, columns 64 j + 16 (l // 16) + [0, 16)."""
    c = codes[:rows * cols].reshape(rows // 16, 16, cols // 64, 4, 16)   # t, fr, j, g, byte
    tiled = c.transpose(0, 2, 3, 1, 4).reshape(-1)                       # t, j, g, fr, byte
    return np.concatenate([tiled, codes[rows * cols:]])


@pytest.mark.parametrize("rows,cols", [(16, 64), (48, 896), (512, 3584)])
def test_fp8_tile16_layout(oracle, qlib, rows, cols):
    """qie_fp8_tile16 is the documented permutation of the codes, bit for bit; the row scales
    are copied unchanged."""
    w = rand_bf16(oracle, (rows, cols), 0.05, seed=rows)
    d, _ = _fp8_dev(qlib, w)
    out = G.zeros((d.nbytes,), np.uint8)
    G.check(qlib.qie_fp8_tile16(G.p(d), rows, cols, G.p(out), None))
    G.check(qlib.qie_synchronize())
    assert np.array_equal(G.host(out), _tile16_host(G.host(d), rows, cols))


def _tiled(qlib, d, rows, cols):
    out = G.zeros((d.nbytes,), np.uint8)
    G.check(qlib.qie_fp8_tile16(G.p(d), rows, cols, G.p(out), None))
    return out


@pytest.mark.parametrize("M", [1, 2, 8, 16])
@pytest.mark.parametrize("K", [896, 3584])
def test_fp8_t16_decode_kernel_equals_plain(oracle, qlib, M, K):
    """The batched-decode kernel on 16-row tiled weights (QIE_LINEAR_FP8_T16, the engine's
    decode projections) only changes where each fragment is loaded from: its outputs equal
    the plain-layout kernel's bit for bit (fused norm + 3-segment STORE with biases and
    arg-max keys, SwiGLU, residual), at M = 1 too (there the plain reference runs at M = 2
    on a duplicated row: rows are independent)."""
    Mr = max(M, 2)
    x = rand_bf16(oracle, (Mr, K), seed=M + K)
    if M == 1:
        x[1] = x[0]
    nw = oracle.f32_to_bf16((1 + 0.2 * rng(12).standard_normal(K)).astype(np.float32))
    fp8 = _lib.QIE_LINEAR_FP8
    t16 = fp8 | _lib.QIE_LINEAR_FP8_T16
    # QKV-shaped, fused norm, biases, arg-max keys
    n = (512, 128, 128)
    q = [_fp8_dev(qlib, rand_bf16(oracle, (r, K), 0.05, seed=30 + i))[0] for i, r in enumerate(n)]
    qt = [_tiled(qlib, d, r, K) for d, r in zip(q, n)]
    bs = [G.dev(rand_bf16(oracle, (r,), 0.1, seed=40 + i)) for i, r in enumerate(n)]
    N = sum(n)
    outs = []
    for ws, fl, m in ((q, fp8, Mr), (qt, t16, M)):
        y = G.zeros_bf16(m, N)
        keys = G.dev(np.zeros(m, np.uint64))
        _linear(qlib, G.dev(x[:m].copy()), list(zip(ws, n)), bs, m, K, N, y, _lib.QIE_EPI_STORE, norm_w=G.dev(nw),
                eps=1e-6, num=0, keys=keys, flags=fl)
        outs.append((G.host_bf16(y)[:M], G.host(keys)[:M]))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    # SwiGLU with the fused norm
    I = 640
    g_, u_ = (_fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=7 + i))[0] for i in range(2))
    gt, ut = _tiled(qlib, g_, I, K), _tiled(qlib, u_, I, K)
    outs = []
    for (a, b), fl, m in (((g_, u_), fp8, Mr), ((gt, ut), t16, M)):
        y = G.zeros_bf16(m, I)
        _linear(qlib, G.dev(x[:m].copy()), [(a, I), (b, I)], [], m, K, I, y, _lib.QIE_EPI_SWIGLU, norm_w=G.dev(nw),
                eps=1e-6, num=0, flags=fl)
        outs.append(G.host_bf16(y)[:M])
    assert np.array_equal(outs[0], outs[1])
    # residual (O-shaped), no norm
    dw = _fp8_dev(qlib, rand_bf16(oracle, (K, K), 0.02, seed=4))[0]
    dwt = _tiled(qlib, dw, K, K)
    res = rand_bf16(oracle, (Mr, K), seed=5)
    outs = []
    for w_, fl, m in ((dw, fp8, Mr), (dwt, t16, M)):
        yr = G.dev(res[:m].copy())
        _linear(qlib, G.dev(x[:m].copy()), [(w_, K)], [], m, K, K, yr, _lib.QIE_EPI_RESIDUAL, flags=fl)
        outs.append(G.host_bf16(yr)[:M])
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("M", [1, 8])
@pytest.mark.parametrize("K,N", [(4864, 896), (18944, 3584)])
def test_fp8_t16_long_k_equals_plain(oracle, qlib, M, K, N):
    """Split-K form on tiled weights (the down projection) == the plain-layout split-K form,
    bit for bit (M = 1 against M = 2 with a duplicated row)."""
    Mr = max(M, 2)
    h = rand_bf16(oracle, (Mr, K), seed=K + M)
    if M == 1:
        h[1] = h[0]
    dw = _fp8_dev(qlib, rand_bf16(oracle, (N, K), 0.02, seed=4))[0]
    dwt = _tiled(qlib, dw, N, K)
    res = rand_bf16(oracle, (Mr, N), seed=5)
    outs = []
    for w_, fl, m in ((dw, _lib.QIE_LINEAR_FP8, Mr), (dwt, _lib.QIE_LINEAR_FP8 | _lib.QIE_LINEAR_FP8_T16, M)):
        yr = G.dev(res[:m].copy())
        _linear(qlib, G.dev(h[:m].copy()), [(w_, N)], [], m, K, N, yr, _lib.QIE_EPI_RESIDUAL, flags=fl)
        outs.append(G.host_bf16(yr)[:M])
    assert np.array_equal(outs[0], outs[1])


def test_fp8_t16_rejected_outside_decode_kernel(qlib):
    """Tiled weights are readable by the batched-decode kernel only: a prefill-sized call
    (M > 16) with the flag fails loudly instead of reading them as plain rows."""
    import ctypes as C
    from qwen_inference_engine_amd._lib import LinearArgsC
    K, N, M = 896, 128, 32
    w = G.zeros((int(qlib.qie_fp8_weight_bytes(N, K)),), np.uint8)
    a = LinearArgsC()
    x, y = G.zeros_bf16(M, K), G.zeros_bf16(M, N)
    a.x, a.ldx = G.p(x), K
    a.w[0], a.seg_rows[0] = G.p(w), N
    a.M, a.K, a.N = M, K, N
    a.y, a.ldy = G.p(y), N
    a.epilogue = _lib.QIE_EPI_STORE
    a.flags = _lib.QIE_LINEAR_FP8 | _lib.QIE_LINEAR_FP8_T16
    assert qlib.qie_linear(C.byref(a), None) != 0


@pytest.mark.parametrize("M", [2, 16])
@pytest.mark.parametrize("tiled", [False, True])
def test_fp8_batched_decode_many_tiles_per_block(oracle, qlib, M, tiled):
    """The batched-decode kernel with several column tiles per block (more tiles than
    resident blocks): the multi-tile loop, the double-buffered partial-tile hand-off and the
    rotating epilogue wave.  Config-4 shapes: SwiGLU I = 18,944 and the QKV-shaped 3-segment
    STORE (N = 4,608) at K = 3,584 with the fused norm; the 8-wave slice shapes K = 2,048 and
    4,096 (STORE, N = 8,192); plain and 16-row tiled weights, against the oracle on the
    dequantised weights (test_fp8_batched_decode_kernel's bars)."""
    fl = _lib.QIE_LINEAR_FP8 | (_lib.QIE_LINEAR_FP8_T16 if tiled else 0)

    def dev_w(rows, K, scale, seed):
        d, dq = _fp8_dev(qlib, rand_bf16(oracle, (rows, K), scale, seed=seed))
        return (_tiled(qlib, d, rows, K) if tiled else d), dq

    K = 3584
    x = rand_bf16(oracle, (M, K), seed=90 + M)
    nw = oracle.f32_to_bf16((1 + 0.2 * rng(13).standard_normal(K)).astype(np.float32))
    # the kernel's own normalised rows (identity weights; they may sit 1 ulp off the oracle's,
    # test_fp8_batched_decode_kernel): the projections are checked on them
    de, _ = _fp8_dev(qlib, oracle.f32_to_bf16(np.eye(K, dtype=np.float32)))
    ye = G.zeros_bf16(M, K)
    _linear(qlib, G.dev(x), [(de, K)], [], M, K, K, ye, _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=1e-6, num=0,
            flags=_lib.QIE_LINEAR_FP8)
    xn = G.host_bf16(ye)
    # SwiGLU, I = 18,944 (1,184 tiles)
    I = 18944
    (dg, qg), (du, qu) = dev_w(I, K, 0.08, 7), dev_w(I, K, 0.08, 8)
    y = G.zeros_bf16(M, I)
    _linear(qlib, G.dev(x), [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU, norm_w=G.dev(nw), eps=1e-6,
            num=0, flags=fl)
    # the SwiGLU bar of test_fp8_batched_decode_kernel / test_linear_swiglu
    want = oracle.silu_mul(oracle.matmul(xn, qg), oracle.matmul(xn, qu))
    d = G.ulp_diff(G.host_bf16(y), want)
    gs = G.bf(oracle.matmul(xn, qg)).astype(np.float64)
    u = np.abs(G.bf(oracle.matmul(xn, qu)).astype(np.float64))
    ill = (np.abs(gs) < 1e-2 * _abs_scale(oracle, xn, qg)) | (u < 1e-2 * _abs_scale(oracle, xn, qu)) | (gs < -4)
    assert (d == 0).mean() > 0.97 and not ((d > 2) & ~ill).any()
    # QKV-shaped, N = 4,608 (288 tiles), biases
    n = (3584, 512, 512)
    q = [dev_w(r, K, 0.05, 30 + i) for i, r in enumerate(n)]
    bs = [rand_bf16(oracle, (r,), 0.1, seed=40 + i) for i, r in enumerate(n)]
    N = sum(n)
    y = G.zeros_bf16(M, N)
    _linear(qlib, G.dev(x), [(dd, r) for (dd, _), r in zip(q, n)], [G.dev(b) for b in bs], M, K, N, y,
            _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=1e-6, num=0, flags=fl)
    want = np.concatenate([oracle.matmul(xn, dq, b) for (_, dq), b in zip(q, bs)], axis=1)
    scale = np.concatenate([_abs_scale(oracle, xn, dq) for _, dq in q], axis=1)
    G.assert_sum_close(G.host_bf16(y), want, scale, what=f"fp8 dec8 qkv N={N} M={M}")
    # 8-wave slice shapes, 512 tiles
    for K2 in (2048, 4096):
        x2 = rand_bf16(oracle, (M, K2), seed=K2 + M)
        N2 = 8192
        dw, qw = dev_w(N2, K2, 0.03, K2)
        y = G.zeros_bf16(M, N2)
        _linear(qlib, G.dev(x2), [(dw, N2)], [], M, K2, N2, y, _lib.QIE_EPI_STORE, flags=fl)
        G.assert_sum_close(G.host_bf16(y), oracle.matmul(x2, qw), _abs_scale(oracle, x2, qw), what=f"fp8 dec8 K={K2}")


@pytest.mark.parametrize("M", [1, 3, 8])
def test_fp8_t16_vocab_projection_skinny(oracle, qlib, M):
    """A vocabulary-sized projection (N > 32,768: the skinny MFMA kernel, not the batched-decode
    one) on 16-row tiled weights, with the fused norm and arg-max keys: equal bit for bit to
    the plain layout (M = 1 against M = 2 with a duplicated row), and the keys' ids equal the
    arg-max of the plain output."""
    K, N = 896, 40960
    Mr = max(M, 2)
    x = rand_bf16(oracle, (Mr, K), seed=500 + M)
    if M == 1:
        x[1] = x[0]
    nw = oracle.f32_to_bf16((1 + 0.2 * rng(14).standard_normal(K)).astype(np.float32))
    d, _ = _fp8_dev(qlib, rand_bf16(oracle, (N, K), 0.05, seed=501))
    dt = _tiled(qlib, d, N, K)
    outs = []
    for w_, fl, m in ((d, _lib.QIE_LINEAR_FP8, Mr), (dt, _lib.QIE_LINEAR_FP8 | _lib.QIE_LINEAR_FP8_T16, M)):
        y = G.zeros_bf16(m, N)
        keys = G.dev(np.zeros(m, np.uint64))
        _linear(qlib, G.dev(x[:m].copy()), [(w_, N)], [], m, K, N, y, _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=1e-6,
                num=0, keys=keys, flags=fl)
        outs.append((G.host_bf16(y)[:M], G.host(keys)[:M]))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
