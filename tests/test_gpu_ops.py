"""GPU parity: every libqie op (C ABI) against the CPU oracle on identical bf16 inputs.

Tolerances (written per test): bit-exact for copies, selection and the elementwise ops
whose arithmetic is restated without contraction; <= 1 bf16 ulp (>= 98 % exact) where
only an fp32 summation order differs (RMSNorm, qk-norm); for dot products
|got - want| <= max(1 bf16 ulp, 1e-5 * sum|a*w|) (accumulation order of K terms).
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as G
from conftest import rng

from qwen_inference_engine_amd import _lib
from qwen_inference_engine_amd._lib import LinearArgsC, KvCacheC, SamplingC

pytestmark = pytest.mark.gpu


def rand_bf16(oracle, shape, scale=1.0, seed=0):
    return oracle.f32_to_bf16((rng(seed).standard_normal(shape) * scale).astype(np.float32))


# ------------------------------------------------------------------------ embedding
def test_embedding_exact(oracle, qlib):
    E = rand_bf16(oracle, (1000, 256), seed=1)
    ids = np.array([0, 999, 5, 5, 123, 999, 0], np.int32)
    out = G.zeros_bf16(len(ids), 256)
    dE, dI = G.dev(E), G.dev(ids)
    G.check(qlib.qie_embedding(G.p(dE), G.p(dI), G.p(out), len(ids), 256, None))
    assert np.array_equal(G.host_bf16(out), E[ids])


# -------------------------------------------------------------------------- RMSNorm
@pytest.mark.parametrize("rows,H", [(1, 128), (3, 896), (17, 3584), (2, 8192)])
@pytest.mark.parametrize("num", ["ref", "hf"])
def test_rmsnorm(oracle, qlib, rows, H, num):
    x = rand_bf16(oracle, (rows, H), seed=rows + H)
    w = oracle.f32_to_bf16((1 + 0.2 * rng(7).standard_normal(H)).astype(np.float32))
    eps = 1e-4 if num == "ref" else 1e-6
    want = oracle.rmsnorm(x, w, eps, num)
    y = G.zeros_bf16(rows, H)
    dx, dw = G.dev(x), G.dev(w)
    G.check(qlib.qie_rmsnorm(G.p(dx), G.p(dw), G.p(y), rows, H, eps, 0 if num == "ref" else 1, None))
    G.assert_bf16_close(G.host_bf16(y), want, max_ulp=1 if num == "ref" else 2, min_exact=0.98, what="rmsnorm")


# --------------------------------------------------------------------------- linear
def _linear(qlib, x, segs, biases, M, K, N, y, epi, norm_w=None, eps=1e-4, num=0, keys=None, ldy=None, flags=0):
    a = LinearArgsC()
    a.x, a.ldx = G.p(x), K
    for i, s in enumerate(segs):
        a.w[i] = G.p(s[0])
        a.seg_rows[i] = s[1]
    for i, b in enumerate(biases):
        a.bias[i] = G.p(b) if b is not None else None
    a.M, a.K, a.N = M, K, N
    a.y, a.ldy = G.p(y), ldy or N
    a.epilogue = epi
    a.norm_w = G.p(norm_w) if norm_w is not None else None
    a.norm_eps, a.numerics = eps, num
    a.argmax_keys = G.p(keys) if keys is not None else None
    a.flags = flags
    G.check(qlib.qie_linear(C.byref(a), None), "qie_linear")


def _abs_scale(oracle, x, w):
    return np.abs(oracle.bf16_to_f32(x).astype(np.float64)) @ np.abs(oracle.bf16_to_f32(w).astype(np.float64)).T


@pytest.mark.parametrize("M", [1, 2, 3, 5, 8, 9, 64, 130, 300])
@pytest.mark.parametrize("K,n", [(128, (64, 32, 32)), (896, (896, 128, 128)), (3584, (512, 128, 128)),
                                 (3696, (200, 8, 48))])
def test_linear_store_bias_3seg(oracle, qlib, M, K, n):
    if M > 64 and K > 1000:
        pytest.skip("covered at smaller M")
    x = rand_bf16(oracle, (M, K), seed=M)
    ws = [rand_bf16(oracle, (r, K), 0.05, seed=10 + i) for i, r in enumerate(n)]
    bs = [rand_bf16(oracle, (r,), 0.1, seed=20 + i) for i, r in enumerate(n)]
    N = sum(n)
    want = np.concatenate([oracle.matmul(x, w, b) for w, b in zip(ws, bs)], axis=1)
    dws, dbs = [G.dev(w) for w in ws], [G.dev(b) for b in bs]
    y = G.zeros_bf16(M, N)
    _linear(qlib, G.dev(x), list(zip(dws, n)), dbs, M, K, N, y, _lib.QIE_EPI_STORE)
    scale = np.concatenate([_abs_scale(oracle, x, w) for w in ws], axis=1)
    G.assert_sum_close(G.host_bf16(y), want, scale, what=f"linear M={M} K={K}")


@pytest.mark.parametrize("M", [1, 4, 8, 33, 256])
@pytest.mark.parametrize("K,N", [(896, 896), (4864, 896), (1024, 8192), (18944, 3584)])
def test_linear_residual(oracle, qlib, M, K, N):
    if M * K * N > 256 * 4864 * 896 * 2:
        pytest.skip("oracle time")
    x = rand_bf16(oracle, (M, K), seed=3)
    w = rand_bf16(oracle, (N, K), 0.02, seed=4)
    res = rand_bf16(oracle, (M, N), seed=5)
    want = oracle.resadd(res, oracle.matmul(x, w))
    y = G.dev(res)
    _linear(qlib, G.dev(x), [(G.dev(w), N)], [], M, K, N, y, _lib.QIE_EPI_RESIDUAL)
    got = G.host_bf16(y)
    # y = bf16(res + bf16(acc)): the inner bf16(acc) may differ by 1 ulp of |acc| (fp32
    # summation order), then one more rounding at |y| — absolute bound, since res + acc
    # can cancel to far below either operand.
    acc = G.bf(oracle.matmul(x, w)).astype(np.float64)
    tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, x, w)
    err = np.abs(G.bf(got).astype(np.float64) - G.bf(want))
    assert (err <= tol).all(), f"worst {(err - tol).max()}"
    assert (G.ulp_diff(got, want) == 0).mean() > 0.99


@pytest.mark.parametrize("M", [1, 2, 8, 17, 128])
@pytest.mark.parametrize("K,I", [(128, 256), (896, 4864), (3584, 640)])
def test_linear_swiglu(oracle, qlib, M, K, I):
    x = rand_bf16(oracle, (M, K), seed=6)
    wg = rand_bf16(oracle, (I, K), 0.08, seed=7)
    wu = rand_bf16(oracle, (I, K), 0.08, seed=8)
    want = oracle.silu_mul(oracle.matmul(x, wg), oracle.matmul(x, wu))
    y = G.zeros_bf16(M, I)
    _linear(qlib, G.dev(x), [(G.dev(wg), I), (G.dev(wu), I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU)
    got = G.host_bf16(y)
    d = G.ulp_diff(got, want)
    assert (d == 0).mean() > 0.97
    # elements off by > 2 ulps must be ill-conditioned: a gate/up sum that cancels to
    # < 1 % of sum|x*w| (fp32 summation order alone moves many bf16 ulps), or a gate
    # g < -4 where silu(g) = g*sigmoid(g) amplifies a relative error of g by |1 + g(1-sig)|
    gs = G.bf(oracle.matmul(x, wg)).astype(np.float64)
    g = np.abs(gs)
    u = np.abs(G.bf(oracle.matmul(x, wu)).astype(np.float64))
    ill = (g < 1e-2 * _abs_scale(oracle, x, wg)) | (u < 1e-2 * _abs_scale(oracle, x, wu)) | (gs < -4)
    assert not ((d > 2) & ~ill).any(), f"well-conditioned element off by {d[~ill].max()} ulps"


@pytest.mark.parametrize("M,K", [(256, 896), (300, 96), (520, 32), (257, 3584)])
@pytest.mark.parametrize("epi", ["store3", "residual", "swiglu", "f32"])
@pytest.mark.parametrize("tile", ["1", "2", "sk"])
def test_linear_big_gemm(oracle, qlib, M, K, epi, tile):
    """The LDS-DMA prefill GEMM, 256x256 (QIE_LINEAR_TILE256) and 256x128 (QIE_LINEAR_TILE128)
    tiles, forced at test sizes (the engine picks them by tile count): every epilogue, ragged
    M and N (clamped rows never stored), K of 1, 3 and 28+ k-tiles (ring prologue / drain);
    "sk" the stream-K form (QIE_LINEAR_STREAMK, K % 64 == 0 and >= 256 only): at these sizes
    every workgroup gets ONE k-tile, so each tile is summed from 14 or 56 segments."""
    fl = {"1": _lib.QIE_LINEAR_TILE256, "2": _lib.QIE_LINEAR_TILE128, "sk": _lib.QIE_LINEAR_STREAMK}[tile]
    x = rand_bf16(oracle, (M, K), seed=M + K)
    if epi == "store3":
        n = (200, 72, 40)
        ws = [rand_bf16(oracle, (r, K), 0.05, seed=30 + i) for i, r in enumerate(n)]
        bs = [rand_bf16(oracle, (r,), 0.1, seed=40 + i) for i, r in enumerate(n)]
        N = sum(n)
        want = np.concatenate([oracle.matmul(x, w, b) for w, b in zip(ws, bs)], axis=1)
        y = G.zeros_bf16(M, N)
        _linear(qlib, G.dev(x), [(G.dev(w), r) for w, r in zip(ws, n)], [G.dev(b) for b in bs], M, K, N, y,
                _lib.QIE_EPI_STORE, flags=fl)
        scale = np.concatenate([_abs_scale(oracle, x, w) for w in ws], axis=1)
        G.assert_sum_close(G.host_bf16(y), want, scale, what=f"big store M={M} K={K}")
    elif epi == "residual":
        N = 320
        w = rand_bf16(oracle, (N, K), 0.02, seed=4)
        res = rand_bf16(oracle, (M, N), seed=5)
        want = oracle.resadd(res, oracle.matmul(x, w))
        y = G.dev(res)
        _linear(qlib, G.dev(x), [(G.dev(w), N)], [], M, K, N, y, _lib.QIE_EPI_RESIDUAL, flags=fl)
        acc = G.bf(oracle.matmul(x, w)).astype(np.float64)
        tol = 2.0 ** -7 * (np.abs(acc) + np.abs(G.bf(want))) + 1e-5 * _abs_scale(oracle, x, w)
        assert (np.abs(G.bf(G.host_bf16(y)).astype(np.float64) - G.bf(want)) <= tol).all()
    elif epi == "swiglu":
        I = 200
        wg = rand_bf16(oracle, (I, K), 0.08, seed=7)
        wu = rand_bf16(oracle, (I, K), 0.08, seed=8)
        want = oracle.silu_mul(oracle.matmul(x, wg), oracle.matmul(x, wu))
        y = G.zeros_bf16(M, I)
        _linear(qlib, G.dev(x), [(G.dev(wg), I), (G.dev(wu), I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU, flags=fl)
        got = G.host_bf16(y)
        d = G.ulp_diff(got, want)
        gs = G.bf(oracle.matmul(x, wg)).astype(np.float64)
        u = np.abs(G.bf(oracle.matmul(x, wu)).astype(np.float64))
        ill = (np.abs(gs) < 1e-2 * _abs_scale(oracle, x, wg)) | (u < 1e-2 * _abs_scale(oracle, x, wu)) | (gs < -4)
        assert (d == 0).mean() > 0.97 and not ((d > 2) & ~ill).any()
    else:
        N = 264
        w = rand_bf16(oracle, (N, K), 0.05, seed=9)
        y = G.zeros((M, N), np.float32)
        _linear(qlib, G.dev(x), [(G.dev(w), N)], [], M, K, N, y, _lib.QIE_EPI_F32, flags=fl)
        want = oracle.bf16_to_f32(x).astype(np.float64) @ oracle.bf16_to_f32(w).astype(np.float64).T
        assert np.abs(G.host(y) - want).max() <= 1e-5 * _abs_scale(oracle, x, w).max() + 1e-6


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("num", ["ref", "hf"])
def test_linear_fused_norm_and_argmax(oracle, qlib, M, num):
    K, N = 896, 5000
    x = rand_bf16(oracle, (M, K), seed=11)
    nw = oracle.f32_to_bf16((1 + 0.2 * rng(12).standard_normal(K)).astype(np.float32))
    w = rand_bf16(oracle, (N, K), 0.05, seed=13)
    eps = 1e-4 if num == "ref" else 1e-6
    xn = oracle.rmsnorm(x, nw, eps, num)
    want = oracle.matmul(xn, w)
    y = G.zeros_bf16(M, N)
    keys = G.dev(np.zeros(M, np.uint64))
    _linear(qlib, G.dev(x), [(G.dev(w), N)], [], M, K, N, y, _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=eps,
            num=0 if num == "ref" else 1, keys=keys)
    got = G.host_bf16(y)
    # the fused RMSNorm may round a few normalised activations 1 ulp differently (sum order);
    # HF numerics round twice (bf16(w * bf16(x/rms))), so allow 2 output ulps there
    G.assert_sum_close(got, want, _abs_scale(oracle, xn, w), rel=1e-4, ulps=1 if num == "ref" else 2,
                       what="fused norm")
    ids = G.zeros((M,), np.int32)
    G.check(qlib.qie_keys_to_ids(G.p(keys), M, G.p(ids), None))
    for m in range(M):   # fused arg-max == reference rule on the kernel's own logits
        assert G.host(ids)[m] == oracle.argmax(got[m])


# -------------------------------------------------------------------- q/k post + KV
def _cache(kc, vc, L, nkv, hd, ctx, seq_stride):
    c = KvCacheC()
    c.k, c.v, c.seq_stride = G.p(kc), G.p(vc), seq_stride
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = L, nkv, hd, ctx
    return c


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("qkn", [False, True])
@pytest.mark.parametrize("num", ["ref", "hf"])
@pytest.mark.parametrize("mode", ["prefill", "decode"])
@pytest.mark.parametrize("heads", [(6, 2), (48, 4)])   # 56 heads: two load batches per wave
def test_qkv_post(oracle, qlib, hd, qkn, num, mode, heads):
    (nq, nkv), L, ctx, layer = heads, 3, 40, 1
    QD, KD = nq * hd, nkv * hd
    if mode == "prefill":
        M, rps = 9, 9
        pos = np.arange(3, 3 + M, dtype=np.int32)
    else:
        M, rps = 3, 1
        pos = np.array([5, 0, 39], np.int32)
    qkv = rand_bf16(oracle, (M, QD + 2 * KD), seed=hd + M)
    qn = oracle.f32_to_bf16((1 + 0.3 * rng(1).standard_normal(hd)).astype(np.float32)) if qkn else None
    kn = oracle.f32_to_bf16((1 + 0.3 * rng(2).standard_normal(hd)).astype(np.float32)) if qkn else None
    eps = 1e-4 if num == "ref" else 1e-6
    cs, sn = oracle.rope_table(ctx, hd, 1e6, num)
    q = qkv[:, :QD].copy()
    k = qkv[:, QD:QD + KD].copy()
    v = qkv[:, QD + KD:].copy()
    if qkn:
        q = oracle.qknorm(q, qn, nq, hd, eps, num)
        k = oracle.qknorm(k, kn, nkv, hd, eps, num)
    q = oracle.rope(q, cs, sn, pos, nq, hd, num)
    k = oracle.rope(k, cs, sn, pos, nkv, hd, num)
    nseq = M // rps
    seq_stride = L * nkv * ctx * hd
    kc = G.zeros_bf16(nseq * seq_stride)
    vc = G.zeros_bf16(nseq * seq_stride)
    qo = G.zeros_bf16(M, QD)
    c = _cache(kc, vc, L, nkv, hd, ctx, seq_stride)
    dcs, dsn = G.dev(cs), G.dev(sn)
    dqn = G.dev(qn) if qkn else None
    dkn = G.dev(kn) if qkn else None
    G.check(qlib.qie_qkv_post(G.p(G.dev(qkv)), M, G.p(G.dev(pos)), rps, G.p(dqn) if qkn else None,
                              G.p(dkn) if qkn else None, G.p(dcs), G.p(dsn), nq, C.byref(c), layer, eps,
                              0 if num == "ref" else 1, G.p(qo), None))
    G.assert_bf16_close(G.host_bf16(qo), q, max_ulp=1, min_exact=0.98 if qkn else 1.0, what="q")
    hk = G.host_bf16(kc).reshape(nseq, L, nkv, ctx, hd)
    hv = G.host_bf16(vc).reshape(nseq, L, nkv, ctx, hd)
    for m in range(M):
        s = m // rps
        for g in range(nkv):
            G.assert_bf16_close(hk[s, layer, g, pos[m]], k[m, g * hd:(g + 1) * hd], 1,
                                0.9 if qkn else 1.0, "k")
            assert np.array_equal(hv[s, layer, g, pos[m]], v[m, g * hd:(g + 1) * hd])
    # nothing else written
    mask = np.zeros_like(hk, bool)
    for m in range(M):
        mask[m // rps, layer, :, pos[m]] = True
    assert not hk[~mask].any() and not hv[~mask].any()


# ----------------------------------------------------------------------- attention
@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("nq,nkv", [(4, 4), (14, 2), (28, 4), (16, 2)])
@pytest.mark.parametrize("ctxs", [[1], [5, 64, 65], [1000], [2049, 3]])
def test_attention_decode(oracle, qlib, hd, nq, nkv, ctxs):
    L, layer, maxc = 2, 1, 2304
    B = len(ctxs)
    seq_stride = L * nkv * maxc * hd
    kc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq)
    vc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq + 1)
    q = rand_bf16(oracle, (B, nq * hd), seed=3)
    pos = np.array(ctxs, np.int32) - 1
    ws_bytes = qlib.qie_attention_workspace_bytes(B, nq, hd, maxc)
    ws = G.zeros_bytes(ws_bytes)
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    out = G.zeros_bf16(B, nq * hd)
    c = _cache(kc, vc, L, nkv, hd, maxc, seq_stride)
    G.check(qlib.qie_attention(G.p(G.dev(q)), B, G.p(G.dev(pos)), 1, C.byref(c), layer, nq, G.p(out), G.p(ws), None))
    got = G.host_bf16(out)
    for b in range(B):
        want = oracle.attention(q[b:b + 1], kc_h[b, layer, :, :ctxs[b]], vc_h[b, layer, :, :ctxs[b]], nq, nkv, hd,
                                False, 0)
        d = np.abs(G.bf(got[b]) - G.bf(want[0]))
        assert d.max() <= 2 ** -7 * max(1.0, np.abs(G.bf(want[0])).max()) * 2, f"ctx {ctxs[b]}: {d.max()}"


@pytest.mark.parametrize("P,hd", [(1, 64), (7, 64), (64, 64), (257, 64), (33, 128), (130, 128), (511, 128)])
def test_attention_prefill_causal(oracle, qlib, P, hd):
    """Causal prefill attention (flash, MFMA) vs the oracle's self_attension.cu restatement."""
    nq, nkv, L, layer, maxc = 14, 2, 1, 0, 512
    seq_stride = L * nkv * maxc * hd
    kc_h = rand_bf16(oracle, (1, L, nkv, maxc, hd), seed=P)
    vc_h = rand_bf16(oracle, (1, L, nkv, maxc, hd), seed=P + 1)
    q = rand_bf16(oracle, (P, nq * hd), seed=P + 2)
    pos = np.arange(P, dtype=np.int32)
    ws_bytes = qlib.qie_attention_workspace_bytes(P, nq, hd, maxc)
    ws = G.zeros_bytes(ws_bytes)
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    out = G.zeros_bf16(P, nq * hd)
    c = _cache(kc, vc, L, nkv, hd, maxc, seq_stride)
    G.check(qlib.qie_attention(G.p(G.dev(q)), P, G.p(G.dev(pos)), P, C.byref(c), layer, nq, G.p(out), G.p(ws), None))
    want = oracle.attention(q, kc_h[0, layer, :, :P], vc_h[0, layer, :, :P], nq, nkv, hd, True, 0)
    d = np.abs(G.bf(G.host_bf16(out)) - G.bf(want))
    assert d.max() <= 2 ** -6, d.max()


# --------------------------------------------------------------------- elementwise
def test_silu_mul_and_residual(oracle, qlib):
    n = 8 * 5000
    g = rand_bf16(oracle, (n,), 3.0, seed=1)
    u = rand_bf16(oracle, (n,), seed=2)
    h = G.zeros_bf16(n)
    G.check(qlib.qie_silu_mul(G.p(G.dev(g)), G.p(G.dev(u)), G.p(h), n, None))
    G.assert_bf16_close(G.host_bf16(h), oracle.silu_mul(g, u), max_ulp=1, min_exact=0.999, what="silu")
    x = G.dev(g)
    G.check(qlib.qie_residual_add(G.p(x), G.p(G.dev(u)), n, None))
    assert np.array_equal(G.host_bf16(x), oracle.resadd(g, u))


# ------------------------------------------------------------------------ sampling
@pytest.mark.parametrize("V", [1000, 151936, 152064])
@pytest.mark.parametrize("kind", ["normal", "ties"])
def test_sampling_greedy_topk_and_draw(oracle, qlib, V, kind):
    M = 3
    r = rng(V)
    if kind == "ties":
        lg = oracle.f32_to_bf16(r.integers(0, 6, (M, V)).astype(np.float32))
    else:
        lg = oracle.f32_to_bf16((r.standard_normal((M, V)) * 3).astype(np.float32))
    dl = G.dev(lg)
    ws = G.zeros_bytes(qlib.qie_sample_workspace_bytes(M, V))
    ids = G.zeros((M,), np.int32)
    step = G.dev(np.array([0, 1, 7], np.int32))
    for k, T, tp in [(1, 1.0, 1.0), (50, 0.7, 1.0), (50, 1.0, 1.0), (5, 1.3, 1.0), (256, 0.9, 1.0), (50, 0.8, 0.9)]:
        s = SamplingC()
        s.top_k, s.temperature, s.top_p, s.seed = k, T, tp, 1234
        G.check(qlib.qie_sample(G.p(dl), M, V, V, C.byref(s), G.p(step), G.p(ids), G.p(ws), None))
        got = G.host(ids)
        for m in range(M):
            sd = 1234 + [0, 1, 7][m]
            want = oracle.argmax(lg[m]) if k == 1 else oracle.sample(lg[m], k, T, tp, sd)
            assert got[m] == want, (k, T, tp, m)


# ---------------------------------------------------------------- synthetic weights
def test_synthetic_fill_device_equals_host(qlib):
    from qwen_inference_engine_amd import weights as W
    n = 1 << 20
    t = G.zeros_bf16(n)
    name = "model.layers.0.self_attn.q_proj.weight"
    G.check(qlib.qie_synthetic_fill(G.p(t), n, W.tensor_id(name), 42, 0.0346, 0.0, None))
    host = W.synthetic_tensor(name, "self_attn.q_proj.weight", n, W.SynthParams(seed=42))
    assert np.array_equal(G.host_bf16(t), host)
    G.check(qlib.qie_synthetic_fill(G.p(t), n, 77, 1, 0.25, 1.0, None))
    h2 = np.empty(n, np.uint16)
    G.check(qlib.qie_synthetic_fill_host(h2.ctypes.data, n, 77, 1, 0.25, 1.0))
    assert np.array_equal(G.host_bf16(t), h2)


# ------------------------------------------------------ fused decode attention
@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("qkn,num", [(False, "ref"), (True, "ref"), (False, "hf"), (True, "hf")])
@pytest.mark.parametrize("nq,nkv", [(28, 4), (14, 2), (5, 1)])
def test_attention_decode_fused(oracle, qlib, hd, qkn, num, nq, nkv):
    """qk-norm + RoPE + KV append + split attention + in-launch combine, one launch,
    against qknorm/rope/attention of the oracle (and the appended cache rows)."""
    L, layer, maxc = 2, 1, 700
    ctxs = [1, 64, 65, 129, 700] if nq == 28 else [3, 200, 640]
    B = len(ctxs)
    QD, KD = nq * hd, nkv * hd
    seq_stride = L * nkv * maxc * hd
    kc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq)
    vc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + nq + 1)
    qkv = rand_bf16(oracle, (B, QD + 2 * KD), seed=5)
    pos = np.array(ctxs, np.int32) - 1
    eps = 1e-4 if num == "ref" else 1e-6
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
    dcs, dsn, dqkv, dpos = G.dev(cs), G.dev(sn), G.dev(qkv), G.dev(pos)
    for rep in range(2):   # second call checks the counters were left zeroed
        G.check(qlib.qie_attention_decode(G.p(dqkv), B, G.p(dpos), G.p(dqn), G.p(dkn), G.p(dcs), G.p(dsn), nq,
                                          C.byref(c), layer, eps, 0 if num == "ref" else 1, G.p(out), G.p(ws), None))
        got = G.host_bf16(out)
        hk = G.host_bf16(kc).reshape(B, L, nkv, maxc, hd)
        hv = G.host_bf16(vc).reshape(B, L, nkv, maxc, hd)
        for b in range(B):
            p = pos[b]
            for g in range(nkv):
                # qk-norm sum order may flip one rounding; HF rounds twice (2 ulps)
                G.assert_bf16_close(hk[b, layer, g, p], k[b, g * hd:(g + 1) * hd], 1 if num == "ref" else 2,
                                    0.9 if qkn else 1.0, "k")
                assert np.array_equal(hv[b, layer, g, p], v[b, g * hd:(g + 1) * hd])
            kk = kc_h[b, layer, :, :p + 1].copy()
            vv = vc_h[b, layer, :, :p + 1].copy()
            kk[:, p] = k[b].reshape(nkv, hd)
            vv[:, p] = v[b].reshape(nkv, hd)
            want = oracle.attention(q[b:b + 1], kk, vv, nq, nkv, hd, False, 0)
            d = np.abs(G.bf(got[b]) - G.bf(want[0]))
            assert d.max() <= 2 ** -7 * max(1.0, np.abs(G.bf(want[0])).max()) * 2, f"ctx {ctxs[b]}: {d.max()}"
    assert not G.host(ws)[:B * nkv * 4].any()


@pytest.mark.parametrize("hd", [64, 128])
def test_attention_decode_pre_roped(oracle, qlib, hd):
    """QIE_ATTN_PREROPED: q / new k arrive rotated (the QKV projection's RoPE epilogue);
    the kernel only appends and attends.  Same cache rows and outputs as the fused form."""
    nq, nkv, L, layer, maxc = 28, 4, 2, 0, 700
    ctxs = [1, 129, 300, 700]
    B = len(ctxs)
    QD, KD = nq * hd, nkv * hd
    kc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + 3)
    vc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + 4)
    qkv = rand_bf16(oracle, (B, QD + 2 * KD), seed=6)
    pos = np.array(ctxs, np.int32) - 1
    cs, sn = oracle.rope_table(maxc, hd, 1e6, "ref")
    q = oracle.rope(qkv[:, :QD].copy(), cs, sn, pos, nq, hd, "ref")
    k = oracle.rope(qkv[:, QD:QD + KD].copy(), cs, sn, pos, nkv, hd, "ref")
    v = qkv[:, QD + KD:].copy()
    pre = np.concatenate([q, k, v], axis=1)
    ws = G.zeros_bytes(qlib.qie_attention_decode_workspace_bytes(B, nq, nkv, hd, maxc))
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    out = G.zeros_bf16(B, QD)
    c = _cache(kc, vc, L, nkv, hd, maxc, L * nkv * maxc * hd)
    dcs, dsn, dqkv, dpos = G.dev(cs), G.dev(sn), G.dev(pre), G.dev(pos)
    G.check(qlib.qie_attention_decode(G.p(dqkv), B, G.p(dpos), None, None, G.p(dcs), G.p(dsn), nq, C.byref(c),
                                      layer, 1e-6, _lib.QIE_ATTN_PREROPED, G.p(out), G.p(ws), None))
    got = G.host_bf16(out)
    hk = G.host_bf16(kc).reshape(B, L, nkv, maxc, hd)
    hv = G.host_bf16(vc).reshape(B, L, nkv, maxc, hd)
    for b in range(B):
        p = pos[b]
        assert np.array_equal(hk[b, layer, :, p], k[b].reshape(nkv, hd))
        assert np.array_equal(hv[b, layer, :, p], v[b].reshape(nkv, hd))
        kk = kc_h[b, layer, :, :p + 1].copy()
        vv = vc_h[b, layer, :, :p + 1].copy()
        kk[:, p] = k[b].reshape(nkv, hd)
        vv[:, p] = v[b].reshape(nkv, hd)
        want = oracle.attention(q[b:b + 1], kk, vv, nq, nkv, hd, False, 0)
        d = np.abs(G.bf(got[b]) - G.bf(want[0]))
        assert d.max() <= 2 ** -7 * max(1.0, np.abs(G.bf(want[0])).max()) * 2, f"ctx {ctxs[b]}: {d.max()}"
    assert not G.host(ws)[:B * nkv * 4].any()
