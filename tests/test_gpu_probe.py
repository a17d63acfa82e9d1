"""GPU structure probes for the MFMA flash-attention prefill kernel: inputs chosen so each
stage (P.V, Q.K^T + softmax) is checked in isolation against closed forms."""
import ctypes as C
import os

import numpy as np
import pytest

import gpu_util as G

from qwen_inference_engine_amd._lib import KvCacheC

pytestmark = pytest.mark.gpu


def run_prefill_attn(qlib, q, k, v, hd, nq, nkv):
    P = q.shape[0]
    maxc = max(64, P)
    kc = np.zeros((1, 1, nkv, maxc, hd), np.uint16)
    vc = np.zeros_like(kc)
    kc[0, 0, :, :P] = k
    vc[0, 0, :, :P] = v
    dk, dv = G.dev(kc), G.dev(vc)
    c = KvCacheC()
    c.k, c.v, c.seq_stride = dk.ptr, dv.ptr, nkv * maxc * hd
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = 1, nkv, hd, maxc
    out = G.zeros_bf16(P, nq * hd)
    ws = G.zeros_bytes(qlib.qie_attention_workspace_bytes(P, nq, hd, maxc))
    G.check(qlib.qie_attention(G.p(G.dev(q)), P, G.p(G.dev(np.arange(P, dtype=np.int32))), P, C.byref(c), 0, nq,
                               G.p(out), G.p(ws), None))
    return G.bf(G.host_bf16(out))


def test_tr16_lane_mapping(qlib):
    """Records what ds_read_b64_tr_b16 delivers per lane (written to gpurun_out/) and
    checks the mapping the flash kernel assumes: within each 16-lane group, lane
    4q + p supplies row q / columns 4p..4p+3 of a 4 x 16 block and lane i receives
    column i of the 4 rows (element q = row q)."""
    out = G.zeros((64 * 4,), np.int32)
    G.check(qlib.qie_debug_tr16_probe(G.p(out)))
    got = G.host(out).reshape(64, 4)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savetxt("gpurun_out/tr16_probe.txt", got, fmt="%d")
    # element index held by LDS at (lane L, e) is 4L + e; under the assumed mapping lane
    # i of group g receives, for element q, the value loaded by lane 16g + 4q + i//4 at
    # position i % 4.
    want = np.zeros_like(got)
    for lane in range(64):
        gq, i = lane // 16, lane % 16
        for q in range(4):
            src = 16 * gq + 4 * q + i // 4
            want[lane, q] = 4 * src + i % 4
    assert np.array_equal(got, want), "tr16 mapping differs; see gpurun_out/tr16_probe.txt"


@pytest.mark.parametrize("hd", [64, 128])
def test_flash_pv_uniform(oracle, qlib, hd):
    """Q = 0: every score is 0, so O[q] = mean(V[0..q])."""
    P = 64
    rng = np.random.default_rng(0)
    v = oracle.f32_to_bf16(rng.standard_normal((1, P, hd)).astype(np.float32))
    q = np.zeros((P, hd), np.uint16)
    k = oracle.f32_to_bf16(rng.standard_normal((1, P, hd)).astype(np.float32))
    got = run_prefill_attn(qlib, q, k, v, hd, 1, 1)
    vf = G.bf(v[0]).astype(np.float64)
    want = np.cumsum(vf, 0) / np.arange(1, P + 1)[:, None]
    err = np.abs(got - want)
    rows = np.where(err.max(1) > 2e-2)[0]
    assert not len(rows), f"rows {rows[:10]} wrong; first bad row err {err[rows[0]].max() if len(rows) else 0}"


def test_flash_probabilities_onehot_v(oracle, qlib):
    """V[key] = e_key (hd = 64 >= P): O[q][d] = softmax probability of key d for query q."""
    P, hd = 48, 64
    rng = np.random.default_rng(1)
    q = oracle.f32_to_bf16(rng.standard_normal((P, hd)).astype(np.float32))
    k = oracle.f32_to_bf16(rng.standard_normal((1, P, hd)).astype(np.float32))
    v = np.zeros((1, P, hd), np.uint16)
    for t in range(P):
        v[0, t, t] = 0x3F80   # 1.0
    got = run_prefill_attn(qlib, q, k, v, hd, 1, 1)
    s = G.bf(q).astype(np.float64) @ G.bf(k[0]).astype(np.float64).T / np.sqrt(hd)
    s[np.triu_indices(P, 1)] = -np.inf
    p = np.exp(s - s.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    err = np.abs(got[:, :P] - p)
    bad = np.argwhere(err > 1e-2)
    assert not len(bad), f"{len(bad)} bad (q, key) entries, e.g. {bad[:8].tolist()}"
