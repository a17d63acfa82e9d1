"""GPU: the reference's operator tier (include/qie/compat.hpp over qie_ops.h) against the
oracle — standalone qk-norm / RoPE / KV write / SiLU / element-mul ops, and the
reference's own layer loop (qwen_main.cu:77-241 prefill, :250-405 decode) written only
against those names (csrc/tools/compat_loop.cpp) on Qwen3-family models (qk-norm, no
bias; the reference's model, utills.cu:8-16), teacher-forced against or_forward.

Bars (written per check): RoPE, KV write, SiLU and element-mul bit-exact (same fp32
expression, one rounding); qk-norm bit-exact in REF mode (the reference's tree order is
reproduced); layer-loop logits and greedy ids under tests/parity.py's bar (norm-relative
error within max(1e-3, 2 x the oracle's own order spread), near-ties counted)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import gpu_util as G
from conftest import ROOT, rng
from parity import OrderPair, check_step, max_flips, oracle_trace

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W

pytestmark = pytest.mark.gpu
LOOP = os.path.join(ROOT, "qwen_inference_engine_amd", "lib", "compat_loop")


def rand_bf16(oracle, shape, seed, scale=1.0):
    return oracle.f32_to_bf16((rng(seed).standard_normal(shape) * scale).astype(np.float32))


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("num", ["ref", "hf"])
def test_qknorm_standalone(oracle, qlib, hd, num):
    rows, nh = 37, 5
    stride = nh * hd + 64   # padded rows: only the heads are touched
    x = rand_bf16(oracle, (rows, stride), 1)
    w = oracle.f32_to_bf16((1 + 0.3 * rng(2).standard_normal(hd)).astype(np.float32))
    want = oracle.qknorm(x, w, nh, hd, 1e-4, num)
    d = G.dev(x)
    G.check(qlib.qie_qknorm(G.p(d), rows, stride, nh, hd, G.p(G.dev(w)), 1e-4, 0 if num == "ref" else 1, None))
    got = G.host_bf16(d)
    assert np.array_equal(got[:, nh * hd:], x[:, nh * hd:])
    if num == "ref":
        assert np.array_equal(got, want)
    else:   # transformers' order: the sequential sum may flip a rounding
        G.assert_bf16_close(got, want, 1, 0.99, "qknorm hf")


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("num", ["ref", "hf"])
@pytest.mark.parametrize("mode", ["pos0", "pos"])
def test_rope_standalone(oracle, qlib, hd, num, mode):
    rows, nh, maxc = 23, 6, 4096
    x = rand_bf16(oracle, (rows, nh * hd), 3)
    cs, sn = oracle.rope_table(maxc, hd, 1e6, num)
    pos = (np.arange(rows) + 1000) if mode == "pos0" else rng(4).integers(0, maxc, rows)
    pos = pos.astype(np.int32)
    want = oracle.rope(x, cs, sn, pos, nh, hd, num)
    d = G.dev(x)
    dp = G.dev(pos) if mode == "pos" else None
    G.check(qlib.qie_rope(G.p(d), rows, nh * hd, nh, hd, G.p(dp), 1000 if mode == "pos0" else 0,
                          G.p(G.dev(cs)), G.p(G.dev(sn)), 0 if num == "ref" else 1, None))
    assert np.array_equal(G.host_bf16(d), want)


def test_silu_and_mul_standalone(oracle, qlib):
    n = 8 * 1000
    g = rand_bf16(oracle, n, 5, 3.0)
    u = rand_bf16(oracle, n, 6)
    want = oracle.silu_mul(g, u)
    dg, du, dh = G.dev(g), G.dev(u), G.zeros_bf16(n)
    G.check(qlib.qie_silu(G.p(dg), n, None))
    G.check(qlib.qie_mul(G.p(du), G.p(dg), G.p(dh), n, None))
    assert np.array_equal(G.host_bf16(dh), want)


@pytest.mark.parametrize("paged", [False, True])
def test_kv_write_into_batch_slot(oracle, qlib, paged):
    """qie_kv_write through qie_batch_kv_cache / qie_batch_reserve lands every row where the
    engine's own attention reads it: prefill rows written op by op == the engine's prefill."""
    spec = S.tiny("t-kv", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=1000,
                  bias=False, qk_norm=True)
    eng = Q.Engine(spec, max_ctx=300).init_synthetic(W.SynthParams(seed=3))
    b = eng.batch(2, 300, page_tokens=128 if paged else None)
    L = _lib.load()
    n, KD = 200, spec.n_kv_heads * spec.head_dim
    k = rand_bf16(oracle, (n, KD), 7)
    v = rand_bf16(oracle, (n, KD), 8)
    b.reserve(1, n)

    c = b.kv_cache(1)
    dk, dv = G.dev(k), G.dev(v)
    G.check(L.qie_kv_write(G.p(dk), G.p(dv), n, KD, 0, C.byref(c), 0, 1, None))
    G.check(L.qie_kv_write(G.p(dk), G.p(dv), 1, KD, n, C.byref(c), 0, 0, None))   # decode-style single row
    got = b.kv_rows(1, 1, n)
    assert np.array_equal(got[0], k.reshape(n, spec.n_kv_heads, spec.head_dim).transpose(1, 0, 2))
    assert np.array_equal(got[1], v.reshape(n, spec.n_kv_heads, spec.head_dim).transpose(1, 0, 2))
    row0 = b.kv_rows(1, 0, n + 1)
    assert np.array_equal(row0[0][:, n], k[0].reshape(spec.n_kv_heads, spec.head_dim))


def run_loop(spec, syn_seed, prompt, G_steps, forced, paged, tmp_path):
    out = str(tmp_path / "loop.bin")
    args = [LOOP, out, spec.n_layers, spec.hidden, spec.n_heads, spec.n_kv_heads, spec.head_dim, spec.ffn,
            spec.vocab, repr(float(spec.rms_eps)), repr(float(spec.rope_theta)), syn_seed, int(paged), G_steps,
            len(prompt), *prompt, len(forced), *forced]
    r = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    raw = np.fromfile(out, np.uint8)
    rec = 4 + 2 * spec.vocab
    assert raw.size == rec * (G_steps + 1)
    toks, lgs = [], []
    for i in range(G_steps + 1):
        blk = raw[i * rec:(i + 1) * rec]
        toks.append(int(blk[:4].view(np.int32)[0]))
        lgs.append(blk[4:].view(np.uint16).copy())
    return toks, lgs


@pytest.mark.parametrize("name,paged", [("tiny-g4", False), ("tiny-g4", True), ("qwen3-14b-2l", False)])
def test_reference_layer_loop_matches_oracle(oracle, name, paged, tmp_path):
    if name == "tiny-g4":
        spec = S.tiny("t-loop", n_layers=3, hidden=512, n_heads=8, n_kv_heads=2, head_dim=128, ffn=1024,
                      vocab=2048, bias=False, qk_norm=True)
        P, n_new = 150, 12    # 150 + 12 positions cross the first 128-token page
    else:   # the reference's model at its real widths (utills.cu:8-16), 2 layers; GQA group 5
        spec = S.QWEN3_14B.replace(n_layers=2)
        P, n_new = 40, 6
    syn = W.SynthParams(seed=5, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
    om = OrderPair(oracle, W.HostWeights.synthetic(spec, syn), P + n_new + 8)
    prompt = [int(t) for t in rng(P).integers(0, spec.vocab, P)]
    ids, outs = oracle_trace(oracle, om, prompt, n_new + 1)
    om.calibrate(spec.vocab)
    toks, lgs = run_loop(spec, 5, prompt, n_new, ids[:-1], paged, tmp_path)
    flips = 0
    for i in range(n_new + 1):
        flips += check_step(lgs[i], outs[i][0], om, toks[i], ids[i], f"step {i}")
    assert flips <= max_flips(n_new + 1)


DRIVER = os.path.join(ROOT, "qwen_inference_engine_amd", "lib", "ref_driver")


@pytest.mark.parametrize("name", ["qwen3-like", "qwen2-like-tied"])
def test_reference_signature_driver_matches_oracle(oracle, name, tmp_path):
    """csrc/tools/ref_driver.cpp: a host written only against the reference's driver-tier
    argument lists (llm(seq, tensors, ifstream&, page_table*, page_size, bf16*),
    create_new_sequence(id, ids, len, tensors, ifstream&), create_page_list(n),
    allocate_page_buffers(node, elems), load_all_weights_to_gpu_chunked(all, ifstream&,
    h_host, chunk, d_base&, total&), parsed_tensors(), build_indexed_tensors()) in the call
    order of iengine.cu:226-456, over a weights.bin + meta_data.txt written in the
    reference's flat layout.  Its greedy tokens (llm() fed back generated_token) against
    or_forward teacher-forced on them: every token the oracle's arg-max or a near-tie within
    the oracle's own order spread (tests/parity.py), at most max_flips."""
    if name == "qwen3-like":   # the reference's model family (qk-norm, no bias, untied)
        spec = S.tiny("t-drv3", n_layers=3, hidden=512, n_heads=8, n_kv_heads=2, head_dim=128, ffn=1024,
                      vocab=4096, bias=False, qk_norm=True)
    else:
        spec = S.tiny("t-drv2", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512,
                      vocab=2048, bias=True, qk_norm=False, tie=True)
    syn = W.SynthParams(seed=9, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
    hw = W.HostWeights.synthetic(spec, syn)
    wb, meta = str(tmp_path / "weights.bin"), str(tmp_path / "meta_data.txt")
    hw.write_weights_bin(wb, meta)
    prompt = [int(t) for t in rng(31).integers(0, spec.vocab, 21)]
    n = 16
    sp = ",".join(str(v) for v in (spec.n_layers, spec.hidden, spec.n_heads, spec.n_kv_heads, spec.head_dim,
                                   spec.ffn, spec.vocab, int(spec.tie_embeddings), int(spec.qkv_bias),
                                   int(spec.qk_norm), repr(float(spec.rms_eps)), repr(float(spec.rope_theta))))
    r = subprocess.run([DRIVER, "--weights", wb, "--meta", meta, "--spec", sp, "--greedy", "--gen", str(n),
                        "--max-ctx", "128", "--prompt", ",".join(map(str, prompt))],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    got = [int(t) for t in [l for l in r.stdout.splitlines() if l.startswith("tokens:")][0].split()[1:]]
    assert len(got) == n
    pair = OrderPair(oracle, hw, len(prompt) + n + 4)
    ids, outs = oracle_trace(oracle, pair, prompt, n, forced=got[:-1])
    pair.calibrate(spec.vocab)
    flips = 0
    for i, (t, (lg0, _)) in enumerate(zip(got, outs)):
        if t != ids[i]:
            gap = abs(float(G.bf(lg0[ids[i]])) - float(G.bf(lg0[t])))
            assert gap <= pair.bars(lg0)[1], f"step {i}: driver {t} vs oracle {ids[i]}, gap {gap}"
            flips += 1
    assert flips <= max_flips(n)
