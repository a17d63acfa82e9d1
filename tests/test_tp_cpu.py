"""CPU check of the tensor-parallel decomposition (world_size 2 and 4, torch.distributed gloo on
127.0.0.1): each rank runs the oracle's ops on ITS shard of the synthetic weights — the
same slicing rule as the engine's plan_slice (engine.hip): q/k/v rows by heads, gate/up
rows by I, O and down columns (row-parallel, fp32 partials all-reduced, then
x = bf16(x + bf16(sum))), lm_head rows by vocab (logit shards all-gathered).  The result
must match the unsharded oracle forward within 4 bf16 ulps of max |logit| (the split
changes only fp32 summation order), and both ranks must agree bit-exactly."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SPECS = {   # key: (spec, world)
    "qwen2-bias": (dict(name="tp-q2", n_layers=2, hidden=128, n_heads=4, n_kv_heads=2, head_dim=64, ffn=256,
                        vocab=512, bias=True), 2),
    "qwen3-qknorm-tied": (dict(name="tp-q3", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=128,
                               ffn=384, vocab=640, bias=False, qk_norm=True, tie=True), 2),
    # uneven q heads with kv replication (Qwen2-7B's 28 / 4 heads at TP 8 in miniature):
    # 6 q / 2 kv heads over 4 ranks -> kv head r // 2 on each rank, q heads 2,1,2,1
    "uneven-kvrep": (dict(name="tp-uneven", n_layers=2, hidden=192, n_heads=6, n_kv_heads=2, head_dim=64, ffn=256,
                          vocab=512, bias=True), 4),
}


def shard_heads(nq, nkv, tp, r):
    """(local q heads, first q head, local kv heads, first kv head) — mirror of engine.hip
    shard_heads: even split, or kv heads replicated on tp / nkv ranks that split the
    group's q heads (the first G % rep ranks one more)."""
    if nkv % tp == 0 and nq % tp == 0:
        return nq // tp, r * (nq // tp), nkv // tp, r * (nkv // tp)
    rep, G = tp // nkv, nq // nkv
    g, sub = r // rep, r % rep
    base, extra = G // rep, G % rep
    n = base + (1 if sub < extra else 0)
    return n, g * G + sub * base + min(sub, extra), 1, g


def shard(hw, spec, name, short, tp, r):
    """This rank's slice of tensor `name` (mirror of engine.hip plan_slice)."""
    a = hw.tensors[name]
    hd = spec.head_dim
    nq, q0, nkv, k0 = shard_heads(spec.n_heads, spec.n_kv_heads, tp, r)
    ffn, V = spec.ffn // tp, spec.vocab // tp
    rows = {"self_attn.q_proj.weight": (nq * hd, q0 * hd), "self_attn.k_proj.weight": (nkv * hd, k0 * hd),
            "self_attn.v_proj.weight": (nkv * hd, k0 * hd), "mlp.gate_proj.weight": (ffn, r * ffn),
            "mlp.up_proj.weight": (ffn, r * ffn), "logits": (V, r * V)}
    cols = {"self_attn.q_proj.bias": (nq * hd, q0 * hd), "self_attn.k_proj.bias": (nkv * hd, k0 * hd),
            "self_attn.v_proj.bias": (nkv * hd, k0 * hd), "self_attn.o_proj.weight": (nq * hd, q0 * hd),
            "mlp.down_proj.weight": (ffn, r * ffn)}
    if short in rows:
        n, o = rows[short]
        return a[o:o + n]
    if short in cols:
        n, o = cols[short]
        return a[..., o:o + n]
    return a


def tp_forward(O, hw, spec, prompt, tp, r, dist, torch):
    f32 = O.bf16_to_f32
    num, eps, hd = spec.numerics, spec.rms_eps, spec.head_dim
    nq, _, nkv, _ = shard_heads(spec.n_heads, spec.n_kv_heads, tp, r)
    P = len(prompt)
    cos, sin = O.rope_table(P + 1, hd, spec.rope_theta, num)
    pos = np.arange(P, dtype=np.int32)

    def lw(l, short):
        return shard(hw, spec, f"model.layers.{l}.{short}", short, tp, r)

    def all_reduce(part):
        t = torch.from_numpy(np.ascontiguousarray(part, np.float32))
        dist.all_reduce(t)
        return t.numpy()

    x = hw.tensors["model.embed_tokens.weight"][np.asarray(prompt)]
    for l in range(spec.n_layers):
        hn = O.rmsnorm(x, hw.layer(l, "input_layernorm.weight"), eps, num)
        q = O.matmul(hn, lw(l, "self_attn.q_proj.weight"), lw(l, "self_attn.q_proj.bias") if spec.qkv_bias else None)
        k = O.matmul(hn, lw(l, "self_attn.k_proj.weight"), lw(l, "self_attn.k_proj.bias") if spec.qkv_bias else None)
        v = O.matmul(hn, lw(l, "self_attn.v_proj.weight"), lw(l, "self_attn.v_proj.bias") if spec.qkv_bias else None)
        if spec.qk_norm:
            q = O.qknorm(q, hw.layer(l, "self_attn.q_norm.weight"), nq, hd, eps, num)
            k = O.qknorm(k, hw.layer(l, "self_attn.k_norm.weight"), nkv, hd, eps, num)
        q = O.rope(q, cos, sin, pos, nq, hd, num)
        k = O.rope(k, cos, sin, pos, nkv, hd, num)
        kc = np.ascontiguousarray(k.reshape(P, nkv, hd).transpose(1, 0, 2))
        vc = np.ascontiguousarray(v.reshape(P, nkv, hd).transpose(1, 0, 2))
        att = O.attention(q, kc, vc, nq, nkv, hd, True, 0)
        part = f32(att) @ f32(lw(l, "self_attn.o_proj.weight")).T
        x = O.resadd(x, O.f32_to_bf16(all_reduce(part)))
        hn = O.rmsnorm(x, hw.layer(l, "post_attention_layernorm.weight"), eps, num)
        h = O.silu_mul(O.matmul(hn, lw(l, "mlp.gate_proj.weight")), O.matmul(hn, lw(l, "mlp.up_proj.weight")))
        part = f32(h) @ f32(lw(l, "mlp.down_proj.weight")).T
        x = O.resadd(x, O.f32_to_bf16(all_reduce(part)))
    last = O.rmsnorm(x[-1:], hw.get("model.norm.weight"), eps, num)
    head = shard(hw, spec, "model.embed_tokens.weight" if spec.tie_embeddings else "lm_head.weight", "logits", tp, r)
    mine = torch.from_numpy(O.matmul(last, head)[0].astype(np.int32))
    parts = [torch.zeros_like(mine) for _ in range(tp)]
    dist.all_gather(parts, mine)
    return np.concatenate([p.numpy() for p in parts]).astype(np.uint16)


def _rank_main(rank, world, port, key, out_dir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from qwen_inference_engine_amd import spec as S, weights as W
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = S.tiny(**SPECS[key][0])
        hw = W.HostWeights.synthetic(spec, W.SynthParams(seed=3, w_scale=0.08, norm_scale=0.25, bias_scale=0.05))
        prompt = [int(t) for t in np.random.default_rng(7).integers(0, spec.vocab, 11)]
        lg = tp_forward(O, hw, spec, prompt, world, rank, dist, torch)
        np.save(os.path.join(out_dir, f"tp{rank}.npy"), lg)
        if rank == 0:
            full = O.Model(hw, 32).forward(prompt, 0)
            np.save(os.path.join(out_dir, "full.npy"), np.asarray(full, np.uint16))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_heads_cover_every_head_once():
    """Every q head on exactly one rank; each rank's q heads inside its kv head's group."""
    for nq, nkv, tp in [(28, 4, 8), (28, 4, 4), (14, 2, 4), (14, 2, 8), (64, 8, 8), (40, 8, 8), (6, 2, 4)]:
        seen = []
        for r in range(tp):
            n, q0, m, k0 = shard_heads(nq, nkv, tp, r)
            assert n >= 1 and m >= 1
            G = nq // nkv
            assert all((q0 + i) // G in range(k0, k0 + m) for i in range(n))
            seen += list(range(q0, q0 + n))
        assert sorted(seen) == list(range(nq)), (nq, nkv, tp)
    assert [shard_heads(28, 4, 8, r)[0] for r in range(8)] == [4, 3] * 4


@pytest.mark.parametrize("key", list(SPECS))
def test_tp_decomposition_matches_oracle(key, tmp_path, oracle):
    import torch.multiprocessing as mp
    world = SPECS[key][1]
    mp.spawn(_rank_main, args=(world, _free_port(), key, str(tmp_path)), nprocs=world, join=True)
    lgs = [np.load(tmp_path / f"tp{r}.npy") for r in range(world)]
    t0, full = lgs[0], np.load(tmp_path / "full.npy")
    for t in lgs[1:]:
        assert np.array_equal(t0, t)
    bf = lambda a: (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64)  # noqa: E731
    tol = 4 * 2.0 ** -7 * max(1.0, float(np.abs(bf(full)).max()))
    assert np.abs(bf(t0) - bf(full)).max() <= tol
    assert oracle.argmax(t0) == oracle.argmax(full) or \
        abs(bf(full)[oracle.argmax(t0)] - bf(full)[oracle.argmax(full)]) <= tol
