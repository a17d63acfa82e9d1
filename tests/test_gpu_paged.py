"""GPU: the paged KV cache (device block table) against the contiguous
cache.  Paging changes only where a (sequence, layer, kv head, token) row lives, never the
arithmetic, so every check here is BIT-EXACT: the same op on the same rows gives the same
bytes whether the rows sit in one contiguous run per sequence or scattered over a pool of
pages in a shuffled order (page 0, the scratch page, is filled with garbage to catch a
wrong lookup).  The contiguous path itself is pinned to the oracle by test_gpu_ops.py /
test_gpu_engine.py.

Reference behaviour replaced: the linked page list of iengine.cu:73-109 (create_page_list,
allocate_page_buffers, free_page_list) walked by include_cuda.cu:165-279.
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as G
from conftest import rng

import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import _lib, spec as S, weights as W
from qwen_inference_engine_amd._lib import KvCacheC

pytestmark = pytest.mark.gpu


def rand_bf16(oracle, shape, scale=1.0, seed=0):
    return oracle.f32_to_bf16((rng(seed).standard_normal(shape) * scale).astype(np.float32))


def _contig(kc, vc, L, nkv, hd, maxc):
    c = KvCacheC()
    c.k, c.v, c.seq_stride = G.p(kc), G.p(vc), L * nkv * maxc * hd
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = L, nkv, hd, maxc
    return c


class Paged:
    """A paged copy of a contiguous host cache [B][L][nkv][maxc][hd]: sequence b's page j
    is pool page table[b][j] (a shuffled permutation of 1..), page 0 holds garbage."""

    def __init__(self, oracle, kc_h, vc_h, T, seed=0):
        B, L, nkv, maxc, hd = kc_h.shape
        self.B, self.L, self.nkv, self.maxc, self.hd, self.T = B, L, nkv, maxc, hd, T
        self.mp = (maxc + T - 1) // T
        self.n_pages = B * self.mp + 1
        perm = rng(seed + 99).permutation(np.arange(1, self.n_pages)).astype(np.int32)
        self.table = perm.reshape(B, self.mp)
        self.kp = self._pool(oracle, kc_h, seed)
        self.vp = self._pool(oracle, vc_h, seed + 1)
        self.dk, self.dv, self.dt = G.dev(self.kp), G.dev(self.vp), G.dev(self.table)

    def _pool(self, oracle, h, seed):
        B, L, nkv, maxc, hd, T = self.B, self.L, self.nkv, self.maxc, self.hd, self.T
        pool = rand_bf16(oracle, (self.n_pages, L, nkv, T, hd), 4.0, seed=seed + 1234)   # garbage everywhere
        for b in range(B):
            for j in range(self.mp):
                n = min(T, maxc - j * T)
                pool[self.table[b, j], :, :, :n] = h[b, :, :, j * T:j * T + n]
        return pool

    def cache(self, seq0=0):
        c = KvCacheC()
        c.k, c.v, c.seq_stride = G.p(self.dk), G.p(self.dv), self.L * self.nkv * self.T * self.hd
        c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = self.L, self.nkv, self.hd, self.maxc
        c.block_table = G.p(self.dt) + seq0 * self.mp * 4
        c.page_tokens, c.max_pages = self.T, self.mp
        return c

    def gather(self, pool_dev):
        """Device pool -> contiguous [B][L][nkv][maxc][hd] view."""
        pool = G.host_bf16(pool_dev).reshape(self.n_pages, self.L, self.nkv, self.T, self.hd)
        out = np.zeros((self.B, self.L, self.nkv, self.mp * self.T, self.hd), np.uint16)
        for b in range(self.B):
            for j in range(self.mp):
                out[b, :, :, j * self.T:(j + 1) * self.T] = pool[self.table[b, j]]
        return out[:, :, :, :self.maxc]


@pytest.mark.parametrize("hd,nq,nkv", [(128, 28, 4), (64, 14, 2)])
@pytest.mark.parametrize("T", [128, 256])
def test_paged_decode_attention_equals_contiguous(oracle, qlib, hd, nq, nkv, T):
    """Fused decode attention (qk-norm + RoPE + KV append + split attention): contexts on,
    just past and far past page boundaries; the new token's K/V row lands in its page."""
    L, layer, maxc = 2, 1, 700
    ctxs = [1, 128, 129, 257, 700]
    B = len(ctxs)
    QD, KD = nq * hd, nkv * hd
    kc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd)
    vc_h = rand_bf16(oracle, (B, L, nkv, maxc, hd), seed=hd + 1)
    qkv = rand_bf16(oracle, (B, QD + 2 * KD), seed=5)
    pos = np.array(ctxs, np.int32) - 1
    qn = oracle.f32_to_bf16((1 + 0.3 * rng(1).standard_normal(hd)).astype(np.float32))
    kn = oracle.f32_to_bf16((1 + 0.3 * rng(2).standard_normal(hd)).astype(np.float32))
    cs, sn = oracle.rope_table(maxc, hd, 1e6, "ref")
    dcs, dsn, dqkv, dpos, dqn, dkn = G.dev(cs), G.dev(sn), G.dev(qkv), G.dev(pos), G.dev(qn), G.dev(kn)
    outs = []
    kc, vc = G.dev(kc_h), G.dev(vc_h)
    pg = Paged(oracle, kc_h, vc_h, T)
    for c in (_contig(kc, vc, L, nkv, hd, maxc), pg.cache()):
        ws = G.zeros_bytes(qlib.qie_attention_decode_workspace_bytes(B, nq, nkv, hd, maxc))
        out = G.zeros_bf16(B, QD)
        G.check(qlib.qie_attention_decode(G.p(dqkv), B, G.p(dpos), G.p(dqn), G.p(dkn), G.p(dcs), G.p(dsn), nq,
                                          C.byref(c), layer, 1e-4, 0, G.p(out), G.p(ws), None))
        outs.append(G.host_bf16(out))
    assert np.array_equal(outs[0], outs[1])
    # appended rows: the paged pool, gathered back through the table, equals the contiguous cache
    assert np.array_equal(pg.gather(pg.dk), G.host_bf16(kc).reshape(kc_h.shape))
    assert np.array_equal(pg.gather(pg.dv), G.host_bf16(vc).reshape(vc_h.shape))
    # and nothing was written to the scratch page
    assert np.array_equal(G.host_bf16(pg.dk).reshape(pg.kp.shape)[0], pg.kp[0])


@pytest.mark.parametrize("P,hd", [(7, 64), (200, 64), (300, 128), (513, 128)])
def test_paged_prefill_equals_contiguous(oracle, qlib, P, hd):
    """Prefill q/k post (KV rows written across page boundaries) + causal attention
    (MFMA flash kernel for P >= 32, the split kernel below) through the block table, for
    two sequences in one call (rows_per_seq = P)."""
    nq, nkv, L, layer, T = 8, 2, 2, 1, 128
    maxc = 600
    nseq = 2
    M = nseq * P
    QD, KD = nq * hd, nkv * hd
    qkv = rand_bf16(oracle, (M, QD + 2 * KD), seed=P)
    pos = np.tile(np.arange(P, dtype=np.int32), nseq)
    cs, sn = oracle.rope_table(maxc, hd, 1e6, "hf")
    dqkv, dpos, dcs, dsn = G.dev(qkv), G.dev(pos), G.dev(cs), G.dev(sn)
    zero = np.zeros((nseq, L, nkv, maxc, hd), np.uint16)
    kc, vc = G.dev(zero), G.dev(zero)
    pg = Paged(oracle, zero, zero, T, seed=P)
    res = []
    for c in (_contig(kc, vc, L, nkv, hd, maxc), pg.cache()):
        q = G.zeros_bf16(M, QD)
        G.check(qlib.qie_qkv_post(G.p(dqkv), M, G.p(dpos), P, None, None, G.p(dcs), G.p(dsn), nq, C.byref(c), layer,
                                  1e-6, 1, G.p(q), None))
        ws = G.zeros_bytes(qlib.qie_attention_workspace_bytes(M, nq, hd, maxc))
        out = G.zeros_bf16(M, QD)
        G.check(qlib.qie_attention(G.p(q), M, G.p(dpos), P, C.byref(c), layer, nq, G.p(out), G.p(ws), None))
        res.append((G.host_bf16(q), G.host_bf16(out)))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
    hk = G.host_bf16(kc).reshape(zero.shape)
    gk = pg.gather(pg.dk)
    assert np.array_equal(gk[:, :, :, :P], hk[:, :, :, :P])
    assert np.array_equal(pg.gather(pg.dv)[:, :, :, :P], G.host_bf16(vc).reshape(zero.shape)[:, :, :, :P])


def test_paged_cache_descriptor_validation(qlib):
    d = G.zeros_bf16(1 << 16)
    t = G.dev(np.zeros(4, np.int32))
    c = KvCacheC()
    c.k = c.v = G.p(d)
    c.n_layers, c.n_kv_heads, c.head_dim, c.max_ctx = 1, 1, 64, 256
    c.block_table, c.seq_stride, c.max_pages = G.p(t), 1 * 1 * 128 * 64, 2
    out = G.zeros_bf16(1, 64)
    pos = G.dev(np.zeros(1, np.int32))
    for T, mp in [(96, 3), (64, 4), (128, 1)]:   # not a power of two >= 128 / table row too short
        c.page_tokens, c.max_pages = T, mp
        assert qlib.qie_attention(G.p(G.dev(np.zeros((1, 64), np.uint16))), 1, G.p(pos), 1, C.byref(c), 0, 1,
                                  G.p(out), None, None) != 0


# ------------------------------------------------------------------------- engine
SPEC = S.tiny("t-paged", n_layers=2, hidden=256, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, vocab=1000,
              bias=True)
SPEC128 = S.tiny("t-paged128", n_layers=2, hidden=512, n_heads=8, n_kv_heads=2, head_dim=128, ffn=768,
                 vocab=1536, bias=False, qk_norm=True)
SYN = W.SynthParams(seed=11, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)


def _run(b, prompts, n_steps, script=()):
    """Prefill every slot, decode n_steps; `script` = [(step, seq, new prompt | None)]
    releases a slot (None) or re-prefills it at that step.  Returns ids + per-step logits."""
    ids = [[b.prefill(i, pr)] for i, pr in enumerate(prompts)]
    lgs = [b.logits()]
    ev = {}
    for st, seq, pr in script:
        ev.setdefault(st, []).append((seq, pr))
    for t in range(n_steps):
        for seq, pr in ev.get(t, []):
            if pr is None:
                b.release(seq)
            else:
                ids[seq].append(("new", b.prefill(seq, pr)))
        nxt = b.decode_step()
        for i in range(len(prompts)):
            ids[i].append(nxt[i])
        lgs.append(b.logits())
    return ids, np.stack(lgs)


@pytest.mark.parametrize("spec", [SPEC, SPEC128], ids=["hd64", "hd128"])
@pytest.mark.parametrize("B", [1, 3])
def test_paged_batch_equals_contiguous(spec, B):
    """Generation through a paged batch == a contiguous batch, ids and logits bit for bit,
    across 128-token page boundaries (prompts 100..140 tokens, 150 steps)."""
    eng = Q.Engine(spec, max_ctx=320).init_synthetic(SYN)
    prompts = [list(rng(i).integers(0, spec.vocab, n)) for i, n in enumerate([127, 100, 140][:B])]
    a = _run(eng.batch(B, 320), prompts, 150)
    pb = eng.batch(B, 320, page_tokens=128)
    b = _run(pb, prompts, 150)
    assert a[0] == b[0]
    assert np.array_equal(a[1], b[1])
    free, per, T = pb.page_stats()
    assert T == 128 and list(per) == [(len(p) + 150 + 127) // 128 for p in prompts]
    tabs = [pb.block_table(i, per[i]) for i in range(B)]
    flat = np.concatenate(tabs)
    assert len(set(flat.tolist())) == len(flat) and 0 not in flat   # distinct pages, never the scratch page


def test_paged_release_reuse_and_exhaustion():
    """Continuous batching: a slot released mid-run returns its pages, a new prompt
    prefilled into it reuses them, and the other slots are unaffected — identical, bit
    for bit, to the same script on a contiguous batch.  A pool too small fails loudly."""
    eng = Q.Engine(SPEC, max_ctx=512).init_synthetic(SYN)
    prompts = [list(rng(10 + i).integers(0, SPEC.vocab, n)) for i, n in enumerate([60, 200, 90])]
    newp = list(rng(77).integers(0, SPEC.vocab, 150))
    script = [(20, 1, None), (40, 1, newp)]
    a = _run(eng.batch(3, 512), prompts, 120, script)
    # 7 usable pages (+ scratch): the run needs 2 per slot at a time but 8 over its life,
    # so the new sequence in slot 1 must reuse the pages its release returned
    pb = eng.batch(3, 512, page_tokens=128, n_pages=8)
    b = _run(pb, prompts, 120, script)
    assert a[0][0] == b[0][0] and a[0][2] == b[0][2]
    assert np.array_equal(a[1][:, [0, 2]], b[1][:, [0, 2]])        # live slots throughout
    # slot 1: its first sequence, then the new one (idle steps in between read the
    # scratch page vs stale rows, so their meaningless ids differ)
    k = [i for i, x in enumerate(a[0][1]) if isinstance(x, tuple)][0]
    assert a[0][1][:21] == b[0][1][:21] and a[0][1][k:] == b[0][1][k:]
    assert np.array_equal(a[1][:21, 1], b[1][:21, 1]) and np.array_equal(a[1][41:, 1], b[1][41:, 1])
    free, per, _ = pb.page_stats()
    assert free == 7 - int(per.sum())
    pb.release(0)
    assert pb.page_stats()[0] == free + per[0]
    with pytest.raises(_lib.QieError):
        pb.prefill(0, list(rng(5).integers(0, SPEC.vocab, 511)))   # 4 pages, not that many free
    small = eng.batch(1, 512, page_tokens=128, n_pages=2)
    small.prefill(0, [1, 2, 3])
    small.decode(100)
    with pytest.raises(_lib.QieError):
        small.decode(40)   # would cross into a second page: pool exhausted, nothing launched
    assert small.positions()[0] == 103


def test_continuous_batcher_matches_isolated_runs():
    """The serving loop (qwen_inference_engine_amd.scheduler): 6 requests through 3 slots of
    a paged batch whose pool (5 usable pages) holds fewer than all of them, so requests
    wait, join mid-run and reuse released pages.  Slot rows are independent, so every
    request's tokens must equal — bit for bit — the same request run alone in slot 0 of
    a fresh 3-slot contiguous batch."""
    from qwen_inference_engine_amd.scheduler import ContinuousBatcher
    eng = Q.Engine(SPEC, max_ctx=512).init_synthetic(SYN)
    lens = [30, 150, 7, 90, 200, 60]
    new = [40, 20, 100, 1, 30, 64]
    prompts = [list(rng(50 + i).integers(0, SPEC.vocab, n)) for i, n in enumerate(lens)]
    cb = ContinuousBatcher(eng, slots=3, max_ctx=512, page_tokens=128, n_pages=6)
    rids = [cb.submit(p, n) for p, n in zip(prompts, new)]
    saw_wait = False
    while not cb.idle():
        cb.step()
        saw_wait |= len(cb.waiting) > 0 and any(s is not None for s in cb.slots)
    got = {rid: cb.requests[rid].tokens for rid in rids}
    assert saw_wait
    assert cb.batch.page_stats()[0] == 5 and cb.budget == 5    # every page back in the pool
    for rid, p, n in zip(rids, prompts, new):
        b = eng.batch(3, 512)
        want = [b.prefill(0, p)]
        while len(want) < n:
            want.append(b.decode_step()[0])
        b.close()
        assert got[rid] == want, f"request {rid}"


def test_batcher_unused_slots_long_run_matches_oracle(oracle):
    """More slots than concurrent requests and more total steps than max_ctx, on a pool
    with one spare page: unused slots idle from creation (no pool pages, rewound before
    max_ctx), so the run never exhausts the pool.  Every request's tokens and logits are
    checked against or_forward, the oracle following the batcher's own tokens (so a
    near-tie never derails the comparison): logits within 4 bf16 ulps of max|logit|, and
    each chosen token the oracle's arg-max or a near-tie within that tolerance."""
    from qwen_inference_engine_amd.scheduler import ContinuousBatcher
    from test_gpu_engine import logit_tol
    eng = Q.Engine(SPEC, max_ctx=256).init_synthetic(SYN)
    hw = W.HostWeights.synthetic(SPEC, SYN)
    cb = ContinuousBatcher(eng, slots=4, max_ctx=256, page_tokens=128, n_pages=3, keep_logits=True)
    reqs, steps = [], 0
    for i in range(4):   # one request at a time: 3 slots stay unused throughout
        pr = [int(t) for t in rng(90 + i).integers(0, SPEC.vocab, 20 + 30 * i)]
        rid = cb.submit(pr, 100)
        while not cb.idle():
            cb.step()
            steps += 1
        reqs.append((rid, pr))
    assert steps > 256                                 # longer than max_ctx in total
    assert cb.batch.page_stats()[0] == 2               # every page back in the pool
    flips = 0
    for rid, pr in reqs:
        r = cb.requests[rid]
        om = oracle.Model(hw, 256)
        lg = om.forward(pr, 0)
        for t, (tok, got) in enumerate(zip(r.tokens, r.logits)):
            d = np.abs(G.bf(got).astype(np.float64) - G.bf(lg))
            assert d.max() <= logit_tol(lg), f"request {rid} token {t}: {d.max()}"
            want = oracle.argmax(lg)
            if tok != want:
                assert abs(float(G.bf(lg[want])) - float(G.bf(lg[tok]))) <= logit_tol(lg)
                flips += 1
            if t + 1 < len(r.tokens):
                lg = om.forward([tok])
    from parity import max_flips
    assert flips <= max_flips(sum(len(cb.requests[rid].tokens) for rid, _ in reqs))


def test_failed_reprefill_leaves_live_slot_intact():
    """A prefill into a live slot that the pool cannot hold fails with nothing changed:
    the slot keeps its pages and continues exactly like an untouched run."""
    eng = Q.Engine(SPEC, max_ctx=512).init_synthetic(SYN)
    pr = list(rng(3).integers(0, SPEC.vocab, 100))
    ref = eng.batch(1, 512, page_tokens=128, n_pages=3)
    t0 = ref.prefill(0, pr)
    want = list(ref.decode(60)[:, 0])
    pb = eng.batch(1, 512, page_tokens=128, n_pages=3)
    assert pb.prefill(0, pr) == t0
    held = pb.page_stats()[1][0]
    with pytest.raises(_lib.QieError):
        pb.prefill(0, list(rng(4).integers(0, SPEC.vocab, 400)))   # 4 pages; 1 held + 1 free
    assert pb.page_stats()[1][0] == held
    assert list(pb.decode(60)[:, 0]) == want


def test_batcher_batched_admission_matches_oracle(oracle):
    """Four equal-length requests submitted together are admitted in one step and prefill
    in one qie_prefill_batch pass (slots 0..3, rows_per_seq 33); a fifth of another length
    waits for a free slot and prefills alone.  Every request's tokens and logits follow
    or_forward (the oracle fed the batcher's own tokens): logits within 4 bf16 ulps of
    max|logit|, each token the oracle's arg-max or a near-tie within that tolerance."""
    from qwen_inference_engine_amd.scheduler import ContinuousBatcher
    from test_gpu_engine import logit_tol
    from parity import max_flips
    eng = Q.Engine(SPEC, max_ctx=256).init_synthetic(SYN)
    hw = W.HostWeights.synthetic(SPEC, SYN)
    cb = ContinuousBatcher(eng, slots=4, max_ctx=256, page_tokens=128, keep_logits=True)
    prompts = [[int(t) for t in rng(300 + i).integers(0, SPEC.vocab, 33 if i < 4 else 21)] for i in range(5)]
    rids = [cb.submit(p, 12 + 3 * i) for i, p in enumerate(prompts)]
    cb.run()
    flips = n_tok = 0
    for rid, pr in zip(rids, prompts):
        r = cb.requests[rid]
        assert len(r.tokens) == 12 + 3 * rid
        om = oracle.Model(hw, 256)
        lg = om.forward(pr, 0)
        for t, (tok, got) in enumerate(zip(r.tokens, r.logits)):
            d = np.abs(G.bf(got).astype(np.float64) - G.bf(lg))
            assert d.max() <= logit_tol(lg), f"request {rid} token {t}: {d.max()}"
            want = oracle.argmax(lg)
            if tok != want:
                assert abs(float(G.bf(lg[want])) - float(G.bf(lg[tok]))) <= logit_tol(lg)
                flips += 1
            if t + 1 < len(r.tokens):
                lg = om.forward([tok])
        n_tok += len(r.tokens)
    assert flips <= max_flips(n_tok)


def test_prefill_batch_all_or_nothing_and_bad_arguments():
    """qie_prefill_batch on a paged pool that cannot hold every prompt fails with nothing
    launched: a live slot keeps its pages and continues exactly like an untouched run;
    slot ranges past B, prompts >= max_ctx and ragged prompts are refused."""
    eng = Q.Engine(SPEC, max_ctx=512).init_synthetic(SYN)
    pr = list(rng(5).integers(0, SPEC.vocab, 100))
    ref = eng.batch(3, 512, page_tokens=128, n_pages=4)
    t0 = ref.prefill(0, pr)
    want = list(ref.decode(40)[:, 0])
    pb = eng.batch(3, 512, page_tokens=128, n_pages=4)   # page 0 scratch + 3
    assert pb.prefill(0, pr) == t0
    stats = pb.page_stats()
    two = [list(rng(6 + z).integers(0, SPEC.vocab, 200)) for z in range(2)]
    with pytest.raises(_lib.QieError):
        pb.prefill_batch(1, two)            # 2 x 2 pages; 2 free
    assert pb.page_stats()[0] == stats[0] and list(pb.page_stats()[1]) == list(stats[1])
    with pytest.raises(_lib.QieError):
        pb.prefill_batch(2, two)            # slots 2..3 of 3
    with pytest.raises(_lib.QieError):
        pb.prefill_batch(1, [[1] * 512, [2] * 512])   # >= max_ctx
    with pytest.raises(ValueError):
        pb.prefill_batch(1, [[1, 2, 3], [4, 5]])
    assert list(pb.decode(40)[:, 0]) == want


def test_prefill_batch_into_live_slots_reuses_their_pages():
    """Re-prefilling live slots whose pages are all the pool has: slot 0 holds 1 page, slot
    1 holds 3, none free; two 200-token prompts need 2 pages each.  The all-or-nothing
    check counts the held pages (4 <= 0 + 4), so the call must succeed — every target slot
    returns its pages before any draws (a slot-by-slot drop-then-draw ran dry at slot 0) —
    and generate exactly what the same prompts do in a fresh batch."""
    eng = Q.Engine(SPEC, max_ctx=512).init_synthetic(SYN)
    pb = eng.batch(2, 512, page_tokens=128, n_pages=5)   # page 0 scratch + 4
    pb.prefill(0, list(rng(7).integers(0, SPEC.vocab, 100)))
    pb.prefill(1, list(rng(8).integers(0, SPEC.vocab, 300)))
    free, per, _ = pb.page_stats()
    assert free == 0 and list(per) == [1, 3]
    two = [list(rng(9 + z).integers(0, SPEC.vocab, 200)) for z in range(2)]
    got = pb.prefill_batch(0, two)
    assert list(pb.page_stats()[1]) == [2, 2]
    gdec = pb.decode(20).tolist()
    fresh = eng.batch(2, 512, page_tokens=128, n_pages=5)
    assert fresh.prefill_batch(0, two) == got
    assert fresh.decode(20).tolist() == gdec
    assert np.array_equal(fresh.logits(), pb.logits())
