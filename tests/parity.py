"""End-to-end parity bar shared by the GPU tests.

SURVEY §8(c) asks for logits within 1e-3 norm-relative of the reference.  The reference
itself cannot meet that against a second valid evaluation of its own arithmetic: it
rounds every op's output to bf16 and leaves the fp32 summation order of its WMMA
matmuls unspecified, so two orders already differ by ~7e-3 (matmul only) to ~9e-3 (every
reduction) norm-relative at 2 layers of Qwen2-7B widths (oracle variants 0 / 1 / 2,
measured in this container).  The bar is therefore measured per input:

* logits: norm-relative error of the engine vs the oracle (order 0) within
  max(1e-3, 2 x the norm-relative spread between oracle order 0 and order 2 — every fp32
  reduction reordered — on the same input), the spread taken as its maximum over the
  whole teacher-forced run (both orders follow the same ids, so the oracle trace is
  computed first; a single step's two orders can coincide by chance, the sensitivity is
  a property of the model and prompt, and the engine's error is held to the same
  statistic: every step within 2 x the run's worst oracle spread), together with the
  spread of a fixed calibration run of the same model (a short run can be degenerate:
  with fp8-dequantised weights every product is exact and two orders may agree on all
  of a 5-token prompt's steps, while one 1-ulp rounding of a transcendental — ocml vs
  glibc expf, both within the C standard's 1 ulp — moves the logits by ~4e-3);
* greedy ids (teacher-forced): equal, or a near-tie whose oracle top-2 gap is within
  max(2 bf16 ulps of max|logit|, the oracle's own max |order-2 - order-0| logit spread
  over the run); the number of such flips is bounded by max_flips(decisions).
"""
import numpy as np

import gpu_util as G

NORM_REL = 1e-3
SPREAD_FACTOR = 2.0
REPORT = []   # (what, engine norm-rel error, bar) of every checked step; conftest writes it out


def max_flips(decisions: int) -> int:
    """Near-tie flips tolerated over `decisions` greedy choices (each one already
    individually within the oracle's own order spread): 1 in 8, at least 2."""
    return max(2, decisions // 8)


def norm_rel(got, want) -> float:
    g, w = G.bf(got).astype(np.float64), G.bf(want).astype(np.float64)
    return float(np.linalg.norm(g - w) / max(np.linalg.norm(w), 1e-30))


class OrderPair:
    """Two oracle models over the same weights: summation order 0 (the restatement) and
    order 2 (every fp32 reduction reordered), stepped in lock-step; tracks the running
    maxima of their norm-relative and absolute logit spreads."""

    def __init__(self, oracle, hw, max_ctx, nthreads=0, with_spread=True, act_fp8=False):
        self.O = oracle
        self.act_fp8 = act_fp8   # the engine's prefill_fp8 numerics (oracle Model prefill_act_fp8)
        self.m0 = oracle.Model(hw, max_ctx, nthreads=nthreads, prefill_act_fp8=act_fp8)
        self.m2 = oracle.Model(hw, max_ctx, nthreads=nthreads, prefill_act_fp8=act_fp8) if with_spread else None
        self.rel_spread = 0.0
        self.abs_spread = 0.0

    def forward(self, ids, start=None):
        lg0 = self.m0.forward(ids, start)
        lg2 = None
        if self.m2 is not None:
            # fp8 activations: order 8 (order 2 + the fp8 MFMA's accumulation model; the
            # quantisation of every projection input turns the hardware's accumulation error
            # into rounding flips an exact-sum order never shows)
            self.O.set_sum_order(8 if self.act_fp8 else 2)
            try:
                lg2 = self.m2.forward(ids, start)
            finally:
                self.O.set_sum_order(0)
            self.rel_spread = max(self.rel_spread, norm_rel(lg2, lg0))
            self.abs_spread = max(self.abs_spread,
                                  float(np.abs(G.bf(lg2).astype(np.float64) - G.bf(lg0)).max()))
        return lg0, lg2

    def calibrate(self, vocab, n_prompt=24, n_steps=6, seed=12345):
        """Spread of a fixed teacher-forced calibration run on fresh oracle models (same
        weights); folds into the running maxima."""
        cal = OrderPair(self.O, self.m0.hw, n_prompt + n_steps + 2, self.m0.nthreads, act_fp8=self.act_fp8)
        prompt = [int(t) for t in np.random.default_rng(seed).integers(0, vocab, n_prompt)]
        oracle_trace(self.O, cal, prompt, n_steps)
        self.rel_spread = max(self.rel_spread, cal.rel_spread)
        self.abs_spread = max(self.abs_spread, cal.abs_spread)
        return self

    def bars(self, lg0):
        """(norm-relative bar, near-tie gap bar) for a step whose order-0 logits are lg0."""
        ulps = 2 * 2.0 ** -7 * float(np.abs(G.bf(lg0)).max())
        return max(NORM_REL, SPREAD_FACTOR * self.rel_spread), max(ulps, self.abs_spread)


def check_step(got_lg, lg0, pair, got_id, want_id, what, bar=None):
    """Asserts the logit bar (`pair`'s running spreads, or an explicit (rel, gap) `bar`);
    returns 1 for a tolerated near-tie flip, else 0."""
    rel_bar, gap_bar = bar if bar is not None else pair.bars(lg0)
    rel = norm_rel(got_lg, lg0)
    REPORT.append((what, rel, rel_bar))
    assert rel <= rel_bar, f"{what}: norm-relative logit error {rel:.3e} > bar {rel_bar:.3e}"
    if got_id != want_id:
        gap = abs(float(G.bf(lg0[want_id])) - float(G.bf(lg0[got_id])))
        assert gap <= gap_bar, f"{what}: engine {got_id} vs oracle {want_id}, oracle gap {gap} > {gap_bar}"
        return 1
    return 0


def oracle_trace(oracle, pair, prompt, n_steps, forced=None):
    """Teacher-forced oracle run: order-0 (and order-2) logits of the prompt and of
    n_steps - 1 decode steps fed the order-0 arg-max (or `forced[i]`).  Returns
    (ids, [(lg0, lg2), ...]); pair's spreads are then the whole run's maxima."""
    outs = [pair.forward(prompt, 0)]
    ids = [oracle.argmax(outs[0][0])]
    for i in range(n_steps - 1):
        nxt = ids[-1] if forced is None else forced[i]
        outs.append(pair.forward([nxt]))
        ids.append(oracle.argmax(outs[-1][0]))
    return ids, outs


# ----------------------------------------------------------------------------------------
# Forced-continuation greedy decisions (full-depth parity in bench.py; the 2-layer P = 2048
# twin in tests/test_gpu_headline.py).  The sequence is a prompt followed by a seeded random
# continuation fed one token per decode step (teacher forcing on a fixed sequence, so no
# decision depends on an earlier one and a degenerate repetition cannot form); at each of
# the n decision points (the prefill's and n - 1 decode steps') the engine's greedy id and
# bf16 logits are compared with four oracle evaluations of the same arithmetic: summation
# order 0 (the restatement), 1 (matmul sums reordered), 2 (every fp32 reduction
# reordered, fast-math exponent) and 7 (the reference build's nvcc -use_fast_math
# arithmetic: contracted fma, approximate division, fast exponent).  Weights: SynthParams with a peaked head (PEAKED).
PEAKED = dict(head_boost_every=4096, head_boost_log2=3)


class OrderSet:
    """Oracle models over the same weights in summation orders 0, 1, 2 and 7 (the reference
    build's nvcc -use_fast_math arithmetic, or_set_sum_order), stepped in lock-step."""

    ORDERS = (0, 1, 2, 7)

    def __init__(self, oracle, hw, max_ctx, nthreads=0, act_fp8=False):
        self.O = oracle
        # fp8 activations: order 8 in the place of order 2 (OrderPair)
        self.orders = tuple(8 if (o == 2 and act_fp8) else o for o in self.ORDERS)
        self.models = [oracle.Model(hw, max_ctx, nthreads=nthreads, prefill_act_fp8=act_fp8) for _ in self.ORDERS]

    def forward(self, ids, start=None):
        out = []
        for o, m in zip(self.orders, self.models):
            self.O.set_sum_order(o)
            try:
                out.append(m.forward(ids, start))
            finally:
                self.O.set_sum_order(0)
        return out


def forced_decisions(oracle, hw, batch, prompt, n, seed=77, nthreads=0, progress=False, act_fp8=False):
    """Runs the protocol above on slot 0 of `batch` (an engine over the same weights as
    `hw`).  Returns the report dict; report["ok"] applies the rule:
      * every step's engine logits within max(1e-3, 2 x the run's max order-0 vs order-2
        norm-relative spread) of order 0;
      * no hard mismatch: an engine id that differs from order 0 must be a near-tie whose
        order-0 top-2 gap is within max(2 bf16 ulps of max|logit|, the run's max absolute
        order-1 / order-2 logit spread);
    Order 7 is the reference's recorded nvcc -use_fast_math build (contracted fma, fast
    division and exponent; or_set_sum_order): the engine's distance to it and order 7's own
    spread are reported as information only — the engine is not a fast-math build, so order 7
    does not widen the bar.
      * near-tie flips <= max_flips(n)."""
    V = hw.spec.vocab
    P = len(prompt)
    forced = [int(t) for t in np.random.default_rng(seed).integers(0, V, max(n - 1, 0))]
    ors = OrderSet(oracle, hw, P + n + 2, nthreads, act_fp8=act_fp8)   # act_fp8: the engine's prefill_fp8
    steps = []
    t_e = batch.prefill(0, prompt)
    for i in range(n):
        lg = ors.forward(prompt, 0) if i == 0 else ors.forward([forced[i - 1]])
        ge = batch.logits()[0]
        f = [G.bf(x).astype(np.float64) for x in lg]
        steps.append(dict(ids=[oracle.argmax(x) for x in lg], gpu=int(t_e), rel=norm_rel(ge, lg[0]),
                          rel01=norm_rel(lg[1], lg[0]), rel02=norm_rel(lg[2], lg[0]),
                          rel07=norm_rel(lg[3], lg[0]), rel_gpu7=norm_rel(ge, lg[3]),
                          abs_spread=float(max(np.abs(f[k] - f[0]).max() for k in (1, 2))),
                          abs_spread7=float(np.abs(f[3] - f[0]).max()),
                          lg0=lg[0], ulps=2 * 2.0 ** -7 * float(np.abs(f[0]).max())))
        if progress and (i % 16 == 0 or i + 1 == n):
            print(f"  forced decision {i + 1}/{n}: rel {steps[-1]['rel']:.2e}", flush=True)
        if i + 1 < n:
            batch.set_position(0, P + i, forced[i])
            t_e = batch.decode_step()[0]
    rel02 = max(s["rel02"] for s in steps)
    rel01 = max(s["rel01"] for s in steps)
    rel07 = max(s["rel07"] for s in steps)
    abs_spread = max(s["abs_spread"] for s in steps)
    # the gate: orders 1 and 2 only (the engine is not a fast-math build); order 7's spread is
    # reported beside it, never folded into the bar
    bar = max(NORM_REL, SPREAD_FACTOR * rel02)
    flips = hard = agreed_flips = 0
    flip_gaps = []
    for s in steps:
        o0 = s["ids"][0]
        if s["gpu"] == o0:
            continue
        lg0 = s["lg0"]
        gap = abs(float(G.bf(lg0[o0])) - float(G.bf(lg0[s["gpu"]])))
        flip_gaps.append(round(gap, 5))
        if gap <= max(s["ulps"], abs_spread):
            flips += 1
            if all(i == o0 for i in s["ids"][1:]):
                agreed_flips += 1
        else:
            hard += 1
    rep = {
        "decisions": n, "prompt": P, "forced_seed": seed,
        "oracle_o1_vs_o0_id_disagreements": sum(s["ids"][1] != s["ids"][0] for s in steps),
        "oracle_o2_vs_o0_id_disagreements": sum(s["ids"][2] != s["ids"][0] for s in steps),
        "oracle_o7_vs_o0_id_disagreements": sum(s["ids"][3] != s["ids"][0] for s in steps),
        "gpu_vs_o0_id_disagreements": sum(s["gpu"] != s["ids"][0] for s in steps),
        "gpu_vs_o7_id_disagreements": sum(s["gpu"] != s["ids"][3] for s in steps),
        "gpu_vs_o7_max_norm_rel": round(max(s["rel_gpu7"] for s in steps), 6),
        "gpu_near_tie_flips": flips, "gpu_flips_where_oracle_orders_agree": agreed_flips,
        "hard_mismatches": hard, "max_flips": max_flips(n),
        "max_norm_rel": round(max(s["rel"] for s in steps), 6),
        "oracle_o1_spread": round(rel01, 6), "oracle_o2_spread": round(rel02, 6),
        "oracle_o7_spread": round(rel07, 6), "bar": round(bar, 6),
        "max_abs_spread": round(abs_spread, 5), "gpu_flip_top2_gaps": flip_gaps,
        "oracle_o7_max_abs_spread": round(max(s["abs_spread7"] for s in steps), 5),
        "bar_rule": "max(1e-3, 2 x max order-2 vs order-0 norm-rel spread); near-tie gap <= max(2 bf16 ulps, "
                    "max |order-1 or order-2 - order-0| logit); order 7 reported, not gating",
        "median_top2_gap": round(float(np.median([abs(np.diff(np.sort(G.bf(s["lg0"]).astype(np.float64))[-2:]))[0]
                                                  for s in steps])), 5),
    }
    rep["ok"] = bool(max(s["rel"] for s in steps) <= bar and hard == 0 and flips <= max_flips(n))
    return rep
