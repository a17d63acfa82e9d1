#!/usr/bin/env python3
"""Attribution of the full-depth greedy flips.

Replays bench.py's full-depth parity sample (tests/parity.py forced_decisions: Qwen2-7B
synthetic weights, peaked head, 16-token prompt, a seeded forced continuation) and, at every
decode decision, snapshots the residual stream after every attention and every MLP block:

  * engine: the captured graph step is run first (its id is the one the bench judges), then
    the same position is re-run eagerly through qie_batch_debug_step (same kernels, K/V
    rewritten with the same values) which copies x_res after each residual add;
  * oracle: or_forward in summation orders 0..4 (ORDERS below) with or_set_layer_dump.

Per decision and per snapshot slot it records the norm-relative difference to order 0 of
the engine and of orders 1 and 2.  For each flip (engine id != order-0 id) it reports:
  * the first slot where the engine's difference exceeds order 1's (the first op whose
    difference exceeds the order-1 spread, the verdict's question), and the slot-wise
    ratio engine / order-1 along the depth;
  * the head decomposition: the final-norm + lm_head logits of each source's final residual
    row re-evaluated in float64 (tie-free), restricted to the competing ids — whether the
    engine's own hidden state already prefers its id (the flip is upstream of the head) or
    the head's arithmetic / bf16 rounding / arg-max tie-break made it (the reference's
    logit_decode.cu:15-33 arg-max over bf16 logits, first index on ties).

Test infrastructure: runs on the GPU box beside bench.py; writes one JSON report to stdout.
  FLIP_DECISIONS (64), FLIP_PROMPT (16), FLIP_SEED (77)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
import gpu_util as G  # noqa: E402
from parity import PEAKED, norm_rel  # noqa: E402
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402


def f64(a):
    return G.bf(a).astype(np.float64)


# oracle summation orders (oracle/qie_oracle.cpp or_set_sum_order): 0 the restatement, 1 matmul
# sums reordered, 2 every reduction reordered + the online-softmax / fast-exp forms, 3 order 0
# with only the attention softmax in 2's form, 4 / 5 / 6 order 0 with only SiLU's exponent / the
# RMSNorm sum of squares / the attention q.k dots in 2's form
ORDERS = (0, 1, 2, 3, 4, 5, 6)


def slot_name(s):
    if s == 0:
        return "embedding"
    l, k = (s - 1) // 2, (s - 1) % 2
    return f"layer {l} {'attention (qkv, attn, o, +res)' if k == 0 else 'mlp (gate/up, down, +res)'}"


def head_logits(hw, x_last, ids):
    """float64 final RMSNorm (reference numerics: x / rms * w, normalization.cu:5-25, the
    normed row rounded to bf16 as every kernel stores it) + lm_head rows `ids`."""
    spec = hw.spec
    x = f64(x_last)
    w = f64(hw.get("model.norm.weight"))
    rms = np.sqrt(np.dot(x, x) / x.size + spec.rms_eps)
    if spec.numerics == "ref":
        y = (x / rms) * w
    else:
        y = w * f64(G.to_bf16((x / rms).astype(np.float32)))
    y = f64(G.to_bf16(y.astype(np.float32)))
    head = hw.lm_head
    return {int(i): float(np.dot(f64(head[int(i)]), y)) for i in ids}


def main():
    n = int(os.environ.get("FLIP_DECISIONS", "64"))
    P = int(os.environ.get("FLIP_PROMPT", "16"))
    seed = int(os.environ.get("FLIP_SEED", "77"))
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    spec = S.QWEN2_7B
    L = spec.n_layers
    t0 = time.time()
    eng = Q.Engine(spec, max_ctx=P + n + 8).init_synthetic(W.SynthParams(seed=0))
    hw = W.HostWeights.synthetic(spec, W.SynthParams(seed=0))
    eng.boost_head(PEAKED["head_boost_every"], PEAKED["head_boost_log2"])
    hw.boost_head(PEAKED["head_boost_every"], PEAKED["head_boost_log2"])
    b = eng.batch(1, P + n + 8)
    prompt = [int(x) for x in np.random.default_rng(5).integers(0, spec.vocab, P)]
    forced = [int(t) for t in np.random.default_rng(seed).integers(0, spec.vocab, max(n - 1, 0))]
    models = [O.Model(hw, P + n + 8, nthreads=threads) for _ in ORDERS]

    def oracle_step(ids, start):
        out = []
        for o, m in zip(ORDERS, models):
            O.set_sum_order(o)
            try:
                out.append(m.forward_dump(ids, start))
            finally:
                O.set_sum_order(0)
        return out

    steps = []
    t_e = b.prefill(0, prompt)
    for i in range(n):
        if i == 0:
            orc = oracle_step(prompt, 0)
            lg_e, xs_e, eager_same = b.logits()[0], None, None
        else:
            orc = oracle_step([forced[i - 1]], None)
            lg_e = b.logits()[0]
            b.set_position(0, P + i - 1, forced[i - 1])
            ids_dbg, xs = b.debug_step()
            xs_e = xs[:, 0, :]
            eager_same = bool(np.array_equal(b.logits()[0], lg_e)) and ids_dbg[0] == t_e
        lgs = [o[0] for o in orc]
        ids = [O.argmax(x) for x in lgs]
        st = {"i": i, "gpu": int(t_e), "o": ids, "rel_logits": [norm_rel(lg_e, lgs[0]), norm_rel(lgs[1], lgs[0]),
                                                                norm_rel(lgs[2], lgs[0])],
              "eager_equals_graph": eager_same}
        if xs_e is not None:
            x0 = [f64(o[1]) for o in orc]
            xe = f64(xs_e)

            def rel(a, b_):
                return [float(np.linalg.norm(a[s] - b_[s]) / max(np.linalg.norm(b_[s]), 1e-30))
                        for s in range(2 * L + 1)]
            st["slot_rel"] = {"gpu": rel(xe, x0[0]), "o1": rel(x0[1], x0[0]), "o2": rel(x0[2], x0[0]),
                              "o3": rel(x0[3], x0[0]), "o4": rel(x0[4], x0[0]), "o5": rel(x0[5], x0[0]),
                              "o6": rel(x0[6], x0[0]), "gpu_vs_o5": rel(xe, x0[5]),
                              "gpu_vs_o2": rel(xe, x0[2]), "gpu_vs_o3": rel(xe, x0[3])}
        if int(t_e) != ids[0]:
            cand = sorted({int(t_e), ids[0], ids[1], ids[2]})
            f0 = f64(lgs[0])
            st["flip"] = {
                "agreed": ids[1] == ids[0] and ids[2] == ids[0],
                "bf16_logits": {src: {c: float(f64(lg)[c]) for c in cand}
                                for src, lg in (("gpu", lg_e), ("o0", lgs[0]), ("o1", lgs[1]), ("o2", lgs[2]))},
                "o0_top2_gap": float(abs(f0[ids[0]] - f0[int(t_e)])),
            }
            if xs_e is not None:
                src_rows = {"gpu": xs_e[2 * L], "o0": orc[0][1][2 * L], "o1": orc[1][1][2 * L], "o2": orc[2][1][2 * L]}
                st["flip"]["head_f64"] = {s: head_logits(hw, r, cand) for s, r in src_rows.items()}
        steps.append(st)
        if i % 8 == 0 or i + 1 == n:
            print(f"flip_attrib: decision {i + 1}/{n}, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        if i + 1 < n:
            b.set_position(0, P + i, forced[i])
            t_e = b.decode_step()[0]

    # ---- summary
    dec = [s for s in steps if "slot_rel" in s]
    nslot = 2 * L + 1
    med = {k: [float(np.median([s["slot_rel"][k][j] for s in dec])) for j in range(nslot)] for k in dec[0]["slot_rel"]}
    ratio = [med["gpu"][j] / med["o1"][j] if med["o1"][j] > 0 else None for j in range(nslot)]
    flips = []
    for s in steps:
        if "flip" not in s:
            continue
        f = dict(i=s["i"], gpu=s["gpu"], o=s["o"], agreed=s["flip"]["agreed"], o0_top2_gap=s["flip"]["o0_top2_gap"],
                 bf16_logits=s["flip"]["bf16_logits"], rel_logits=s["rel_logits"])
        if "slot_rel" in s:
            g, o1 = s["slot_rel"]["gpu"], s["slot_rel"]["o1"]
            first = next((j for j in range(1, nslot) if g[j] > o1[j]), None)
            f["first_slot_over_o1"] = None if first is None else {"slot": first, "op": slot_name(first),
                                                                  "gpu": g[first], "o1": o1[first]}
            f["final_residual_rel"] = {"gpu": g[-1], "o1": o1[-1], "o2": s["slot_rel"]["o2"][-1]}
            h = s["flip"]["head_f64"]
            a, c = s["o"][0], s["gpu"]
            f["head_f64_margin_gpu_minus_o0id"] = {src: h[src][c] - h[src][a] for src in h}
            f["upstream"] = bool(h["gpu"][c] > h["gpu"][a])
        flips.append(f)
    # first slot where the median engine difference exceeds the median order-1 difference
    first_med = next((j for j in range(1, nslot) if med["gpu"][j] > med["o1"][j]), None)
    rep = {
        "decisions": n, "prompt": P, "forced_seed": seed, "seconds": round(time.time() - t0, 1),
        "eager_equals_graph_all": all(s["eager_equals_graph"] for s in dec),
        "gpu_vs_o0_id_disagreements": sum(s["gpu"] != s["o"][0] for s in steps),
        "o1_vs_o0_id_disagreements": sum(s["o"][1] != s["o"][0] for s in steps),
        "o2_vs_o0_id_disagreements": sum(s["o"][2] != s["o"][0] for s in steps),
        "o3_vs_o0_id_disagreements": sum(s["o"][3] != s["o"][0] for s in steps),
        "o4_vs_o0_id_disagreements": sum(s["o"][4] != s["o"][0] for s in steps),
        "o5_vs_o0_id_disagreements": sum(s["o"][5] != s["o"][0] for s in steps),
        "o6_vs_o0_id_disagreements": sum(s["o"][6] != s["o"][0] for s in steps),
        "max_rel_logits": {"gpu": max(s["rel_logits"][0] for s in steps), "o1": max(s["rel_logits"][1] for s in steps),
                           "o2": max(s["rel_logits"][2] for s in steps)},
        "median_slot_rel": {k: [round(v, 6) for v in vals] for k, vals in med.items()},
        "median_ratio_gpu_over_o1": [None if r is None else round(r, 3) for r in ratio],
        "first_slot_median_gpu_over_o1": None if first_med is None else {"slot": first_med, "op": slot_name(first_med)},
        "flips": flips,
    }
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
