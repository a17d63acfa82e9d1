#!/usr/bin/env python3
"""In-process A/B of the hipGraph decode step (and optionally prefill) over development-build
knobs.  One engine (synthetic weights); per variant a fresh batch — so the decode graph is
captured under that variant's environment — a prefill, a warm-up, then timed decode steps.
Variants run interleaved over AB_ROUNDS rounds; the median per variant is printed as JSON,
with the greedy ids of the timed steps compared against the first variant's (a knob that
only reorders work must reproduce them bit for bit; one that changes numerics may not).

  QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so AB_VARIANTS='[{}, {"QIE_X": "1"}]' \\
      python tools/ab_decode.py

Env: AB_MODEL (Qwen2-7B), AB_P (2048), AB_STEPS (256), AB_ROUNDS (3), AB_BATCH (1),
AB_FP8 (0), AB_KERNELS (1: also the live per-kernel timings), AB_PREFILL (0: also time one
prefill per variant; a variant key "_PAGE": N runs that variant on a paged KV cache of
N-token pages), AB_ENGINE (0; 1: a fresh engine per variant and round, for knobs read
when the weights are loaded, e.g. QIE_FP8_T16)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

KNAMES = {0: "gate_up", 1: "down", 2: "qkv", 3: "o", 4: "lm_head", 5: "attn"}


def main():
    spec = S.PRESETS[os.environ.get("AB_MODEL", "Qwen2-7B")]
    P = int(os.environ.get("AB_P", "2048"))
    steps = int(os.environ.get("AB_STEPS", "256"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    B = int(os.environ.get("AB_BATCH", "1"))
    fp8 = os.environ.get("AB_FP8", "0") == "1"
    kern = os.environ.get("AB_KERNELS", "1") == "1"
    do_pf = os.environ.get("AB_PREFILL", "0") == "1"
    variants = json.loads(os.environ.get("AB_VARIANTS", "[{}]"))
    max_ctx = P + steps + 64
    per_engine = os.environ.get("AB_ENGINE", "0") == "1"
    eng = None if per_engine else Q.Engine(spec, max_ctx=max_ctx, weight_fp8=fp8).init_synthetic(W.SynthParams(seed=0))
    prompts = np.random.default_rng(1).integers(0, spec.vocab, size=(B, P), dtype=np.int32)
    res = {i: {"tok_s": [], "prefill_ms": [], "kern": {}} for i in range(len(variants))}
    ids_ref = None
    t_start = time.time()
    for rnd in range(rounds):
        for i, env in enumerate(variants):
            # "_PAGE": page_tokens of the variant's batch (paged KV cache), not an env knob
            page = int(env["_PAGE"]) if "_PAGE" in env else None
            knobs = {k: v for k, v in env.items() if k != "_PAGE"}
            saved = {k: os.environ.get(k) for k in knobs}
            os.environ.update({k: str(v) for k, v in knobs.items()})
            try:
                if per_engine:
                    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=fp8).init_synthetic(W.SynthParams(seed=0))
                b = eng.batch(B, max_ctx, page_tokens=page)
                first = b.prefill_batch(0, prompts) if B > 1 else [b.prefill(0, prompts[0])]
                if do_pf:
                    eng.sync()
                    t0 = time.perf_counter()
                    first = b.prefill_batch(0, prompts) if B > 1 else [b.prefill(0, prompts[0])]
                    eng.sync()
                    res[i]["prefill_ms"].append((time.perf_counter() - t0) * 1e3)
                b.decode(8, want_ids=False)          # graph capture + warm-up
                for s in range(B):
                    b.set_position(s, P, first[s])
                eng.sync()
                t0 = time.perf_counter()
                ids = b.decode(steps)
                eng.sync()
                dt = time.perf_counter() - t0
                res[i]["tok_s"].append(B * steps / dt)
                if rnd == 0:
                    if ids_ref is None:
                        ids_ref = ids
                    res[i]["ids_equal"] = bool(np.array_equal(ids, ids_ref))
                    res[i]["ids_diff_steps"] = int(np.sum(np.any(ids != ids_ref, axis=1)))
                if kern:
                    for w, name in KNAMES.items():
                        us, _ = b.time_kernel(w, 54)
                        res[i]["kern"].setdefault(name, []).append(us)
                b.close()
                if per_engine:
                    eng.close()
                    eng = None
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        print(f"ab_decode: round {rnd + 1}/{rounds} done, {time.time() - t_start:.0f} s", file=sys.stderr, flush=True)
    for i, env in enumerate(variants):
        r = res[i]
        out = {"env": env, "tok_s_median": round(float(np.median(r["tok_s"])), 2),
               "tok_s": [round(x, 2) for x in r["tok_s"]], "ids_equal": r.get("ids_equal"),
               "ids_diff_steps": r.get("ids_diff_steps")}
        if r["prefill_ms"]:
            out["prefill_ms_median"] = round(float(np.median(r["prefill_ms"])), 3)
        if r["kern"]:
            out["kern_us"] = {k: round(float(np.median(v)), 3) for k, v in r["kern"].items()}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
