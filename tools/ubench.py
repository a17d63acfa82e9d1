#!/usr/bin/env python3
"""Kernel A/B micro-benchmarks on the real Qwen2-7B decode state (one process, interleaved
rounds, cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per measurement.
The knobs exist only in the development build: run with
QIE_LIB=qwen_inference_engine_amd/lib/dev/libqie.so (make -C ... DEV=1)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

NAMES = {0: "gate_up", 1: "down", 2: "qkv", 3: "o", 4: "lm_head", 5: "attn"}


def main():
    spec = S.PRESETS[os.environ.get("UB_MODEL", "Qwen2-7B")]
    P = int(os.environ.get("UB_P", "2048"))
    eng = Q.Engine(spec, max_ctx=P + 528).init_synthetic(W.SynthParams(seed=0))
    b = eng.batch(1, P + 528)
    ids = np.random.default_rng(1).integers(0, spec.vocab, P)
    b.prefill(0, ids)
    b.decode(256, want_ids=False)          # ctx ~2300
    sets = os.environ.get("UB_SET", "attn,gemv").split(",")
    variants = []
    if os.environ.get("UB_VARIANTS"):   # JSON list of [kernel name, which, {env}]
        variants += [tuple(v) for v in json.loads(os.environ["UB_VARIANTS"])]
        sets = []
    if "attn" in sets:
        variants += [("attn", 5, {})]
        for sp in ("8", "16", "24", "48"):
            variants.append(("attn", 5, {"QIE_DEC_SPLITS": sp}))
        variants += [("attn", 5, {"QIE_DEC_DBG": d}) for d in ("1", "8", "16", "64")]
    if "gemv" in sets:
        for which in (0, 1, 2, 3, 4):
            variants.append((NAMES[which], which, {}))
            variants.append((NAMES[which], which, {"QIE_GEMV_BALANCED": "0"}))
            variants.append((NAMES[which], which, {"QIE_GEMV_XFIRST": "0"}))
            for bpc in ("0", "16"):
                variants.append((NAMES[which], which, {"QIE_GEMV_BLOCKS_PER_CU": bpc}))
    res = {}
    for rnd in range(3):
        for name, which, env in variants:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            us, by = b.time_kernel(which, 100)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            key = (name, json.dumps(env, sort_keys=True))
            res.setdefault(key, []).append(us)
    for (name, env), v in res.items():
        print(json.dumps({"kernel": name, "env": json.loads(env), "us_median": round(float(np.median(v)), 3),
                          "us_min": round(float(np.min(v)), 3)}))


if __name__ == "__main__":
    main()
