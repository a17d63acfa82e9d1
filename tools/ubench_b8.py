#!/usr/bin/env python3
"""Batch-8 decode kernel timings (qie_batch_time_kernel) under environment variants
(UB8_ENVS: ';'-separated 'K=V,K=V' lists; '-' = none).  UB8_DECODE=N: N decode steps first;
UB8_PAGE=T: paged KV cache of T-token pages.  One process, interleaved rounds."""
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
    spec = S.PRESETS["Qwen2-7B"]
    B, P = int(os.environ.get("UB8_B", "8")), 1024
    eng = Q.Engine(spec, max_ctx=P + 64 + int(os.environ.get("UB8_DECODE", "0")), weight_fp8=os.environ.get("UB8_FP8") == "1").init_synthetic(W.SynthParams(seed=0))
    b = eng.batch(B, P + 64 + int(os.environ.get("UB8_DECODE", "0")), page_tokens=int(os.environ["UB8_PAGE"]) if os.environ.get("UB8_PAGE") else None)
    for sq in range(B):
        b.prefill(sq, np.random.default_rng(sq).integers(0, spec.vocab, P))
    nd = int(os.environ.get("UB8_DECODE", "0"))   # decode steps before timing (graph + RoPE row state)
    if nd:
        b.decode(nd, want_ids=False)
        eng.sync()
    envs = [e for e in os.environ.get("UB8_ENVS", "-").split(";")]
    res = {}
    for rnd in range(3):
        for e in envs:
            kv = {} if e == "-" else dict(x.split("=") for x in e.split(","))
            saved = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            for which in [int(w) for w in os.environ.get("UB8_WHICH", "0,1,2,3").split(",")]:
                us, by = b.time_kernel(which, 50)
                res.setdefault((e, which), []).append((us, by))
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    for (e, which), v in res.items():
        us = float(np.median([x[0] for x in v]))
        print(json.dumps({"env": e, "kernel": NAMES[which], "us": round(us, 2), "GBps": round(v[0][1] / us / 1e3, 1)}))


if __name__ == "__main__":
    main()
