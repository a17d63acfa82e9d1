#!/usr/bin/env python3
"""Layer-chain (k_chain.hip) vs its four separate GEMV launches on the Qwen2-7B decode
state, live hipEvent timing (qie_batch_time_kernel 6 vs 3 + 0 + 1 + 2); with
QIE_CHAIN_DBG=1 the chain also prints per-phase wall-clock stamps to stderr."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402


def main():
    spec = S.PRESETS[os.environ.get("UB_MODEL", "Qwen2-7B")]
    P = int(os.environ.get("UB_P", "512"))
    eng = Q.Engine(spec, max_ctx=P + 64).init_synthetic(W.SynthParams(seed=0))
    b = eng.batch(1, P + 64)
    b.prefill(0, np.random.default_rng(1).integers(0, spec.vocab, P))
    b.decode(8, want_ids=False)
    res = {}
    for rnd in range(3):
        for name, which in (("chain", 6), ("o", 3), ("gate_up", 0), ("down", 1), ("qkv", 2)):
            us, by = b.time_kernel(which, 54)
            res.setdefault(name, []).append(us)
    med = {k: round(float(np.median(v)), 2) for k, v in res.items()}
    med["parts_sum"] = round(med["o"] + med["gate_up"] + med["down"] + med["qkv"], 2)
    print(json.dumps(med), flush=True)


if __name__ == "__main__":
    main()
