#!/usr/bin/env python3
"""Fixed launch sequence for the MFMA counter passes (tools/pmc_mfma.sh): the Qwen2-7B bf16
prefill at P = 2048 (one warm-up prefill, then PMC_PREFILLS measured ones) through the
engine's own dispatch.  tools/pmc_mfma_summary.py maps every dispatch to its role (QKV / O /
gate-up / down GEMM, flash attention) by its place in the layer and turns the counters into
MFMA busy fractions next to the algorithmic-flop rate (profiles/rNN_pmc_mfma.json)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

N = int(os.environ.get("PMC_PREFILLS", "1"))


def main():
    spec = S.PRESETS["Qwen2-7B"]
    P = int(os.environ.get("PMC_PROMPT", "2048"))
    eng = Q.Engine(spec, max_ctx=P + 64).init_synthetic(W.SynthParams(seed=0))
    b = eng.batch(1, P + 64)
    ids = np.random.default_rng(1).integers(0, spec.vocab, P)
    b.prefill(0, ids)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(N):
        b.prefill(0, ids)
    eng.sync()
    meta = {"model": spec.name, "prompt": P, "prefills": N, "warmup_prefills": 1,
            "wall_ms_per_prefill": (time.perf_counter() - t0) * 1e3 / N}
    out = os.path.join(ROOT, "gpurun_out", "pmc_mfma_meta.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
