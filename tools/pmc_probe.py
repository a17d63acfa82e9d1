#!/usr/bin/env python3
"""Fixed launch sequence for rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE): each decode
kernel of the Qwen2-7B step (layer 0 weights, context 2048) launched ITERS times in
isolation through qie_batch_time_kernel, in the order gate_up, down, qkv, o, lm_head,
attention.  tools/pmc_summary.py turns the per-dispatch counters into HBM bytes per
launch (profiles/)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

ITERS = int(os.environ.get("PMC_ITERS", "8"))
ORDER = [(0, "gate_up"), (1, "down"), (2, "qkv"), (3, "o"), (4, "lm_head"), (5, "attn")]


def main():
    spec = S.PRESETS["Qwen2-7B"]
    fp8b8 = os.environ.get("PMC_CONFIG") == "fp8b8"   # BASELINE config 4: fp8 weights, batch 8, prompt 1024
    P, B = (1024, 8) if fp8b8 else (2048, 1)
    eng = Q.Engine(spec, max_ctx=P + 64, weight_fp8=fp8b8).init_synthetic(W.SynthParams(seed=0))
    # PMC_PAGED=N: the paged KV cache of N-token pages (bench.py's config 4 runs 128)
    b = eng.batch(B, P + 64, page_tokens=int(os.environ["PMC_PAGED"]) if os.environ.get("PMC_PAGED") else None)
    prompts = np.random.default_rng(1).integers(0, spec.vocab, (B, P))
    if B > 1:
        b.prefill_batch(0, prompts)
    else:
        b.prefill(0, prompts[0])
    meta = []
    for which, name in ORDER:
        us, by = b.time_kernel(which, ITERS)   # min(L, 4) warm-up + ITERS launches (qie_batch_time_kernel)
        wu = min(spec.n_layers, 4)
        meta.append({"kernel": name, "which": which, "launches": ITERS + wu, "warmup": wu, "algorithmic_bytes": by,
                     "avg_us": us})
    out = os.path.join(ROOT, "gpurun_out", "pmc_probe_meta.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"iters": ITERS, "order": meta}, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
