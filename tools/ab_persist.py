#!/usr/bin/env python3
"""In-process A/B of the decode structure: five launches per layer (mode 0) against the
persistent layer stack (mode 1, k_persist.hip), on one engine with synthetic weights.
Per mode and round: a fresh batch, a prefill, a warm-up, then timed graph decode steps;
modes interleaved over AB_ROUNDS; greedy ids of mode 1 must equal mode 0's bit for bit.
Also the live hipEvent time of the persistent launch alone (qie_batch_time_kernel 6).

Env: AB_MODEL (Qwen2-7B), AB_P (2048), AB_STEPS (128), AB_ROUNDS (3)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402


def main():
    spec = S.PRESETS[os.environ.get("AB_MODEL", "Qwen2-7B")]
    P = int(os.environ.get("AB_P", "2048"))
    steps = int(os.environ.get("AB_STEPS", "128"))
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    warm = 8
    max_ctx = P + steps + warm + 16
    eng = Q.Engine(spec, max_ctx=max_ctx).init_synthetic(W.SynthParams(seed=0))
    prompt = [int(t) for t in np.random.default_rng(1).integers(0, spec.vocab, P)]
    res = {0: [], 1: []}
    ids = {}
    kern = []
    t0 = time.time()
    for rnd in range(rounds):
        for mode in (0, 1):
            b = eng.batch(1, max_ctx)
            b.set_decode_mode(mode)
            b.prefill(0, prompt)
            b.decode(warm)
            eng.sync()
            t = time.perf_counter()
            got = b.decode(steps)[:, 0].tolist()
            dt = time.perf_counter() - t
            res[mode].append(steps / dt)
            ids.setdefault(mode, got)
            if mode == 1 and rnd == 0:
                us, by = b.time_kernel(6, 10)
                kern.append({"persistent_us": round(us, 2), "bytes": by, "tb_s": round(by / us / 1e6, 3)})
            b.close()
            print(f"round {rnd} mode {mode}: {res[mode][-1]:.1f} tok/s ({time.time() - t0:.0f} s)", file=sys.stderr,
                  flush=True)
    out = {"model": spec.name, "prompt": P, "steps": steps,
           "launches_tok_s": [round(x, 1) for x in res[0]], "persistent_tok_s": [round(x, 1) for x in res[1]],
           "median_launches": round(float(np.median(res[0])), 1), "median_persistent": round(float(np.median(res[1])), 1),
           "ids_equal": ids.get(0) == ids.get(1), "persistent_kernel": kern}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
