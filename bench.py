#!/usr/bin/env python3
"""Headline benchmark: Qwen2-7B bf16, batch 1, prompt 2048, gen 512 on MI355X.

BASELINE.json metric: "decode tokens/s + prefill tok/s, Qwen2-7B bf16 batch=1, 1/2/4/8
MI355X".  A step = one decode step (one token per sequence) of the hipGraph-captured
forward; `value` = decode tokens/s summed over all ranks.  Prefill tok/s is reported
beside it.  Weights are random-init at the real Qwen2-7B shapes (synthetic; no
checkpoints exist offline), prompts are random token ids.

N>1 (torch.distributed.run, one process per GPU): each rank runs an independent replica
of the batch-1 workload (weak scaling, no data-path collective) — see DESIGN.md §multi-GPU.

JSON extras: "roofline" for the dominant kernel (gate/up GEMV, timed live with hipEvents
on the engine stream), "step_roofline" for the whole decode step, "cpu_baseline" (the
naive C++ oracle forward over the same synthetic weights on host cores, rank 0 / N=1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=511)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--model", default="Qwen2-7B", choices=sorted(S.PRESETS))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=2048)
    ap.add_argument("--gen", type=int, default=512)
    ap.add_argument("--prefill-iters", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-prompt", type=int, default=16)
    ap.add_argument("--cpu-decode", type=int, default=8)
    ap.add_argument("--fp8", action="store_true",
                    help="linear weights + lm_head as OCP e4m3 with power-of-two row scales")
    ap.add_argument("--page-tokens", type=int, default=0,
                    help="paged KV cache (device block table) with pages of this many tokens; 0 = contiguous")
    ap.add_argument("--tp", action="store_true",
                    help="tensor-parallel over all ranks (RCCL) instead of independent replicas")
    return ap.parse_args()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    group = None
    if world > 1:
        from qwen_inference_engine_amd.dist import FileGroup
        group = FileGroup(rank, world)

    spec = S.PRESETS[a.model]
    B, P = a.batch, a.prompt
    max_ctx = P + max(a.gen, a.steps, a.warmup) + 16
    comm = None
    if a.tp and world > 1:   # one RCCL communicator over all ranks; the id travels by file
        uid = Q.Comm.unique_id().hex() if rank == 0 else None
        uid = group.allgather(uid)[0]
        comm = Q.Comm.rccl(bytes.fromhex(uid), world, rank, local)
    eng = Q.Engine(spec, device=local, max_ctx=max_ctx, use_graph=not a.no_graph, comm=comm, weight_fp8=a.fp8)
    eng.init_synthetic(W.SynthParams(seed=0))
    batch = eng.batch(B, max_ctx, page_tokens=a.page_tokens or None)
    prompts = np.random.default_rng(1 + rank).integers(0, spec.vocab, size=(B, P), dtype=np.int32)

    # ---------------- prefill (first call warms up; best of the timed ones)
    first = [batch.prefill(s, prompts[s]) for s in range(B)]
    pts = []
    for _ in range(max(1, a.prefill_iters)):
        eng.sync()
        t0 = time.perf_counter()
        first = [batch.prefill(s, prompts[s]) for s in range(B)]
        eng.sync()
        pts.append(time.perf_counter() - t0)
    t_prefill = float(np.median(pts))

    # ---------------- decode: warmup, rewind to the prompt end, then K timed steps
    batch.decode(a.warmup, want_ids=False)
    for s in range(B):
        batch.set_position(s, P, first[s])
    eng.sync()
    if group:
        group.barrier()
    t0 = time.perf_counter()
    batch.decode(a.steps, want_ids=False)
    eng.sync()
    if group:
        group.barrier()
    dt = time.perf_counter() - t0
    if group:
        dt = group.max(dt)
        t_prefill = group.max(t_prefill)

    ms_step = dt * 1e3 / max(a.steps, 1)
    groups = 1 if comm else world          # TP: all ranks produce ONE batch's tokens together
    value = groups * B * a.steps / dt
    prefill_tok_s = groups * B * P / t_prefill

    # ---------------- dominant kernel, timed live with hipEvents on the engine stream
    kern = {}
    for which, name in [(0, "gate_up_gemv"), (1, "down_gemv"), (2, "qkv_gemv"), (3, "o_gemv"),
                        (4, "lm_head_gemv"), (5, "attention")]:
        us, by = batch.time_kernel(which, 50)
        kern[name] = {"avg_us": round(us, 3), "bytes": by, "GBps": round(by / us / 1e3, 1)}
    dom = kern["gate_up_gemv"]
    traffic, traffic_src = pmc_traffic("gate_up") if spec.name == "Qwen2-7B" and B == 1 and not a.fp8 else (None, None)
    avg_ctx = P + (a.steps + 1) / 2.0
    step_bytes = spec.decode_weight_bytes(fp8=a.fp8) + B * spec.kv_bytes_per_position() * avg_ctx
    step_gbs = step_bytes / (ms_step * 1e-3) / 1e9 / (world if comm else 1)   # per GPU

    out = {
        "metric": "decode tokens/s + prefill tok/s, Qwen2-7B bf16 batch=1, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if comm else "weak",
        "vs_baseline": None,
        "dtype": "fp8-e4m3 weights, bf16 activations / fp32 accumulate" if a.fp8 else "bf16",
        "data": "synthetic: random-init weights at real shapes, random prompt ids",
        "config": {"workload": f"{spec.name} {'fp8' if a.fp8 else 'bf16'} decode, batch={B}, prompt={P}, gen={a.gen}",
                   "batch_per_gpu": B, "prompt": P, "gen": a.gen,
                   "parallelism": (f"tp{world}" if comm else f"replicas{world}") if world > 1 else "single",
                   "graph": not a.no_graph, "kv": f"paged{a.page_tokens}" if a.page_tokens else "contiguous"},
        "prefill_tok_s": round(prefill_tok_s, 1),
        "prefill_ms": round(t_prefill * 1e3, 3),
        "roofline": {"bound": "hbm", "kernel": "gate_up_gemv (rms + gate/up GEMV + SwiGLU, layer 0)",
                     "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(dom["GBps"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes": dom["bytes"], "traffic_source": traffic_src},
        "step_roofline": {"bytes_per_step": step_bytes, "achieved_GBps_per_gpu": round(step_gbs, 1),
                          "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                          "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / step_bytes * B * world, 1)},
        "kernels": kern,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.fp8 and B == 1:
        out["cpu_baseline"] = cpu_baseline(spec, a, batch, eng)
    if rank == 0:
        print(json.dumps(out), flush=True)


def pmc_traffic(kernel="gate_up"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes over
    tools/pmc_probe.py, same model / layer / shapes; gfx950 FETCH_SIZE correction applied
    by tools/pmc_summary.py).  Counters cannot be read from inside this process."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    doc = json.load(open(files[-1]))
    for k in doc["kernels"]:
        if k["kernel"] == kernel:
            return k["hbm_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_baseline(spec, a, batch, eng):
    """Naive C++ CPU forward (oracle/qie_oracle.cpp, OpenMP) over the same synthetic
    weights: a bounded sample = cpu_prompt-token prefill + cpu_decode greedy decode steps.
    The GPU then replays the same sample teacher-forced (tests/test_gpu_engine.py rule):
    per-step logit error and near-tie arg-max flips are reported — a size-independent
    parity check at the full model size."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    t0 = time.perf_counter()
    hw = W.HostWeights.synthetic(spec, W.SynthParams(seed=0))
    t_gen = time.perf_counter() - t0
    m = O.Model(hw, a.cpu_prompt + a.cpu_decode + 4, nthreads=threads)
    prompt = [int(x) for x in np.random.default_rng(5).integers(0, spec.vocab, a.cpu_prompt)]
    t0 = time.perf_counter()
    lgs = [m.forward(prompt, 0)]
    t_pf = time.perf_counter() - t0
    ids = [O.argmax(lgs[0])]
    t0 = time.perf_counter()
    for _ in range(a.cpu_decode):
        lgs.append(m.forward([ids[-1]]))
        ids.append(O.argmax(lgs[-1]))
    t_dec = time.perf_counter() - t0
    # order-sensitivity of the reference algorithm itself at full depth: the same forward
    # with another (equally valid) matmul summation order, teacher-forced on the same ids
    O.set_sum_order(1)
    m1 = O.Model(hw, a.cpu_prompt + a.cpu_decode + 4, nthreads=threads)
    lgs1 = [m1.forward(prompt, 0)] + [m1.forward([t]) for t in ids[:-1]]
    O.set_sum_order(0)
    del hw, m, m1
    # GPU, teacher-forced on the oracle's ids
    bf = lambda v: (np.asarray(v, np.uint16).astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    t_e = batch.prefill(0, prompt)
    max_err, tol_max, spread_max, flips, hard = 0.0, 0.0, 0.0, 0, 0
    for i, lg in enumerate(lgs):
        ge = batch.logits()[0]
        spread = float(np.abs(bf(lgs1[i]) - bf(lg)).max())
        spread_max = max(spread_max, spread)
        tol = max(4 * 2.0 ** -7 * max(1.0, float(np.abs(bf(lg)).max())), 2.0 * spread)
        max_err = max(max_err, float(np.abs(bf(ge) - bf(lg)).max()))
        tol_max = max(tol_max, tol)
        if t_e != ids[i]:
            if abs(bf(lg[ids[i]]) - bf(lg[t_e])) <= tol:
                flips += 1
            else:
                hard += 1
            batch.set_position(0, len(prompt) + i, ids[i])
        if i + 1 < len(lgs):
            t_e = batch.decode_step()[0]
    return {"value": round(a.cpu_decode / t_dec, 4), "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"{spec.name}: {a.cpu_prompt}-token prefill ({t_pf:.2f} s, "
                      f"{a.cpu_prompt / t_pf:.2f} tok/s) + {a.cpu_decode} greedy decode steps "
                      f"({t_dec:.2f} s); weights generated in {t_gen:.1f} s",
            "prefill_tok_s": round(a.cpu_prompt / t_pf, 3),
            "gpu_parity": {"steps": len(lgs), "max_abs_dlogit": max_err, "tol": tol_max,
                           "oracle_order_spread": spread_max,
                           "tol_rule": "max(4 bf16 ulps of max|logit|, 2 x oracle order spread)",
                           "near_tie_flips": flips, "hard_mismatches": hard,
                           "ok": max_err <= tol_max and hard == 0}}


if __name__ == "__main__":
    main()
