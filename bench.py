#!/usr/bin/env python3
"""Headline benchmark: Qwen2-7B bf16, batch 1, prompt 2048, gen 512 on MI355X.

BASELINE.json metric: "decode tokens/s + prefill tok/s, Qwen2-7B bf16 batch=1, 1/2/4/8
MI355X".  A step = one decode step (one token per sequence) of the hipGraph-captured
forward; `value` = decode tokens/s of the whole job.  Prefill tok/s is reported beside it.
Weights are random-init at the real Qwen2-7B shapes (synthetic; no checkpoints exist
offline), prompts are random token ids.

Multi-GPU: `--gpus N` with N > 1 runs N ranks, one process per GPU —
launched by torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK from the environment),
or, without WORLD_SIZE, started here as N child processes (subprocess, before any HIP
call in this process; never exec).  Default `--parallel tp`: ONE batch-1 sequence,
tensor-parallel over the N GPUs with RCCL all-reduces inside the decode hipGraph
(Qwen2-7B at TP 8 uses uneven q-head shards with kv-head replication); "scaling":
"strong".  `--parallel replicas`: N independent batch-1 replicas ("weak").

JSON extras: "roofline" for the dominant kernel (gate/up GEMV, timed live with hipEvents on
the engine stream, launches cycling over layers 1..L-1 as the step does), "step_roofline"
for the whole decode step, "cpu_baseline" (the naive C++ oracle forward over the same
synthetic weights on host cores, rank 0 / N = 1) with the BASELINE config-1 CPU run and a
full-depth GPU-vs-oracle parity sample.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Measured stream bandwidth of the dominant kernel's own bytes at its own grid on this part
# (frac also against a measured stream-copy peak): tools/step_floor.hip, 28
# back-to-back gate/up-sized pure streams (271.6 MB each, grid-stride 4 blocks x 4 waves per
# CU, 16-B nt loads) in one hipGraph: 42.29 us per launch, the fastest grid measured for the
# plain stream (6 blocks per CU: 42.97; profiles/r05_step_floor.txt).  The engine's gate/up
# on its 6-per-CU grid runs ~41.3 us, so frac_vs_stream can exceed 1: the probe is a plain
# load loop, not a bound on what a kernel of those bytes can reach.
STREAM_GATE_UP_GBS = 271.633408e6 / 42.29e-6 / 1e9
STREAM_SRC = "profiles/r05_step_floor.txt (tools/step_floor.hip)"
METRIC = "decode tokens/s + prefill tok/s, Qwen2-7B bf16 batch=1, 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=511)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--model", default="Qwen2-7B")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=2048)
    ap.add_argument("--gen", type=int, default=512)
    ap.add_argument("--prefill-iters", type=int, default=3)
    ap.add_argument("--prefill-single", action="store_true",
                    help="B > 1: prefill the B prompts one qie_prefill call each (default: one batched pass)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-prompt", type=int, default=16)
    ap.add_argument("--cpu-decode", type=int, default=8)
    ap.add_argument("--cpu-full", action="store_true",
                    help="CPU baseline at BASELINE.md §3's sizes instead of the bounded sample: the headline "
                         "model's full prompt (--prompt) prefill + --cpu-decode steps, median of 3 (minutes)")
    ap.add_argument("--parity-decisions", type=int, default=64,
                    help="full-depth greedy decisions of the GPU-vs-oracle parity sample (cpu_baseline leg)")
    ap.add_argument("--fp8", action="store_true",
                    help="linear weights + lm_head as OCP e4m3 with power-of-two row scales")
    ap.add_argument("--page-tokens", type=int, default=0,
                    help="paged KV cache (device block table) with pages of this many tokens; 0 = contiguous")
    ap.add_argument("--parallel", choices=["tp", "replicas"], default="tp",
                    help="N > 1: one tensor-parallel sequence (RCCL) or N independent replicas")
    ap.add_argument("--tp", action="store_true", help="(compat) same as --parallel tp")
    ap.add_argument("--comm", choices=["rccl", "peer"], default="rccl",
                    help="tensor-parallel exchange: RCCL (default) or the peer backend (HIP IPC buffers, "
                         "one kernel per exchange with the residual add fused; DESIGN.md §6). The peer backend "
                         "has run across processes on ONE GPU only; across GPUs (xGMI) it is unverified")
    ap.add_argument("--c5-steps", type=int, default=64,
                    help="N > 1 (tensor-parallel): timed decode steps of the Qwen2-72B config-5 line")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other single-GPU BASELINE configs (2 and 4) in the default line")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher only: print the child ranks' environments as JSON and exit (no GPU)")
    return ap.parse_args(argv)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_envs(n, base=None):
    """Environment of each of the n ranks this process would start."""
    base = dict(os.environ if base is None else base)
    port = str(free_port())
    group_dir = tempfile.mkdtemp(prefix="qie_group_")
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port, QIE_GROUP_DIR=group_dir)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def launch(a, argv):
    """N > 1 without a launcher: start N ranks as child processes of this one (which has
    made no HIP call), relay rank 0's output, exit with the worst child status."""
    envs = child_envs(a.gpus)
    if a.dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "QIE_GROUP_DIR")
        print(json.dumps([{k: e[k] for k in keys} for e in envs]))
        return 0
    procs = []
    for r, e in enumerate(envs):
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e, stdout=out))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.tp:
        a.parallel = "tp"
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(a, argv)
    if a.dry_run:
        print(json.dumps({"world": int(os.environ.get("WORLD_SIZE", "1"))}))
        return 0
    return run(a)


def run(a):
    import qwen_inference_engine_amd as Q
    from qwen_inference_engine_amd import spec as S, weights as W
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("QIE_BENCH_ONE_DEVICE") == "1":   # rehearsal of the N-rank path on a 1-GPU box
        local = 0
    group = None
    if world > 1:
        from qwen_inference_engine_amd.dist import FileGroup
        group = FileGroup(rank, world)

    spec = S.PRESETS[a.model]
    B, P = a.batch, a.prompt
    max_ctx = P + max(a.gen, a.steps, a.warmup) + 16
    comm, tp_note = None, None
    if world > 1 and a.parallel == "tp":
        ok, why = S.tp_shardable(spec, world)
        if not ok:
            tp_note = f"tp{world} not possible for {spec.name} ({why}): replicas"
        else:   # one communicator over all ranks; ids / IPC handles travel through the group
            err = None
            if a.comm == "rccl":
                uid = Q.Comm.unique_id().hex() if rank == 0 else None
                uid = group.allgather(uid)[0]
            try:
                if a.comm == "rccl":
                    comm = Q.Comm.rccl(bytes.fromhex(uid), world, rank, local)
                else:
                    comm = Q.Comm.peer(world, rank, local,
                                       lambda h: [bytes.fromhex(x) for x in group.allgather(h.hex())])
            except Exception as ex:   # reported in the JSON line, never silently
                err = str(ex)
            errs = [e for e in group.allgather(err) if e]
            if errs:                  # every rank agrees: no communicator anywhere -> fail the run
                if comm:              # (never report replicas for a tensor-parallel request)
                    comm.close()
                print(f"bench: tp{world} communicator failed on some rank: {errs[0][:300]}", file=sys.stderr,
                      flush=True)
                group.close()
                return 3
    tp = world if comm else 1
    eng = Q.Engine(spec, device=local, max_ctx=max_ctx, use_graph=not a.no_graph, comm=comm, weight_fp8=a.fp8)
    eng.init_synthetic(W.SynthParams(seed=0))
    batch = eng.batch(B, max_ctx, page_tokens=a.page_tokens or None)
    seed = 1 if comm else 1 + rank        # TP ranks process the same sequence
    prompts = np.random.default_rng(seed).integers(0, spec.vocab, size=(B, P), dtype=np.int32)

    # ---------------- prefill (first call warms up; median of the timed ones).  B > 1: the
    # B equal-length prompts in one qie_prefill_batch pass (one GEMM over B*P rows) unless
    # --prefill-single asks for B separate qie_prefill calls.
    def prefill_all():
        if B > 1 and not a.prefill_single:
            return batch.prefill_batch(0, prompts)
        return [batch.prefill(s, prompts[s]) for s in range(B)]

    first = prefill_all()
    pts = []
    for _ in range(max(1, a.prefill_iters)):
        eng.sync()
        if group:
            group.barrier()
        t0 = time.perf_counter()
        first = prefill_all()
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
    dt = time.perf_counter() - t0
    if group:
        group.barrier()
        dt = group.max(dt)
        t_prefill = group.max(t_prefill)

    ms_step = dt * 1e3 / max(a.steps, 1)
    groups = 1 if comm else world          # TP: all ranks produce ONE batch's tokens together
    value = groups * B * a.steps / dt
    prefill_tok_s = groups * B * P / t_prefill

    # ---------------- per-kernel live timing (hipEvents on the engine stream; weight
    # kernels cycle through layers 1..L-1 so no layer's weights are replayed from cache)
    kern = {}
    for which, name in [(0, "gate_up_gemv"), (1, "down_gemv"), (2, "qkv_gemv"), (3, "o_gemv"),
                        (4, "lm_head_gemv"), (5, "attention")]:
        us, by = batch.time_kernel(which, 54)
        kern[name] = {"avg_us": round(us, 3), "bytes": by, "GBps": round(by / us / 1e3, 1)}
    dom = kern["gate_up_gemv"]
    # PMC summaries exist for the headline (bf16, B = 1) and config 4 (fp8, B = 8) shapes
    pmc_tag = ("" if B == 1 and not a.fp8 else "fp8_b8_" if B == 8 and a.fp8 else None) \
        if spec.name == "Qwen2-7B" and tp == 1 else None
    traffic, traffic_src = pmc_traffic("gate_up", pmc_tag) if pmc_tag is not None else (None, None)
    avg_ctx = P + (a.steps + 1) / 2.0
    step_bytes = spec.decode_weight_bytes(fp8=a.fp8) + B * spec.kv_bytes_per_position() * avg_ctx
    step_gbs = step_bytes / (ms_step * 1e-3) / 1e9 / tp   # per GPU (TP: each streams ~1/tp of the weights)

    par = "single" if world == 1 else (f"tp{world}" if comm else f"replicas{world}")
    out = {
        "metric": METRIC,
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
                   "batch_per_gpu": B if not comm else None, "batch": B, "prompt": P, "gen": a.gen,
                   "ctx_timed": [P + 1, P + a.steps], "parallelism": par,
                   "tp_comm": a.comm if comm else None,
                   "graph": not a.no_graph, "kv": f"paged{a.page_tokens}" if a.page_tokens else "contiguous"},
        "prefill_tok_s": round(prefill_tok_s, 1),
        "prefill_ms": round(t_prefill * 1e3, 3),
        "prefill_mode": "batched" if B > 1 and not a.prefill_single else "per-sequence",
        # whole-job prefill TFLOP/s (all groups' prompts; TP ranks compute one prompt together)
        "prefill_tflops_job": round(groups * spec.prefill_flops(P, B) / t_prefill / 1e12, 1),
        "roofline": {"bound": "hbm", "kernel": "gate_up_gemv (rms + gate/up GEMV + SwiGLU, layers 1..L-1)",
                     "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(dom["GBps"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "stream_peak": round(STREAM_GATE_UP_GBS, 1),
                     "frac_vs_stream": round(dom["GBps"] / STREAM_GATE_UP_GBS, 4), "stream_source": STREAM_SRC,
                     "algorithmic_bytes": dom["bytes"], "traffic_source": traffic_src},
        "step_roofline": {"bytes_per_step": step_bytes, "achieved_GBps_per_gpu": round(step_gbs, 1),
                          "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                          "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 * tp / step_bytes * B * (world // tp), 1)},
        "kernels": kern,
        "cpu_baseline": None,
    }
    if tp_note:
        out["note"] = tp_note
    if comm is not None and a.comm == "peer":   # a timed-out exchange must not yield a number
        errs = group.allgather(comm.peer_error())
        out["config"]["peer_error_words"] = errs
        if any(errs):
            print(f"bench: peer exchange error words {errs}: the run is invalid", file=sys.stderr, flush=True)
            group.close()
            return 4
    headline = (spec.name == "Qwen2-7B" and B == 1 and P == 2048 and not a.fp8 and not a.page_tokens
                and world == 1 and not a.no_graph)
    if rank == 0 and headline and not a.no_configs:
        out["configs"] = other_configs(Q, S, W)
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.fp8 and B == 1:
        out["cpu_baseline"] = cpu_baseline(spec, a, batch, eng)
    if comm is not None and not a.no_configs:   # BASELINE configs[4]: the 72B curve, every rank
        batch.close()
        eng.close()
        out["configs"] = {"config5": config5(Q, S, W, a, comm, group, rank, local)}
    if group:
        group.barrier()
        group.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0


# BASELINE.json configs[1] and configs[3]: the other single-GPU configurations, timed by the
# driver's own default bench run (one engine each, after the headline)
OTHER_CONFIGS = [
    {"key": "config2", "model": "Qwen2-0.5B", "batch": 1, "prompt": 128, "gen": 128, "fp8": False,
     "workload": "Qwen2-0.5B bf16, batch=1, prompt=128, gen=128 (BASELINE configs[1])"},
    # config 4 on the paged KV cache (128-token pages; the reference's own cache is paged,
    # iengine.cu:73-109): measured in one process against the contiguous cache, 3,533 vs 3,484
    # tok/s (decode attention 14.3 vs 14.9 µs live; tools/ab_decode.py "_PAGE")
    {"key": "config4", "model": "Qwen2-7B", "batch": 8, "prompt": 1024, "gen": 256, "fp8": True, "fp8_mfma": True,
     "page_tokens": 128,
     "workload": "Qwen2-7B fp8 weights, batch=8, prompt=1024, gen=256, paged KV (128-token pages) (BASELINE configs[3])"},
]


def other_configs(Q, S, W):
    res = {}
    for c in OTHER_CONFIGS:
        t_cfg = time.perf_counter()
        try:
            res[c["key"]] = run_config(Q, S, W, c)
        except Exception as ex:   # reported in the line, never silently dropped
            res[c["key"]] = {"workload": c["workload"], "error": str(ex)[:300]}
        res[c["key"]]["wall_s"] = round(time.perf_counter() - t_cfg, 1)
    return res


def run_config(Q, S, W, c):
    spec = S.PRESETS[c["model"]]
    B, P, G = c["batch"], c["prompt"], c["gen"]
    steps = G - 1                         # the tokens after the prefill's first
    max_ctx = P + G + 16
    eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=c["fp8"]).init_synthetic(W.SynthParams(seed=0))
    b = None
    try:
        b = eng.batch(B, max_ctx, page_tokens=c.get("page_tokens"))
        prompts = np.random.default_rng(1).integers(0, spec.vocab, size=(B, P), dtype=np.int32)

        def prefill():
            return b.prefill_batch(0, prompts) if B > 1 else [b.prefill(0, prompts[0])]
        first = prefill()
        pts = []
        for _ in range(2):
            eng.sync()
            t0 = time.perf_counter()
            first = prefill()
            eng.sync()
            pts.append(time.perf_counter() - t0)
        t_pf = float(np.median(pts))
        b.decode(8, want_ids=False)
        for s_ in range(B):
            b.set_position(s_, P, first[s_])
        eng.sync()
        t0 = time.perf_counter()
        b.decode(steps, want_ids=False)
        eng.sync()
        dt = time.perf_counter() - t0
        ms = dt * 1e3 / steps
        us_dom, by_dom = b.time_kernel(0, 54)
        mx = None
        if c.get("fp8_mfma"):   # the same prefill with fp8 activations on the block-scaled fp8 MFMA
            lg_ref = None
            b.prefill_batch(0, prompts) if B > 1 else b.prefill(0, prompts[0])
            lg_ref = b.logits()
            mx = fp8_mfma_prefill(Q, spec, W, B, P, max_ctx, prompts, lg_ref, t_pf)
        step_bytes = spec.decode_weight_bytes(fp8=c["fp8"]) + B * spec.kv_bytes_per_position() * (P + (steps + 1) / 2.0)
        gbs = step_bytes / (ms * 1e-3) / 1e9
        return {"workload": c["workload"], "value": round(B * steps / dt, 2), "unit": "tokens/s",
                "kv": f"paged{c['page_tokens']}" if c.get("page_tokens") else "contiguous",
                "ms_per_step": round(ms, 4), "steps": steps, "prefill_tok_s": round(B * P / t_pf, 1),
                "prefill_ms": round(t_pf * 1e3, 3),
                "step_roofline": {"bytes_per_step": step_bytes, "achieved_GBps": round(gbs, 1),
                                  "frac": round(gbs / HBM_PEAK_GBS, 4),
                                  "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / step_bytes * B, 1)},
                "dominant_kernel": {"kernel": "gate_up (rms + gate/up + SwiGLU)", "live_us": round(us_dom, 3),
                                    "algorithmic_bytes": by_dom,
                                    "live_frac": round(by_dom / us_dom / 1e3 / HBM_PEAK_GBS, 4),
                                    "timing": "hipEvents on the engine stream around 54 launches cycling over "
                                              "layers 1..L-1 (in-graph durations: profiles/r05_*rocprof*)"},
                **({"prefill_fp8_mfma": mx} if mx else {})}
    finally:
        if b is not None:   # the batch before its engine
            b.close()
        eng.close()


def config5(Q, S, W, a, comm, group, rank, local):
    """BASELINE configs[4] at TP = world: Qwen2-72B bf16, B = 1, P = 2048, over the headline's
    communicator (every rank runs this; the max over ranks is reported).  Bounded steps
    (--c5-steps), so a SCALE run carries the 72B curve north_star names.  Also times the
    step's exchanges alone: 2 row-parallel all-reduces (+ residual add) of [B][H] per layer and
    the arg-max key reduction, on the engine stream, as the graph runs them."""
    spec = S.QWEN2_72B
    world = comm.world
    ok, why = S.tp_shardable(spec, world)
    res = {"workload": f"Qwen2-72B bf16 TP={world}, batch=1, prompt={a.prompt}, gen={a.gen} (BASELINE configs[4])",
           "tp": world, "tp_comm": a.comm}
    if not ok:
        res["error"] = f"not shardable at tp{world}: {why}"
        return res
    t_cfg = time.perf_counter()
    P, steps, warm = a.prompt, a.c5_steps, 4
    max_ctx = P + steps + warm + 16
    eng = b = None
    lib = Q._lib.load()
    bufs = []
    try:
        eng = Q.Engine(spec, device=local, max_ctx=max_ctx, comm=comm).init_synthetic(W.SynthParams(seed=0))
        b = eng.batch(1, max_ctx)
        prompt = np.random.default_rng(1).integers(0, spec.vocab, size=P, dtype=np.int32)
        first = b.prefill(0, prompt)           # warm
        eng.sync()
        group.barrier()
        t0 = time.perf_counter()
        first = b.prefill(0, prompt)
        eng.sync()
        t_pf = group.max(time.perf_counter() - t0)
        b.decode(warm, want_ids=False)
        b.set_position(0, P, first)
        eng.sync()
        group.barrier()
        t0 = time.perf_counter()
        b.decode(steps, want_ids=False)
        eng.sync()
        dt = group.max(time.perf_counter() - t0)
        ms = dt * 1e3 / steps
        # the step's numbers first: an exchange measurement that fails below costs only its own entry
        step_bytes = spec.decode_weight_bytes() + spec.kv_bytes_per_position() * (P + (steps + 1) / 2.0)
        per_gpu = step_bytes / world / (ms * 1e-3) / 1e9
        res.update({"value": round(steps / dt, 3), "unit": "tokens/s", "ms_per_step": round(ms, 4), "steps": steps,
                    "ctx_timed": [P + 1, P + steps], "prefill_tok_s": round(P / t_pf, 1),
                    "prefill_ms": round(t_pf * 1e3, 3),
                    "prefill_tflops_job": round(spec.prefill_flops(P, 1) / t_pf / 1e12, 1),
                    "step_roofline": {"bytes_per_step": step_bytes, "achieved_GBps_per_gpu": round(per_gpu, 1),
                                      "frac": round(per_gpu / HBM_PEAK_GBS, 4),
                                      "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 * world / step_bytes, 1)}})
        H, L = spec.hidden, spec.n_layers
        import ctypes as C
        part, x, keys = C.c_void_p(), C.c_void_p(), C.c_void_p()
        for p_, n_ in ((part, H * 4), (x, H * 2), (keys, 64)):
            Q._lib.check(lib.qie_malloc(C.byref(p_), n_), "qie_malloc")
            Q._lib.check(lib.qie_memset(p_, 0, n_), "qie_memset")
            bufs.append(p_)
        st = eng.stream
        reps = 8

        def time_exchange(form):
            """µs per row-parallel exchange of H elements: 2L of them captured in one graph
            (qie_comm_time_exchange), max over ranks"""
            us = C.c_float()
            group.barrier()
            Q._lib.check(lib.qie_comm_time_exchange(comm.h, part, x, H, 2 * L, reps, form, st, C.byref(us)),
                         "qie_comm_time_exchange")
            return group.max(float(us.value))

        # the per-step arg-max key exchange (one max-u64 all-reduce), eager, amortised
        Q._lib.check(lib.qie_comm_allreduce_max_u64(comm.h, keys, 1, st), "exchange")
        eng.sync()
        group.barrier()
        t0 = time.perf_counter()
        for _ in range(32):
            Q._lib.check(lib.qie_comm_allreduce_max_u64(comm.h, keys, 1, st), "exchange")
        eng.sync()
        key_ms = group.max(time.perf_counter() - t0) * 1e3 / 32
        if a.comm == "peer":
            ex_us = time_exchange(0)
            how = ("row-parallel exchanges: 2L captured in one hipGraph on the engine stream (qie_comm_time_exchange, "
                   "hipEvents), max over ranks; the key exchange eager")
        else:   # RCCL: eager, as the r05 line measured it (its captured form is not rehearsed on one GPU)
            for _ in range(2 * L):
                Q._lib.check(lib.qie_comm_allreduce_residual_bf16(comm.h, part, x, H, st), "exchange")
            eng.sync()
            group.barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                for _ in range(2 * L):
                    Q._lib.check(lib.qie_comm_allreduce_residual_bf16(comm.h, part, x, H, st), "exchange")
            eng.sync()
            ex_us = group.max(time.perf_counter() - t0) * 1e6 / (reps * 2 * L)
            how = "row-parallel exchanges enqueued eagerly on the engine stream, max over ranks; the key exchange eager"
        ex_ms = (2 * L * ex_us) / 1e3 + key_ms
        exch = {"ms_per_step": round(ex_ms, 4), "frac_of_step": round(ex_ms / ms, 4),
                "per_step": f"{2 * L} all-reduce+residual of {H} fp32 + 1 max-u64 arg-max key",
                "us_per_exchange": round(ex_us, 3), "key_exchange_ms": round(key_ms, 4), "timing": how}
        if a.comm == "peer":
            # verdict r05 item 6: the exchange's cost with and without the producer-side send.
            # "with": tagged words pushed by the O / down GEMV epilogues (the default mode, the
            # step timed above); "without": the flagged form (push, flags, wait, reduce in the
            # exchange kernel), the same engine re-captured in that mode.  With the send inside
            # the projection, the exchange's cost is what the step pays beyond the projections:
            # ms_with - (ms_without - exchanges_without).
            flagged_us = time_exchange(1)
            empty_us = time_exchange(2)
            comm.set_peer_mode(tagged=True, push=False)
            tagged_us = time_exchange(0)
            comm.set_peer_mode(tagged=False, push=False)
            b2 = eng.batch(1, max_ctx)
            try:
                first2 = b2.prefill(0, prompt)
                b2.decode(warm, want_ids=False)
                b2.set_position(0, P, first2)
                eng.sync()
                group.barrier()
                t0 = time.perf_counter()
                b2.decode(steps, want_ids=False)
                eng.sync()
                ms_wo = group.max(time.perf_counter() - t0) * 1e3 / steps
            finally:
                b2.close()
                comm.set_peer_mode(tagged=True, push=True)
            ex_wo = (2 * L * flagged_us) / 1e3 + key_ms
            ex_with_raw = ms - (ms_wo - ex_wo)   # < 0: hidden within the two runs' noise
            ex_with = max(0.0, ex_with_raw)
            exch.update({
                "us_per_exchange": {"tagged_exchange_alone": round(tagged_us, 3),
                                    "flagged_exchange_alone": round(flagged_us, 3),
                                    "empty_flagged_exchange_same_grid": round(empty_us, 3)},
                "with_overlap": {"mode": "tagged, pushed by the producing GEMV's epilogue", "ms_per_step": round(ms, 4),
                                 "exchange_ms_per_step": round(ex_with, 4), "frac_of_step": round(ex_with / ms, 4),
                                 "exchange_ms_per_step_unclamped": round(ex_with_raw, 4)},
                "without_overlap": {"mode": "flagged exchange kernel (r05 form)", "ms_per_step": round(ms_wo, 4),
                                    "exchange_ms_per_step": round(ex_wo, 4), "frac_of_step": round(ex_wo / ms_wo, 4)},
                "rule": "without: 2L x flagged exchange alone + key exchange; with: step_with - (step_without - "
                        "exchanges_without), i.e. what the step pays beyond the projections when the send rides in "
                        "their epilogues"})
            ex_ms = ex_with
            exch["ms_per_step"] = round(ex_with, 4)
            exch["frac_of_step"] = round(ex_with / ms, 4)
        res["exchange"] = exch
    except Exception as ex:   # reported, never silently dropped
        res["error"] = str(ex)[:300]
    finally:
        for p_ in bufs:
            lib.qie_free(p_)
        if b is not None:
            b.close()
        if eng is not None:
            eng.close()
    res["wall_s"] = round(time.perf_counter() - t_cfg, 1)
    return res


def fp8_mfma_prefill(Q, spec, W, B, P, max_ctx, prompts, lg_ref, t_ref):
    """Config 4's prefill with the numerics flag prefill_fp8: every projection on the
    block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4; activations quantised per row
    to e4m3).  A different model from the bf16-activation one: its change to the first
    decision's logits (norm-relative, all B rows) is reported beside the speed; parity against
    the oracle's identical quantisation is tests/test_gpu_fp8_mx.py."""
    eng = b = None
    try:
        eng = Q.Engine(spec, max_ctx=max_ctx, weight_fp8=True, prefill_fp8=True).init_synthetic(W.SynthParams(seed=0))
        b = eng.batch(B, max_ctx)

        def prefill():
            return b.prefill_batch(0, prompts) if B > 1 else [b.prefill(0, prompts[0])]
        prefill()
        lg = b.logits()
        pts = []
        for _ in range(2):
            eng.sync()
            t0 = time.perf_counter()
            prefill()
            eng.sync()
            pts.append(time.perf_counter() - t0)
        t = float(np.median(pts))
        g = (lg.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        r = (lg_ref.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        rel = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30))
        return {"prefill_tok_s": round(B * P / t, 1), "prefill_ms": round(t * 1e3, 3),
                "speedup_vs_bf16_activations": round(t_ref / t, 3),
                "prefill_tflops_job": round(spec.prefill_flops(P, B) / t / 1e12, 1),
                "first_logits_change_norm_rel": round(rel, 5),
                "numerics": "prefill_fp8: per-row e4m3 activations x fp8 weights on v_mfma_scale_f32_16x16x128_f8f6f4 "
                            "(a different model; parity vs the oracle's identical quantisation in tests)"}
    except Exception as ex:
        return {"error": str(ex)[:300]}
    finally:
        if b is not None:
            b.close()
        if eng is not None:
            eng.close()


def pmc_traffic(kernel="gate_up", tag=""):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this
    configuration (profiles/rNN_<tag>pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE and
    WRITE_SIZE passes over tools/pmc_probe.py, same model / layer / shapes — tag "" the
    headline, "fp8_b8_" config 4 (PMC_CONFIG=fp8b8); gfx950 FETCH_SIZE correction applied
    by tools/pmc_summary.py).  Counters cannot be read from inside this process."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{tag}pmc_traffic.json")))
    if not files:
        return None, None
    doc = json.load(open(files[-1]))
    for k in doc["kernels"]:
        if k["kernel"] == kernel:
            return k["hbm_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_threads():
    """Host threads for the CPU baseline: the process's CPU share (affinity mask, capped by
    OMP_NUM_THREADS — 16 per GPU on the GPU box, whose nproc counts the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def cpu_baseline(spec, a, batch, eng):
    """Naive C++ CPU forward (oracle/qie_oracle.cpp, OpenMP) over the same synthetic
    weights, on a bounded sample: cpu_prompt-token prefill + cpu_decode greedy steps of the
    headline model, plus BASELINE config 1 (Qwen2-0.5B, prompt 16, gen 16) timed in full.
    Then the full-depth greedy parity sample (tests/parity.py forced_decisions): the GPU
    and oracle orders 0 / 1 / 2 over --parity-decisions teacher-forced decisions on a
    peaked-head copy of the same weights — a size-independent parity check at full depth."""
    threads = cpu_threads()
    # a progress line every minute on stderr: a GPU runner takes minutes of silence for a hang
    # (the --cpu-full prefill of 2,048 tokens alone runs ~80 s per repetition)
    import threading
    t_start = time.perf_counter()
    stop = threading.Event()

    def beat():
        while not stop.wait(60.0):
            print(f"cpu_baseline: {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    try:
        return _cpu_baseline(spec, a, batch, eng, threads)
    finally:
        stop.set()


def _cpu_baseline(spec, a, batch, eng, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from parity import PEAKED, forced_decisions
    from qwen_inference_engine_amd import spec as S, weights as W
    # ---- BASELINE config 1: Qwen2-0.5B, P = 16, G = 16, greedy, timed in full
    s05 = S.QWEN2_0_5B
    hw05 = W.HostWeights.synthetic(s05, W.SynthParams(seed=0))
    m05 = O.Model(hw05, 40, nthreads=threads)
    p05 = [int(x) for x in np.random.default_rng(1).integers(0, s05.vocab, 16)]
    t0 = time.perf_counter()
    ids05 = m05.generate_greedy(p05, 16)[0]
    t_c1 = time.perf_counter() - t0
    del hw05, m05
    # ---- headline model sample
    t0 = time.perf_counter()
    hw = W.HostWeights.synthetic(spec, W.SynthParams(seed=0))
    t_gen = time.perf_counter() - t0
    n_pf = a.prompt if a.cpu_full else a.cpu_prompt
    full_prompt = [int(x) for x in np.random.default_rng(5).integers(0, spec.vocab, n_pf)]
    prompt = full_prompt[:a.cpu_prompt]
    runs = []
    for _ in range(3 if a.cpu_full else 1):   # median of 3 at full size
        m0 = O.Model(hw, n_pf + a.cpu_decode + 4, nthreads=threads)
        t0 = time.perf_counter()
        lg0 = m0.forward(full_prompt, 0)
        t_pf = time.perf_counter() - t0
        ids = [O.argmax(lg0)]
        t0 = time.perf_counter()
        for _ in range(a.cpu_decode):
            ids.append(O.argmax(m0.forward([ids[-1]])))
        runs.append((t_pf, time.perf_counter() - t0))
        del m0
    t_pf = float(np.median([r[0] for r in runs]))
    t_dec = float(np.median([r[1] for r in runs]))
    # ---- full-depth greedy parity (tests/parity.py forced_decisions): the engine's
    # lm_head and the host copy get the same exact peaked-head boost (parity.PEAKED), then
    # a 16-token prompt + a seeded random continuation, a.parity_decisions decisions,
    # each against oracle summation orders 0 / 1 / 2
    eng.boost_head(PEAKED["head_boost_every"], PEAKED["head_boost_log2"])
    hw.boost_head(PEAKED["head_boost_every"], PEAKED["head_boost_log2"])
    t0 = time.perf_counter()
    par = forced_decisions(O, hw, batch, prompt, a.parity_decisions, nthreads=threads)
    par["seconds"] = round(time.perf_counter() - t0, 1)
    par["gpu_over_o1_spread"] = round(par["max_norm_rel"] / max(par["oracle_o1_spread"], 1e-30), 3)
    par["gpu_over_o2_spread"] = round(par["max_norm_rel"] / max(par["oracle_o2_spread"], 1e-30), 3)
    # not computed by this run: a pointer to the one attribution study that was (its build and config)
    par["attribution_ref"] = {"file": "profiles/r04_flip_attrib.json", "tool": "tools/flip_attrib.py",
                              "measured_on": "round-4 build, Qwen2-7B full depth, this sample's prompt/seed/64 decisions",
                              "note": "not re-run by this bench; see DESIGN.md section 5"}
    par["weights"] = (f"the timed model's weights with lm_head rows r % {PEAKED['head_boost_every']} == 0 "
                      f"x 2^{PEAKED['head_boost_log2']} (exact), applied after the timed regions")
    par["rule"] = ("per step norm-relative logit error <= bar = max(1e-3, 2 x the run's max oracle order-0 vs "
                   "order-2 spread); engine ids that differ from order 0 only at near-ties (order-0 top-2 gap "
                   "within max(2 bf16 ulps, the run's max order-1/order-2 absolute logit spread)), at most "
                   "max_flips(decisions); order 7 (nvcc -use_fast_math model) reported, not gating; "
                   "tests/parity.py forced_decisions")
    del hw
    return {"value": round(a.cpu_decode / t_dec, 4), "unit": "tokens/s", "cores": threads, "kind": "port",
            "host_nproc": os.cpu_count(),
            "sample": f"{spec.name}: {n_pf}-token prefill ({t_pf:.2f} s, "
                      f"{n_pf / t_pf:.2f} tok/s) + {a.cpu_decode} greedy decode steps at ctx {n_pf + 1}.. "
                      f"({t_dec:.2f} s){', median of 3' if a.cpu_full else ''}; weights generated in {t_gen:.1f} s",
            "prefill_tok_s": round(n_pf / t_pf, 3),
            "config1": {"workload": "Qwen2-0.5B, prompt=16, gen=16, greedy (BASELINE config 1), timed in full",
                        "seconds": round(t_c1, 3), "tokens_s": round(16 / t_c1, 2), "ids_head": ids05[:4],
                        "cores": threads},
            "gpu_parity": par}


if __name__ == "__main__":
    sys.exit(main())
