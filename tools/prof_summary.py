#!/usr/bin/env python3
"""Condense a rocprofv3 --kernel-trace --stats run (gpu_check.sh PROFILE=1: bench.py under
rocprofv3) into profiles/<tag>_rocprof_summary.md + the raw stats CSV.  Kernel templates are
kept apart (the stats CSV folds every gemv_kernel<...> instantiation into one row)."""
import collections
import csv
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# Qwen2-7B call sites: kernel template (qie:: and "void " stripped) + workgroups x threads
ROLE = {
    "gemv_kernel<1, 2, 2, 7, 2, 0, 256> [g 948 x 256]": "decode gate/up GEMV (+RMSNorm, SwiGLU)  [dominant]",
    "gemv_kernel<1, 2, 1, 8, 1, 0, 576> [g 256 x 448]": "decode down GEMV (+residual, x from L2), one block per CU",
    "gemv_kernel<1, 2, 0, 7, 2, 0, 576> [g 256 x 576]": "decode QKV GEMV (+RMSNorm, bias), one block per CU",
    "gemv_kernel<1, 2, 1, 7, 1, 0, 576> [g 256 x 448]": "decode O-proj GEMV (+residual, x from L2), one block per CU",
    "gemv_kernel<1, 2, 0, 8, 2, 0, 256> [g 761 x 256]": "lm_head GEMV (+final RMSNorm, arg-max keys)",
    "gemv_kernel<1, 2, 0, 8, 3, 0, 256> [g 761 x 256]": "lm_head GEMV (+final RMSNorm per wave, arg-max keys)",
    "gemv_kernel<1, 1, 1, 7, 1, 0, 1024> [g 256 x 896]": "decode O-proj GEMV (+residual), one row per wave, one block per CU",
    "gemv_kernel<1, 1, 0, 7, 1, 0, 1024> [g 256 x 896]": "bench live timing of O-proj (store epilogue)",
    "attn_decode_mfma2_kernel<128, false>": "decode attention (fused qk-norm/RoPE/KV append, split-K, in-launch combine)",
    "attn_decode_mfma2_kernel<128, false, 4, false>": "decode attention (fused RoPE/KV append, split-K, in-launch combine)",
    "rmsnorm_kernel": "prefill RMSNorm",
    "qkv_post_kernel<false>": "prefill RoPE + KV-cache write",
    "attn_prefill_mfma2_kernel<128, false, 8>": "prefill flash attention (MFMA, 32 rows/wave, 8-wave workgroups)",
    "gemm_big_kernel<2, 256>": "prefill gate/up GEMM (256x256 LDS-DMA, SwiGLU)",
    "gemm_big_kernel<1, 128>": "prefill O / down GEMM (256x128 LDS-DMA, +residual)",
    "gemm_big_kernel<0, 256>": "prefill QKV GEMM (256x256 LDS-DMA, one round, +bias)",
    "finalize_kernel": "token -> history, position++, next embedding row, RoPE row of the new position",
    # round 4
    "gemv_kernel<1, 2, 2, 7, 4, 0, 256> [g 512 x 256]": "decode gate/up GEMV (+RMSNorm in registers, SwiGLU), full-residency grid  [dominant]",
    "gemm8_kernel<2>": "prefill gate/up GEMM (phase-interleaved 256x256, SwiGLU)",
    "gemm8_kernel<1>": "prefill down GEMM (phase-interleaved 256x256, split-K 2, +residual)",
    "gemm8_kernel<0>": "prefill QKV GEMM (phase-interleaved 256x256, +bias)",
    "attn_decode_mfma2_kernel<128, false, 4, false, 128>": "decode attention (fused RoPE/KV append, speculative K/V step, split-K, in-launch combine)",
    "dec8r_kernel<2, 8, 7, 8>": "fp8 decode gate/up, A in LDS + 4-step ring  [dominant]",
    "dec8r_kernel<0, 8, 7, 8>": "fp8 decode QKV, A in LDS + 4-step ring",
    "dec8r_kernel<1, 8, 7, 8>": "fp8 decode O-proj, A in LDS + 4-step ring",
    "gemv_kernel<1, 2, 0, 8, 1, 0, 576> [g 256 x 448]": "bench live timing of down (store epilogue)",
    "gemv_kernel<1, 2, 0, 7, 1, 0, 576> [g 256 x 448]": "bench live timing of O-proj (store epilogue)",
    "synth_kernel": "synthetic weight fill (setup)",
    # config 4 (fp8 weights, batch 8): k_decode_fp8.hip and the skinny MFMA kernel
    "dec8_kernel<2, 8, 7>": "fp8 decode gate/up (+fused RMSNorm, SwiGLU)  [dominant]",
    "dec8_kernel<0, 8, 7>": "fp8 decode QKV (+fused RMSNorm, bias); bench live timing of O (store)",
    "dec8_kernel<1, 8, 7>": "fp8 decode O-proj (+residual)",
    "skinny_mfma_kernel<1, 1, 0, 4, 0>": "fp8 decode down (+residual, x from L2)",
    "skinny_mfma_kernel<0, 1, 0, 4, 0>": "bench live timing of down (store epilogue)",
    "skinny_mfma_kernel<0, 1, 1, 4, 7>": "fp8 lm_head (rows staged, arg-max keys)",
    "rmsnorm_reg_kernel<2>": "final RMSNorm (batch head) / prefill RMSNorm",
    "gemm_kernel<1, 0>": "prefill O / down GEMM (128x128 tiles, +residual)",
    "quantize_fp8_kernel": "fp8 weight quantisation (setup)",
    # round 4, config 4 on 16-row tiled fp8 weights (dec8_kernel<EPI, KU, KS, split-K, tiled>)
    "dec8_kernel<2, 8, 7, false, true>": "fp8 decode gate/up (+fused RMSNorm, SwiGLU), tiled weights  [dominant]",
    "dec8_kernel<0, 8, 7, false, true>": "fp8 decode QKV (+fused RMSNorm, bias), tiled; bench live timing of O (store)",
    "dec8_kernel<1, 8, 7, false, true>": "fp8 decode O-proj (+residual), tiled weights",
    "dec8_kernel<1, 4, 8, true, true>": "fp8 decode down (+residual), split-K 10 x (8 waves x 4 units), tiled",
    "dec8_kernel<0, 4, 8, true, true>": "bench live timing of down (store epilogue)",
    "fp8_tile16_kernel": "fp8 16-row tiling of the decode projections (setup)",
    "gemm_big_kernel<1, 128> [g 224 x 512]": "prefill O GEMM (256x128 LDS-DMA, one round of 224 tiles, +residual)",
    "dequantize_fp8_kernel": "fp8 -> bf16 prefill copy (setup)",
    # round 5: grids per measured shape (gate/up 6 blocks per CU, lm_head 2)
    "gemv_kernel<1, 2, 2, 7, 4, 0, 256> [g 1536 x 256]": "decode gate/up GEMV (+RMSNorm in registers, SwiGLU), 6 blocks per CU  [dominant]",
    "gemv_kernel<1, 2, 0, 8, 3, 0, 256> [g 512 x 256]": "lm_head GEMV (+final RMSNorm per wave, arg-max keys), 2 blocks per CU",
    "gemv_kernel<1, 2, 0, 7, 2, 0, 256> [g 512 x 256]": "decode QKV GEMV (+RMSNorm, bias), 2 four-wave blocks per CU",
    # round 5: LDS-form fused norm (dec8_kernel<..., LF>), paged KV in the config-4 line
    "dec8_kernel<2, 8, 7, false, true, true>": "fp8 decode gate/up (+fused RMSNorm, LDS form, SwiGLU), tiled weights  [dominant]",
    "dec8_kernel<0, 8, 7, false, true, true>": "fp8 decode QKV (+fused RMSNorm, LDS form, bias), tiled weights",
    "dec8_kernel<0, 8, 7, false, true, false>": "bench live timing of O (store epilogue)",
    "dec8_kernel<1, 8, 7, false, true, false>": "fp8 decode O-proj (+residual), tiled weights",
    "dec8_kernel<1, 4, 8, true, true, false>": "fp8 decode down (+residual), split-K 10 x (8 waves x 4 units), tiled",
    "dec8_kernel<0, 4, 8, true, true, false>": "bench live timing of down (store epilogue)",
    "attn_decode_mfma2_kernel<128, true, 4, false, 128>": "decode attention, paged KV (fused RoPE/KV append, split-K, in-launch combine)",
    "attn_prefill_mfma2_kernel<128, true, 8>": "prefill flash attention, paged KV (MFMA, 32 rows/wave, 8-wave workgroups)",
}


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("qie::", "")
    return n


def in_graph_decode(trace):
    """Per-layer in-graph decode durations: the launches between two finalize_kernel
    dispatches are one hipGraph decode step (5 per layer + lm_head + finalize); layer 0 is
    left out (its weights follow the previous step's lm_head) and so are the bench's
    live-timing loops (after the last finalize).  Gap = this kernel's start minus the
    previous kernel's end (the dependent-launch boundary)."""
    t = sorted(trace, key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(t) if short(r["Kernel_Name"]) == "finalize_kernel"]
    roles = ["QKV GEMV", "attention", "O GEMV", "gate/up GEMV", "down GEMV"]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    steps = []
    for a, b in zip(fin, fin[1:]):
        seg = t[a + 1:b + 1]
        # layers: groups of 5 launches whose second is the decode attention; what follows
        # (optional final norm, lm_head, finalize) is the head
        L = 0
        while 5 * L + 1 < len(seg) and short(seg[5 * L + 1]["Kernel_Name"]).startswith("attn_decode"):
            L += 1
        if L < 2:
            continue
        steps.append((int(seg[-1]["End_Timestamp"]) - int(t[a]["End_Timestamp"])) / 1e3)
        for i, r in enumerate(seg):
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            pe = int(seg[i - 1]["End_Timestamp"]) if i else int(t[a]["End_Timestamp"])
            if i < 5 * L:
                if i // 5 == 0:
                    continue
                role = roles[i % 5]
            elif i == len(seg) - 1:
                role = "finalize"
            elif short(r["Kernel_Name"]).startswith("rmsnorm"):
                role = "final RMSNorm"
            else:
                role = "lm_head GEMV"
            dur[role].append((e0 - s0) / 1e3)
            gap[role].append((s0 - pe) / 1e3)
    if not steps:
        return []
    out = ["", f"## In-graph decode step ({len(steps)} steps, layers 1..L-1; layer 0 excluded)", "",
           "Kernel durations only: under --kernel-trace the profiler serialises graph nodes, so "
           "its inter-kernel gaps (and step spans) are profiler artefacts, not the bench's clock.", "",
           "| role | launches | avg us | median us |", "|---|---|---|---|"]
    for role in roles + ["final RMSNorm", "lm_head GEMV", "finalize"]:
        v = dur[role]
        if not v:
            continue
        out.append(f"| {role} | {len(v)} | {statistics.mean(v):.2f} | {statistics.median(v):.2f} |")
    per_layer = sum(statistics.mean(dur[r]) for r in roles)
    out.append("")
    out.append(f"Sum of in-graph kernel durations per layer: {per_layer:.1f} us; "
               f"gate/up in-graph average {statistics.mean(dur['gate/up GEMV']):.2f} us.")
    return out


HEADLINE = ("`rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --steps 64 --warmup 4 "
            "--prefill-iters 1 --no-cpu-baseline --no-configs` (Qwen2-7B bf16, batch 1, prompt 2048; prefill x2 + 4 "
            "warm-up + 64 timed hipGraph decode steps + bench's live kernel timings).")


def main(tag="r01", src="gpurun_out/prof", desc=HEADLINE, how="tools/gpu_check.sh PROFILE=1"):
    src = os.path.join(ROOT, src)
    trace = list(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))))
    groups = collections.defaultdict(list)
    for r in trace:
        key = short(r["Kernel_Name"])
        if key.startswith("gemv_kernel"):
            # call sites apart: workgroups x threads identify the GEMV
            wg = int(r["Workgroup_Size_X"])
            key += f" [g {int(r['Grid_Size_X']) // wg} x {wg}]"
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in groups.values())
    lines = [f"# rocprofv3 kernel summary ({tag})", "",
             f"Command ({how}, one MI355X):", desc, "",
             "| kernel | role | calls | avg us | median us | total ms | % |", "|---|---|---|---|---|---|---|"]
    for name, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{name}` | {ROLE.get(name, '')} | {len(v)} | {statistics.mean(v):.2f} | "
                     f"{statistics.median(v):.2f} | {sum(v) / 1e3:.3f} | {100 * sum(v) / total:.2f} |")
    lines += in_graph_decode(trace)
    stats = os.path.join(src, "run_kernel_stats.csv")
    if os.path.exists(stats):
        lines += ["", "Raw per-kernel stats (rocprofv3 `--stats`, template arguments folded): "
                  f"`{tag}_kernel_stats.csv`."]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{tag}_rocprof_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    print("\n".join(lines))


if __name__ == "__main__":
    if any(x.startswith("-") for x in sys.argv[1:]):
        sys.exit("usage: tools/prof_summary.py TAG [SRC_DIR] [DESCRIPTION] [HOW]")
    main(*sys.argv[1:])
