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
ROLE_7B = {   # Qwen2-7B call sites by (grid blocks, static LDS bytes; dynamic LDS is not reported)
    "gemv_kernel [grid 2048, lds 0]": "decode gate/up GEMV (+RMSNorm, SwiGLU)  [dominant]",
    "gemv_kernel [grid 448, lds 0]": "decode down GEMV and O-proj GEMV (+residual; same grid)",
    "gemv_kernel [grid 576, lds 512]": "decode QKV GEMV (+RMSNorm, bias)",
    "gemv_kernel [grid 2048, lds 512]": "lm_head GEMV (+final RMSNorm, arg-max keys)",
    "gemv_kernel [grid 448, lds 512]": "bench live timing of down / O-proj (store epilogue)",
    "gemm_kernel [grid 16, lds 0]": "prefill GEMMs (MFMA 128x128 tiles)",
}
ROLE = {
    "gemv_kernel<1, 2, 2, 8, false>": "decode gate/up GEMV (+RMSNorm, SwiGLU)  [dominant]",
    "gemv_kernel<1, 2, 1, 8, false>": "decode O-proj / down GEMV (+residual)",
    "gemv_kernel<1, 2, 0, 8, false>": "decode QKV GEMV (+RMSNorm, bias) / lm_head (+arg-max)",
    "attn_decode_mfma_kernel<128>": "decode attention (fused qk-norm/RoPE/KV append, split-K)",
    "attn_prefill_mfma_kernel<128>": "prefill flash attention (MFMA)",
    "gemm_kernel<0>": "prefill GEMM (store/bias)",
    "gemm_kernel<1>": "prefill GEMM (+residual)",
    "gemm_kernel<2>": "prefill GEMM (gate/up + SwiGLU)",
}


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("qie::", "")
    return n


def main(tag="r01", src="gpurun_out/prof"):
    src = os.path.join(ROOT, src)
    trace = list(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))))
    groups = collections.defaultdict(list)
    for r in trace:
        key = short(r["Kernel_Name"])
        if key.startswith("gemv_kernel") or key.startswith("gemm_kernel"):
            # instantiations / call sites apart: grid and LDS bytes identify the GEMV (K sizes LDS)
            key += f" [grid {int(r['Grid_Size_X']) // 256}, lds {r['LDS_Block_Size']}]"
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in groups.values())
    lines = [f"# rocprofv3 kernel summary ({tag})", "",
             "Command (tools/gpu_check.sh PROFILE=1, one MI355X):",
             "`rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --steps 64 --warmup 4 "
             "--prefill-iters 1 --no-cpu-baseline` (Qwen2-7B bf16, batch 1, prompt 2048; prefill x2 + 4 warm-up + "
             "64 timed hipGraph decode steps + bench's live kernel timings).", "",
             "| kernel | role | calls | avg us | median us | total ms | % |", "|---|---|---|---|---|---|---|"]
    for name, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{name}` | {ROLE.get(name, ROLE_7B.get(name, ''))} | {len(v)} | {statistics.mean(v):.2f} | "
                     f"{statistics.median(v):.2f} | {sum(v) / 1e3:.3f} | {100 * sum(v) / total:.2f} |")
    lines += ["", "Raw per-kernel stats (rocprofv3 `--stats`, template arguments folded): "
              f"`{tag}_kernel_stats.csv`."]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{tag}_rocprof_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    shutil.copy(os.path.join(src, "run_kernel_stats.csv"), os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
