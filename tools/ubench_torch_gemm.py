#!/usr/bin/env python3
"""Reference point for the prefill GEMMs: torch.matmul (hipBLASLt / rocBLAS) on the
Qwen2-7B P = 2048 projection shapes, bf16, timed with events over 20 launches.  Only a
yardstick for DESIGN.md §3 — the engine does not call it."""
import json
import torch

M, H, I, QKV = 2048, 3584, 18944, 4608
shapes = {"qkv": (M, H, QKV), "o": (M, H, H), "gate_up": (M, H, 2 * I), "down": (M, I, H)}
out = {}
for name, (m, k, n) in shapes.items():
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
    for _ in range(3):
        y = a @ w.t()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        y = a @ w.t()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    out[name] = {"us": round(us, 1), "tflops": round(2.0 * m * n * k / us / 1e6, 1)}
print(json.dumps(out))
