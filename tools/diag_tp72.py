#!/usr/bin/env python3
"""Diagnostic: Qwen2-72B widths, 2 layers: prefill logits of TP 1 and TP 8 (local
communicator) and of the CPU oracle, norm-relative differences."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O
import qwen_inference_engine_amd as Q
from qwen_inference_engine_amd import spec as S, weights as W
from test_gpu_tp import run_ranks
from parity import norm_rel

L = int(os.environ.get("DIAG_L", "2"))
spec = S.QWEN2_72B.replace(n_layers=L)
syn = W.SynthParams(seed=0)
prompt = [int(t) for t in np.random.default_rng(72).integers(0, spec.vocab, 16)]
hw = W.HostWeights.synthetic(spec, syn)
ref = O.Model(hw, 32).forward(prompt, 0)
del hw
e1 = Q.Engine(spec, max_ctx=64).init_synthetic(syn)
b1 = e1.batch(1, 64)
t1 = b1.prefill(0, prompt)
l1 = b1.logits()[0]
e1.close()
np.savez(os.path.join(ROOT, "gpurun_out", "diag72.npz"), tp1=l1, ref=ref)
print(f"tp1 id {t1} oracle id {O.argmax(ref)} rel {norm_rel(l1, ref):.3e}", flush=True)
for world in [int(x) for x in os.environ.get("DIAG_WORLDS", "2,4,8").split(",")]:
    def fn(rank, comm):
        e = Q.Engine(spec, max_ctx=64, comm=comm).init_synthetic(syn)
        b = e.batch(1, 64)
        t = b.prefill(0, prompt)
        lg = b.logits()[0]
        e.close()
        return t, lg
    res = run_ranks(world, fn, timeout=600)
    tw, lw = res[0]
    print(f"tp{world}: shape {lw.shape} id {tw} | tp1 id {t1} | oracle id {O.argmax(ref)} | "
          f"rel(tp1, oracle) {norm_rel(l1, ref):.3e} rel(tp{world}, tp1) {norm_rel(lw, l1):.3e} "
          f"rel(tp{world}, oracle) {norm_rel(lw, ref):.3e}", flush=True)
