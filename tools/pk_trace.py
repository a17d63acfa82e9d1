#!/usr/bin/env python3
"""Phase timeline of the persistent decode step (decode mode 1, qie_batch_pk_trace): every CU
stamps s_memrealtime (100 MHz, chip-wide) at its phase boundaries; this prints, per phase,
the median over layers 1..L-1 of the CUs' median and maximum time since the layer's first
start, and the layer period.  Slots: 0 start, 1 x gathered, 2 QKV done, 3 attention done
(attention CUs), 4 attention output gathered (O CUs), 5 O done, 6 x' gathered (+norm),
7 gate/up done, 8 h gathered, 9 down done.

Env: PT_MODEL (Qwen2-7B), PT_P (2048), PT_OUT (optional .npz of the raw stamps)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import _lib, spec as S, weights as W  # noqa: E402

NAMES = {1: "x_gathered", 2: "qkv_done", 3: "attn_done", 4: "att_gathered", 5: "o_done", 6: "x1_gathered",
         7: "gate_up_done", 8: "h_gathered", 9: "down_done"}


def main():
    spec = S.PRESETS[os.environ.get("PT_MODEL", "Qwen2-7B")]
    P = int(os.environ.get("PT_P", "2048"))
    eng = Q.Engine(spec, max_ctx=P + 64).init_synthetic(W.SynthParams(seed=0))
    b = eng.batch(1, P + 64)
    b.set_decode_mode(1)
    lib = b.lib
    _lib.check(lib.qie_batch_pk_trace(b.h, 1, None, 0), "pk_trace")
    b.prefill(0, [int(t) for t in np.random.default_rng(1).integers(0, spec.vocab, P)])
    b.decode(4)
    L = spec.n_layers
    import ctypes
    n = 1024 * L * 12   # >= n_cu * L * 12; rows past the device's CU count stay zero
    buf = np.zeros(n, np.uint64)
    _lib.check(lib.qie_batch_pk_trace(b.h, 1, buf.ctypes.data_as(ctypes.c_void_p), n), "pk_trace read")
    full = buf.reshape(1024, L, 12)
    props = int((full[:, :, 0] > 0).any(axis=1).sum())
    t = full[:props].astype(np.int64)
    if os.environ.get("PT_OUT"):
        np.savez_compressed(os.environ["PT_OUT"], stamps=t)
    res = {"model": spec.name, "ctx": P + 4, "n_cu": props, "units": "us"}
    per = []
    for l in range(1, L):
        s0 = t[:, l, 0].min()
        row = {}
        for k, name in NAMES.items():
            v = t[:, l, k]
            v = v[v > 0]
            if len(v) == 0:
                continue
            d = (v - s0) / 100.0
            row[name] = (float(np.median(d)), float(d.max()))
        if l + 1 < L:
            row["period"] = (float((t[:, l + 1, 0].min() - s0) / 100.0),) * 2
        per.append(row)
    keys = list(NAMES.values()) + ["period"]
    summ = {}
    for k in keys:
        med = [r[k][0] for r in per if k in r]
        mx = [r[k][1] for r in per if k in r]
        if med:
            summ[k] = {"cu_median": round(float(np.median(med)), 2), "cu_max": round(float(np.median(mx)), 2)}
    res["phases_since_layer_start"] = summ
    k0 = t[:, 0, 0]
    res["kernel_span_us"] = round(float((t[:, L - 1, 9].max() - k0.min()) / 100.0), 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
