#!/usr/bin/env python3
"""Dev build (QIE_LIB=.../dev/libqie.so, QIE_GRAPH_DUMP=1): print every node of the batch-1
decode graph (kernel grid / block / dynamic LDS) for GD_MODEL, after a GD_P-token prefill."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qwen_inference_engine_amd as Q  # noqa: E402
from qwen_inference_engine_amd import spec as S, weights as W  # noqa: E402

spec = S.PRESETS[os.environ.get("GD_MODEL", "Qwen2-0.5B")]
P = int(os.environ.get("GD_P", "128"))
eng = Q.Engine(spec, max_ctx=P + 64).init_synthetic(W.SynthParams(seed=0))
b = eng.batch(1, P + 64)
b.prefill(0, [int(t) for t in np.random.default_rng(1).integers(0, spec.vocab, P)])
print(b.decode(2).tolist())
