"""qie — MI355X-native (gfx950 / CDNA4) Qwen decoder inference engine.

A drop-in for the per-token decoder hot path of Rafae1130/qwen_inference_engine
(prefill + decode, layers/src/qwen_main.cu), re-designed for MI355X: hand-written HIP
kernels in libqie.so behind a C ABI (include/qie/*.h), driven from C++ or from this
thin Python layer.  See DESIGN.md.
"""
from .spec import ModelSpec, PRESETS, QWEN2_0_5B, QWEN2_7B, QWEN2_72B, QWEN3_14B, tiny  # noqa: F401
from .weights import HostWeights, SynthParams, synthetic_index, parse_meta, format_meta  # noqa: F401
from .engine import Engine, Batch, Comm, Sampling, GREEDY  # noqa: F401

__version__ = "0.1.0"
