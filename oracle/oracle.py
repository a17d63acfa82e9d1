"""numpy/ctypes front-end of the CPU oracle (oracle/qie_oracle.cpp).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  Each function names the reference
kernel it restates (see qie_oracle.cpp for file:line citations).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "liboracle.so")
REF_ROPE_LIB = os.path.join(_HERE, "_ref", "libref_rope.so")
_lib = None

sys.path.insert(0, os.path.dirname(_HERE))
from qwen_inference_engine_amd import _lib as qlib  # noqa: E402  (struct layouts only)


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = C.CDLL(_LIB)
        P = C.c_void_p
        I64, I32, F = C.c_int64, C.c_int32, C.c_float
        sig = {
            "or_rope_table_ref": (None, [P, P, C.c_int, C.c_int, F]),
            "or_rope_table_hf": (None, [P, P, C.c_int, C.c_int, F]),
            "or_rmsnorm": (None, [P, P, P, I64, I64, F, C.c_int]),
            "or_matmul": (None, [P, P, P, P, I64, I64, I64, C.c_int]),
            "or_qknorm": (None, [P, P, I64, I64, C.c_int, C.c_int, F, C.c_int]),
            "or_rope": (None, [P, P, P, P, I64, I64, C.c_int, C.c_int, C.c_int]),
            "or_silu_mul": (None, [P, P, P, I64]),
            "or_resadd": (None, [P, P, I64]),
            "or_embedding": (None, [P, P, P, I64, I64]),
            "or_attention": (None, [P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, I64, C.c_int]),
            "or_topk_ref": (C.c_int, [P, I64, C.c_int, P, P]),
            "or_argmax_ref": (C.c_int, [P, I64]),
            "or_sample_ref": (C.c_int, [P, I64, C.c_int, F, F, C.c_uint64]),
            "or_curand_uniform_first": (F, [C.c_uint64]),
            "or_set_sum_order": (None, [C.c_int]),
            "or_set_act_fp8": (None, [C.c_int]),
            "or_set_hf_eager": (None, [C.c_int]),
            "or_quant_rows_fp8": (None, [P, C.c_int64, C.c_int64, P]),
            "or_e4m3_round": (C.c_float, [C.c_float]),
            "or_set_layer_dump": (None, [P]),
            "or_forward": (C.c_int, [C.POINTER(qlib.ModelSpecC), C.POINTER(qlib.ModelWeightsC), P, P,
                                     C.c_int, P, C.c_int, C.c_int, P, P, C.c_int]),
        }
        for n, (r, a) in sig.items():
            f = getattr(_lib, n)
            f.restype, f.argtypes = r, a
    return _lib


def _p(a: np.ndarray) -> int:
    assert a.flags.c_contiguous
    return a.ctypes.data


def bf16_to_f32(a: np.ndarray) -> np.ndarray:
    return (a.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = 0x7FFF
    return r


def rope_table(n_pos: int, head_dim: int, theta: float = 1e6, numerics: str = "ref"):
    c = np.zeros((n_pos, head_dim // 2), np.float32)
    s = np.zeros_like(c)
    f = lib().or_rope_table_ref if numerics == "ref" else lib().or_rope_table_hf
    f(_p(c), _p(s), n_pos, head_dim, theta)
    return c, s


def rmsnorm(x, w, eps, numerics="ref"):
    x = np.ascontiguousarray(x, np.uint16)
    y = np.zeros_like(x)
    H = x.shape[-1]
    lib().or_rmsnorm(_p(x), _p(np.ascontiguousarray(w, np.uint16)), _p(y), x.size // H, H, eps,
                     0 if numerics == "ref" else 1)
    return y


def matmul(a, w, bias=None, nthreads=0):
    a = np.ascontiguousarray(a, np.uint16)
    w = np.ascontiguousarray(w, np.uint16)
    K = a.shape[-1]
    M = a.size // K
    N = w.shape[0]
    out = np.zeros((M, N), np.uint16)
    b = None if bias is None else np.ascontiguousarray(bias, np.uint16)
    lib().or_matmul(_p(a), _p(w), None if b is None else _p(b), _p(out), M, K, N, nthreads)
    return out


def qknorm(x, w, nheads, hd, eps, numerics="ref"):
    x = np.array(x, np.uint16, copy=True, order="C")
    rows = x.shape[0]
    lib().or_qknorm(_p(x), _p(np.ascontiguousarray(w, np.uint16)), rows, x.shape[1], nheads, hd, eps,
                    0 if numerics == "ref" else 1)
    return x


def rope(x, cos, sin, pos, nheads, hd, numerics="ref"):
    x = np.array(x, np.uint16, copy=True, order="C")
    pos = np.ascontiguousarray(pos, np.int32)
    lib().or_rope(_p(x), _p(cos), _p(sin), _p(pos), x.shape[0], x.shape[1], nheads, hd,
                  0 if numerics == "ref" else 1)
    return x


def silu_mul(gate, up):
    gate = np.ascontiguousarray(gate, np.uint16)
    h = np.zeros_like(gate)
    lib().or_silu_mul(_p(gate), _p(np.ascontiguousarray(up, np.uint16)), _p(h), gate.size)
    return h


def resadd(x, y):
    x = np.array(x, np.uint16, copy=True, order="C")
    lib().or_resadd(_p(x), _p(np.ascontiguousarray(y, np.uint16)), x.size)
    return x


def attention(q, kc, vc, nq, nkv, hd, causal, q_abs_base, nthreads=0):
    """q [mq, nq*hd]; kc/vc [nkv, ctx, hd] (one layer)."""
    q = np.ascontiguousarray(q, np.uint16)
    kc = np.ascontiguousarray(kc, np.uint16)
    vc = np.ascontiguousarray(vc, np.uint16)
    mq, mkv = q.shape[0], kc.shape[1]
    out = np.zeros((mq, nq * hd), np.uint16)
    lib().or_attention(_p(q), _p(kc), _p(vc), _p(out), mq, mkv, nq, nkv, hd, int(causal), q_abs_base,
                       mkv * hd, nthreads)
    return out


def topk(logits, k):
    logits = np.ascontiguousarray(logits, np.uint16)
    idx = np.zeros(256, np.int32)
    val = np.zeros(256, np.float32)
    n = lib().or_topk_ref(_p(logits), logits.size, k, _p(idx), _p(val))
    return idx[:n], val[:n]


def set_sum_order(v: int) -> None:
    """Matmul summation-order variant (0 default, 1 alternative; see or_set_sum_order)."""
    lib().or_set_sum_order(int(v))


def set_hf_eager(v: int) -> None:
    """HF numerics attention form: 0 = fp32 scores / softmax (transformers' sdpa and fused
    kernels; the engine's), 1 = transformers' eager_attention_forward (bf16 scores and
    probabilities; the tests/golden/hf_* fixtures)."""
    lib().or_set_hf_eager(int(v))


def quant_rows_fp8(x):
    """Per-row e4m3 activation quantisation (or_quant_rows_fp8): (dequantised bf16 rows,
    exponents e with scale 2^e)."""
    x = np.array(x, np.uint16, copy=True, order="C")
    rows, cols = x.shape
    e = np.zeros(rows, np.int32)
    lib().or_quant_rows_fp8(_p(x), rows, cols, _p(e))
    return x, e


def argmax(logits) -> int:
    logits = np.ascontiguousarray(logits, np.uint16)
    return lib().or_argmax_ref(_p(logits), logits.size)


def sample(logits, k, temperature, top_p=1.0, seed=1234) -> int:
    logits = np.ascontiguousarray(logits, np.uint16)
    return lib().or_sample_ref(_p(logits), logits.size, k, temperature, top_p, seed)


class Model:
    """Full reference-semantics forward (or_forward) over a HostWeights checkpoint."""

    def __init__(self, hw, max_ctx: int, nthreads: int = 0, prefill_act_fp8: bool = False):
        from qwen_inference_engine_amd.engine import weights_struct
        self.prefill_act_fp8 = prefill_act_fp8   # the engine's prefill_fp8 numerics (or_set_act_fp8)
        self.hw = hw
        self.spec = hw.spec
        self.max_ctx = max_ctx
        self.nthreads = nthreads
        self._arrs = {n: np.ascontiguousarray(a, np.uint16) for n, a in hw.tensors.items()}
        self._w, self._layers = weights_struct(self.spec, {n: a.ctypes.data for n, a in self._arrs.items()})
        self._spec_c = self.spec.to_c()
        s = self.spec
        self.k = np.zeros((s.n_layers, s.n_kv_heads, max_ctx, s.head_dim), np.uint16)
        self.v = np.zeros_like(self.k)
        self.pos = 0

    def forward(self, ids, start_pos=None):
        """Process ids at positions start_pos.. (default: continue); return bf16 logits [V]."""
        ids = np.ascontiguousarray(ids, np.int32)
        sp = self.pos if start_pos is None else start_pos
        logits = np.zeros(self.spec.vocab, np.uint16)
        hidden = np.zeros(self.spec.hidden, np.uint16)
        q8 = self.prefill_act_fp8 and sp == 0   # the prefill call (decode steps keep bf16 activations)
        if q8:
            lib().or_set_act_fp8(1)
        try:
            rc = lib().or_forward(C.byref(self._spec_c), C.byref(self._w), _p(self.k), _p(self.v), self.max_ctx,
                                  _p(ids), ids.size, sp, _p(logits), _p(hidden), self.nthreads)
        finally:
            if q8:
                lib().or_set_act_fp8(0)
        if rc != 0:
            raise RuntimeError("or_forward failed")
        self.pos = sp + ids.size
        self.last_hidden = hidden
        return logits

    def forward_dump(self, ids, start_pos=None):
        """forward() that also returns the last token's residual rows bf16 [2L + 1][H] (slot 0
        after the embedding, 2l + 1 / 2l + 2 after layer l's attention / MLP residual adds)."""
        buf = np.zeros((2 * self.spec.n_layers + 1, self.spec.hidden), np.uint16)
        lib().or_set_layer_dump(_p(buf))
        try:
            lg = self.forward(ids, start_pos)
        finally:
            lib().or_set_layer_dump(None)
        return lg, buf

    def generate_greedy(self, prompt, n_new):
        """Prefill + (n_new - 1) decode steps; returns (ids, per-step logits)."""
        out, lg = [], []
        logits = self.forward(prompt, 0)
        for i in range(n_new):
            t = argmax(logits)
            out.append(t)
            lg.append(logits)
            if i + 1 < n_new:
                logits = self.forward([t])
        return out, lg
