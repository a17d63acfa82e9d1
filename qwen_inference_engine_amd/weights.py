"""Reference-compatible weight index and flat ``weights.bin`` tooling.

Mirrors the reference loader (layers/src/tensor_parser.cpp:31-165, tensor_parser.hh:204-210):

* ``parsed_tensors`` — walk safetensors shard headers in order, each header's keys in
  sorted order (nlohmann::json's std::map), keep ``model.*`` and ``lm_*`` keys, re-base
  every tensor's byte range into ONE contiguous weights.bin;
* ``build_indexed_tensors`` — ``index[short_name][layer]`` lookup (globals at [0]);
* ``format_meta`` / ``parse_meta`` — the reference's ``meta_data.txt`` text format
  (``operator<<`` at tensor_parser.cpp:19-28, one blank line after each tensor);
* ``convert_safetensors`` — writes weights.bin + meta_data.txt from HF shards (the
  reference's writer is commented out, tensor_parser.cpp:49,118-121).

Also the synthetic-checkpoint generator (no weights ship in this environment): every
tensor is filled by libqie's counter-based generator (qie_synthetic_fill_host), which is
bit-identical to the device fill used by ``Engine.init_synthetic``.
"""
from __future__ import annotations

import dataclasses
import json
import os
import struct
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .spec import ModelSpec


@dataclasses.dataclass
class Tensor:
    tensor_name: str
    shape: List[int]
    data_offsets: List[int]
    layer_index: int = -1
    short_name: str = ""

    @property
    def nbytes(self) -> int:
        return self.data_offsets[1] - self.data_offsets[0]


def classify(key: str) -> Optional[Tuple[int, str]]:
    """(layer_index, short_name) per tensor_parser.cpp:69-116, or None if skipped."""
    if key.startswith("model."):
        lp = key.find("layers.")
        if lp >= 0:
            dot = key.find(".", lp + 7)
            return int(key[lp + 7:dot]), key[dot + 1:]
        return -1, key[6:]
    if key.startswith("lm_"):
        return -1, "logits"
    return None


def parsed_tensors(shard_headers: Sequence[Dict[str, dict]]) -> List[Tensor]:
    """Re-based index from parsed safetensors headers (one dict per shard, in shard order)."""
    out: List[Tensor] = []
    glob = 0
    for hdr in shard_headers:
        for key in sorted(hdr.keys()):
            c = classify(key)
            if c is None:
                continue
            v = hdr[key]
            size = int(v["data_offsets"][1]) - int(v["data_offsets"][0])
            out.append(Tensor(key, [int(s) for s in v["shape"]], [glob, glob + size], c[0], c[1]))
            glob += size
    return out


def build_indexed_tensors(tensors: Iterable[Tensor]) -> Dict[str, List[Optional[Tensor]]]:
    idx: Dict[str, List[Optional[Tensor]]] = {}
    for t in tensors:
        lst = idx.setdefault(t.short_name, [])
        li = t.layer_index if t.layer_index >= 0 else 0
        if len(lst) <= li:
            lst.extend([None] * (li + 1 - len(lst)))
        lst[li] = t
    return idx


def format_meta(tensors: Iterable[Tensor]) -> str:
    parts = []
    for t in tensors:
        shape = " ".join(str(s) for s in t.shape)
        parts.append(f"Tensor: {t.tensor_name}\n  layer: {t.layer_index}\n  short_name: {t.short_name}\n"
                     f"  shape: [ {shape} ]\n  offsets: [ {t.data_offsets[0]}, {t.data_offsets[1]} ]\n\n")
    return "".join(parts)


def parse_meta(text: str) -> List[Tensor]:
    out: List[Tensor] = []
    cur: Optional[Tensor] = None
    for raw in text.splitlines():
        s = raw.strip()
        if s.startswith("Tensor:"):
            if cur is not None:
                out.append(cur)
            cur = Tensor(s[7:].strip(), [], [0, 0])
        elif cur is None:
            continue
        elif s.startswith("layer:"):
            cur.layer_index = int(s[6:])
        elif s.startswith("short_name:"):
            cur.short_name = s[11:].strip()
        elif s.startswith("shape:"):
            cur.shape = [int(x) for x in s[6:].strip(" []").split()]
        elif s.startswith("offsets:"):
            a, b = s[8:].strip(" []").split(",")
            cur.data_offsets = [int(a), int(b)]
    if cur is not None:
        out.append(cur)
    return out


def read_safetensors_header(path: str) -> Dict[str, dict]:
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        return json.loads(f.read(n))


def hf_tensor_shapes(spec: ModelSpec) -> "OrderedDict[str, List[int]]":
    H, hd, QD, KD, I, V = spec.hidden, spec.head_dim, spec.q_dim, spec.kv_dim, spec.ffn, spec.vocab
    d: "OrderedDict[str, List[int]]" = OrderedDict()
    d["model.embed_tokens.weight"] = [V, H]
    d["model.norm.weight"] = [H]
    if not spec.tie_embeddings:
        d["lm_head.weight"] = [V, H]
    for l in range(spec.n_layers):
        p = f"model.layers.{l}."
        d[p + "input_layernorm.weight"] = [H]
        d[p + "post_attention_layernorm.weight"] = [H]
        d[p + "self_attn.q_proj.weight"] = [QD, H]
        d[p + "self_attn.k_proj.weight"] = [KD, H]
        d[p + "self_attn.v_proj.weight"] = [KD, H]
        d[p + "self_attn.o_proj.weight"] = [H, QD]
        if spec.qkv_bias:
            d[p + "self_attn.q_proj.bias"] = [QD]
            d[p + "self_attn.k_proj.bias"] = [KD]
            d[p + "self_attn.v_proj.bias"] = [KD]
        if spec.qk_norm:
            d[p + "self_attn.q_norm.weight"] = [hd]
            d[p + "self_attn.k_norm.weight"] = [hd]
        d[p + "mlp.gate_proj.weight"] = [I, H]
        d[p + "mlp.up_proj.weight"] = [I, H]
        d[p + "mlp.down_proj.weight"] = [H, I]
    return d


def synthetic_index(spec: ModelSpec) -> List[Tensor]:
    """Index of a one-shard HF checkpoint of ``spec`` (same as libqie's qie_index_synthetic)."""
    hdr = {}
    off = 0
    for name, shape in hf_tensor_shapes(spec).items():
        n = int(np.prod(shape)) * 2
        hdr[name] = {"dtype": "BF16", "shape": shape, "data_offsets": [off, off + n]}
        off += n
    return parsed_tensors([hdr])


# ------------------------------------------------------------------ fp8 weights
def e4m3_table() -> np.ndarray:
    """float32 value of every OCP e4m3fn code (0x7F / 0xFF are NaN)."""
    c = np.arange(256)
    ex, man = (c >> 3) & 0xF, c & 7
    v = np.where(ex == 0, man * 2.0 ** -9, (1 + man / 8.0) * 2.0 ** (ex - 7.0))
    v = np.where((c & 0x7F) == 0x7F, np.nan, v)
    return np.where(c & 0x80, -v, v).astype(np.float32)


def quantize_fp8(w: np.ndarray):
    """bf16 [rows, cols] -> (e4m3 codes uint8 [rows, cols], fp32 power-of-two row scales),
    libqie's host quantiser (bit-identical to the device one, qie_quantize_fp8)."""
    w = np.ascontiguousarray(w, np.uint16)
    rows, cols = w.shape
    lib = _lib.load()
    out = np.empty(int(lib.qie_fp8_weight_bytes(rows, cols)), np.uint8)
    _lib.check(lib.qie_quantize_fp8_host(w.ctypes.data, rows, cols, out.ctypes.data), "qie_quantize_fp8_host")
    return out[:rows * cols].reshape(rows, cols), out[rows * cols:].view(np.float32).copy()


def dequantize_fp8(codes: np.ndarray, scales: np.ndarray) -> np.ndarray:
    """codes x row scale as bf16 bits (exact: 3 mantissa bits x 2^k)."""
    v = e4m3_table()[codes] * scales[:, None].astype(np.float32)
    b = v.view(np.uint32)
    assert not (b & 0xFFFF).any(), "dequantised fp8 value not exactly representable in bf16"
    return (b >> 16).astype(np.uint16)


# ------------------------------------------------------------------ synthetic values
@dataclasses.dataclass(frozen=True)
class SynthParams:
    seed: int = 0
    w_scale: float = 0.0346   # uniform[-a, a) with std 0.02 (N(0, 0.02))
    norm_scale: float = 0.0   # norm weights 1 + norm_scale*u   (reference init: 1)
    bias_scale: float = 0.0346
    # Peaked head (parity runs only): lm_head rows r with r % head_boost_every == 0 are
    # multiplied by 2^head_boost_log2 (exact in bf16).  A random head gives near-flat
    # logits whose top-2 gaps sit inside the ~4 % full-depth summation-order spread of any
    # bf16 pipeline; a few boosted rows concentrate the competition the way a trained
    # model's unembedding does.  0 = off.  A tied head is the embedding.
    head_boost_every: int = 0
    head_boost_log2: int = 0

    def for_tensor(self, short_name: str) -> Tuple[float, float]:
        """(scale, offset) of a tensor by role."""
        if "norm" in short_name:
            return self.norm_scale, 1.0
        if "bias" in short_name:
            return self.bias_scale, 0.0
        return self.w_scale, 0.0


def tensor_id(name: str) -> int:
    h = 2166136261
    for ch in name.encode():
        h ^= ch
        h = (h * 16777619) & 0xFFFFFFFF
    return h


def synthetic_tensor(name: str, short_name: str, numel: int, p: SynthParams) -> np.ndarray:
    lib = _lib.load()
    out = np.empty(numel, dtype=np.uint16)
    scale, offset = p.for_tensor(short_name)
    _lib.check(lib.qie_synthetic_fill_host(out.ctypes.data, numel, tensor_id(name), p.seed, scale, offset),
               "qie_synthetic_fill_host")
    return out


class HostWeights:
    """All tensors of a checkpoint as host bf16 (uint16) arrays, by full tensor name."""

    def __init__(self, spec: ModelSpec, tensors: Dict[str, np.ndarray]):
        self.spec = spec
        self.tensors = tensors

    @classmethod
    def synthetic(cls, spec: ModelSpec, p: SynthParams = SynthParams()) -> "HostWeights":
        t = {}
        for name, shape in hf_tensor_shapes(spec).items():
            c = classify(name)
            t[name] = synthetic_tensor(name, c[1], int(np.prod(shape)), p).reshape(shape)
        hw = cls(spec, t)
        if p.head_boost_every > 0 and p.head_boost_log2 != 0:
            hw.boost_head(p.head_boost_every, p.head_boost_log2)
        return hw

    def boost_head(self, every: int, log2f: int) -> None:
        """lm_head rows r % every == 0 times 2^log2f (libqie's qie_scale_rows_pow2 on the host)."""
        name = "model.embed_tokens.weight" if self.spec.tie_embeddings else "lm_head.weight"
        w = self.tensors[name].copy()
        f = (w[::every].astype(np.uint32) << 16).view(np.float32) * np.float32(2.0 ** log2f)
        assert np.isfinite(f).all()
        w[::every] = (f.view(np.uint32) >> 16).astype(np.uint16)
        self.tensors[name] = w

    @classmethod
    def from_weights_bin(cls, spec: ModelSpec, bin_path: str, meta_path: str) -> "HostWeights":
        with open(meta_path) as f:
            idx = parse_meta(f.read())
        mm = np.memmap(bin_path, dtype=np.uint16, mode="r")
        t = {}
        for e in idx:
            a, b = e.data_offsets
            t[e.tensor_name] = np.asarray(mm[a // 2:b // 2]).reshape(e.shape)
        return cls(spec, t)

    def get(self, name: str) -> Optional[np.ndarray]:
        return self.tensors.get(name)

    def layer(self, l: int, short: str) -> Optional[np.ndarray]:
        return self.tensors.get(f"model.layers.{l}.{short}")

    @property
    def lm_head(self) -> np.ndarray:
        if self.spec.tie_embeddings:
            return self.tensors["model.embed_tokens.weight"]
        return self.tensors["lm_head.weight"]

    def fp8_dequantized(self) -> "HostWeights":
        """The model the fp8 engine computes (``qie_engine_opts.weight_fp8``): every linear
        weight and the lm_head replaced by its e4m3 x power-of-two-scale dequantisation
        (exactly representable in bf16).  A tied head gets its own (quantised) copy, so the
        returned spec is untied; the token embedding stays bf16."""
        t = dict(self.tensors)
        spec = self.spec
        for l in range(spec.n_layers):
            for short in ("self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
                          "self_attn.o_proj.weight", "mlp.gate_proj.weight", "mlp.up_proj.weight",
                          "mlp.down_proj.weight"):
                name = f"model.layers.{l}.{short}"
                t[name] = dequantize_fp8(*quantize_fp8(t[name]))
        t["lm_head.weight"] = dequantize_fp8(*quantize_fp8(self.lm_head))
        return HostWeights(spec.replace(tie_embeddings=False), t)

    def write_weights_bin(self, bin_path: str, meta_path: str) -> List[Tensor]:
        """Write the reference flat layout: tensors in parsed_tensors order, no gaps."""
        hdr = {n: {"shape": list(a.shape), "data_offsets": [0, a.nbytes]} for n, a in self.tensors.items()}
        idx = parsed_tensors([hdr])
        with open(bin_path, "wb") as f:
            for e in idx:
                assert f.tell() == e.data_offsets[0]
                f.write(np.ascontiguousarray(self.tensors[e.tensor_name]).tobytes())
        with open(meta_path, "w") as f:
            f.write(format_meta(idx))
        return idx


def convert_safetensors(shards: Sequence[str], bin_path: str, meta_path: str,
                        chunk: int = 1 << 26) -> List[Tensor]:
    """HF safetensors shards -> reference weights.bin + meta_data.txt (bf16 tensors only)."""
    headers = []
    for p in shards:
        h = read_safetensors_header(p)
        h.pop("__metadata__", None)
        for k, v in h.items():
            if classify(k) is not None and v.get("dtype", "BF16") != "BF16":
                raise ValueError(f"{p}:{k} has dtype {v.get('dtype')}; weights.bin is bf16")
        headers.append(h)
    idx = parsed_tensors(headers)
    with open(bin_path, "wb") as out:
        for p, h in zip(shards, headers):
            with open(p, "rb") as f:
                n = struct.unpack("<Q", f.read(8))[0]
                base = 8 + n
                for key in sorted(h.keys()):
                    if classify(key) is None:
                        continue
                    a, b = h[key]["data_offsets"]
                    f.seek(base + a)
                    left = b - a
                    while left > 0:
                        buf = f.read(min(chunk, left))
                        out.write(buf)
                        left -= len(buf)
    with open(meta_path, "w") as f:
        f.write(format_meta(idx))
    return idx
