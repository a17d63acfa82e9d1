"""Model specs (replace the reference's hard-coded Qwen3-14B dims).

Reference literals: layers/src/utills.cu:8-16 (dims), layers/include/iengine.cuh:19-21
(CONTEXT_SIZE, HIDDEN_DIM_KV, NUM_OF_LAYERS), normalization.cu:9 / qk_norm.cu:46 (eps 1e-4),
include.cpp:7 (RoPE base 1e6).  In ``ref`` numerics the reference's eps/base are used for
every model (they are op semantics of the reference engine); ``hf`` numerics take the
model's own config values.
"""
from __future__ import annotations

import dataclasses
import json

from ._lib import ModelSpecC, QIE_NUMERICS_HF, QIE_NUMERICS_REF

REF_EPS = 1e-4        # normalization.cu:9, qk_norm.cu:46
REF_THETA = 1e6       # include.cpp:7


@dataclasses.dataclass(frozen=True)
class ModelSpec:
    name: str
    n_layers: int
    hidden: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn: int
    vocab: int
    tie_embeddings: bool
    qkv_bias: bool
    qk_norm: bool
    hf_eps: float
    hf_theta: float = 1e6
    numerics: str = "ref"

    @property
    def rms_eps(self) -> float:
        return REF_EPS if self.numerics == "ref" else self.hf_eps

    @property
    def rope_theta(self) -> float:
        return REF_THETA if self.numerics == "ref" else self.hf_theta

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    def with_numerics(self, numerics: str) -> "ModelSpec":
        assert numerics in ("ref", "hf")
        return dataclasses.replace(self, numerics=numerics)

    def replace(self, **kw) -> "ModelSpec":
        return dataclasses.replace(self, **kw)

    def to_c(self) -> ModelSpecC:
        s = ModelSpecC()
        s.n_layers, s.hidden, s.n_heads = self.n_layers, self.hidden, self.n_heads
        s.n_kv_heads, s.head_dim, s.ffn, s.vocab = self.n_kv_heads, self.head_dim, self.ffn, self.vocab
        s.tie_embeddings, s.qkv_bias, s.qk_norm = int(self.tie_embeddings), int(self.qkv_bias), int(self.qk_norm)
        s.rms_eps, s.rope_theta = self.rms_eps, self.rope_theta
        s.numerics = QIE_NUMERICS_REF if self.numerics == "ref" else QIE_NUMERICS_HF
        return s

    # ------------------------------------------------------------ accounting
    def layer_weight_bytes(self) -> int:
        H, I = self.hidden, self.ffn
        n = (self.q_dim + 2 * self.kv_dim) * H + H * self.q_dim + 3 * H * I + 2 * H
        if self.qkv_bias:
            n += self.q_dim + 2 * self.kv_dim
        if self.qk_norm:
            n += 2 * self.head_dim
        return 2 * n

    def decode_weight_bytes(self, fp8: bool = False) -> int:
        """Weights streamed per decode step: every layer + final norm + lm_head once.
        fp8: linear weights and lm_head at 1 byte per weight + one fp32 scale per row."""
        if not fp8:
            return self.n_layers * self.layer_weight_bytes() + 2 * self.hidden + 2 * self.vocab * self.hidden
        lin = self.linear_params_per_layer()
        rows = self.q_dim + 2 * self.kv_dim + self.hidden + 2 * self.ffn + self.hidden
        other = self.layer_weight_bytes() - 2 * lin            # norms, biases (bf16)
        per_layer = lin + 4 * rows + other
        return self.n_layers * per_layer + 2 * self.hidden + (self.vocab * self.hidden + 4 * self.vocab)

    def kv_bytes_per_position(self) -> int:
        return self.n_layers * 2 * self.kv_dim * 2

    def linear_params_per_layer(self) -> int:
        H, I = self.hidden, self.ffn
        return (self.q_dim + 2 * self.kv_dim) * H + H * self.q_dim + 3 * H * I

    def prefill_flops(self, P: int, B: int = 1) -> float:
        lin = 2.0 * P * B * self.n_layers * self.linear_params_per_layer()
        attn = self.n_layers * 4.0 * self.q_dim * P * (P + 1) / 2 * B
        head = 2.0 * self.hidden * self.vocab * B
        return lin + attn + head

    @classmethod
    def from_hf_config(cls, cfg: dict, name: str = "hf", numerics: str = "ref") -> "ModelSpec":
        hd = cfg.get("head_dim") or cfg["hidden_size"] // cfg["num_attention_heads"]
        mt = cfg.get("model_type", "qwen2")
        return cls(name=name, n_layers=cfg["num_hidden_layers"], hidden=cfg["hidden_size"],
                   n_heads=cfg["num_attention_heads"], n_kv_heads=cfg["num_key_value_heads"],
                   head_dim=hd, ffn=cfg["intermediate_size"], vocab=cfg["vocab_size"],
                   tie_embeddings=bool(cfg.get("tie_word_embeddings", False)),
                   qkv_bias=(mt == "qwen2") or bool(cfg.get("attention_bias", False)),
                   qk_norm=(mt == "qwen3"), hf_eps=float(cfg.get("rms_norm_eps", 1e-6)),
                   hf_theta=float(cfg.get("rope_theta", 1e6)), numerics=numerics)

    @classmethod
    def from_json(cls, path: str, numerics: str = "ref") -> "ModelSpec":
        with open(path) as f:
            return cls.from_hf_config(json.load(f), name=path, numerics=numerics)


QWEN2_0_5B = ModelSpec("Qwen2-0.5B", 24, 896, 14, 2, 64, 4864, 151936, True, True, False, 1e-6)
QWEN2_7B = ModelSpec("Qwen2-7B", 28, 3584, 28, 4, 128, 18944, 152064, False, True, False, 1e-6)
QWEN2_72B = ModelSpec("Qwen2-72B", 80, 8192, 64, 8, 128, 29568, 152064, False, True, False, 1e-5)
QWEN3_14B = ModelSpec("Qwen3-14B", 40, 5120, 40, 8, 128, 17408, 151936, False, False, True, 1e-6)

PRESETS = {s.name: s for s in (QWEN2_0_5B, QWEN2_7B, QWEN2_72B, QWEN3_14B)}


def tiny(name: str = "tiny-qwen2", *, n_layers=2, hidden=128, n_heads=4, n_kv_heads=2, head_dim=64,
         ffn=256, vocab=512, tie=False, bias=True, qk_norm=False, numerics="ref") -> ModelSpec:
    """Small test configurations (oracle finishes in well under a second)."""
    return ModelSpec(name, n_layers, hidden, n_heads, n_kv_heads, head_dim, ffn, vocab, tie, bias,
                     qk_norm, 1e-6, 1e6, numerics)


def shard_heads(nq: int, nkv: int, tp: int, rank: int):
    """(local q heads, first q head, local kv heads, first kv head) of `rank` — the rule of
    engine.hip shard_heads: even split when tp divides the kv heads, else every kv head on
    tp / nkv ranks that split its group's q heads (the first G % rep ranks one more);
    None when the heads do not shard."""
    if nkv % tp == 0 and nq % tp == 0:
        return nq // tp, rank * (nq // tp), nkv // tp, rank * (nkv // tp)
    if tp % nkv:
        return None
    rep, G = tp // nkv, nq // nkv
    if rep > G:
        return None
    g, sub = rank // rep, rank % rep
    base, extra = G // rep, G % rep
    return base + (1 if sub < extra else 0), g * G + sub * base + min(sub, extra), 1, g


def tp_shardable(spec: ModelSpec, tp: int):
    """(ok, reason): can `spec` run tensor-parallel over `tp` ranks (qie_engine_create's check)?"""
    if shard_heads(spec.n_heads, spec.n_kv_heads, tp, 0) is None:
        return False, f"{spec.n_heads} q / {spec.n_kv_heads} kv heads do not shard {tp} ways"
    if spec.ffn % tp or (spec.ffn // tp) % 8:
        return False, f"ffn {spec.ffn} / {tp} is not a multiple of 8"
    if spec.vocab % tp:
        return False, f"vocab {spec.vocab} not divisible by {tp}"
    return True, ""
