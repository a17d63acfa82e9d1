"""Python host mirror of the reference driver, over libqie.so's C ABI.

Reference driver (layers/src/iengine.cu:226-456, qwen_main.cu:64-417):
``create_new_sequence`` -> ``llm()`` with ``state == prefill`` -> loop ``llm()`` with
``state == decode`` (one token per call).  Here: ``Engine`` (weights + RoPE tables),
``Batch`` (KV cache + per-sequence state for B sequences), ``Batch.prefill`` and
``Batch.decode_step`` / ``Batch.decode`` (hipGraph replays).  All compute runs in
libqie's HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from .spec import ModelSpec
from .weights import SynthParams

REF_PREFILL_SAMPLING = dict(top_k=50, temperature=1.0, seed=1234)   # qwen_main.cu:241
REF_DECODE_SAMPLING = dict(top_k=50, temperature=0.7, seed=1234)    # qwen_main.cu:381-388 (+ step)
REF_EOS = 151645                                                    # qwen_main.cu:257


@dataclasses.dataclass
class Sampling:
    top_k: int = 1
    temperature: float = 1.0
    top_p: float = 1.0
    seed: int = 1234

    def to_c(self) -> _lib.SamplingC:
        s = _lib.SamplingC()
        s.top_k, s.temperature, s.top_p, s.seed = self.top_k, self.temperature, self.top_p, self.seed
        return s


GREEDY = Sampling()

_ROLE_FIELDS = {
    "input_layernorm.weight": "attn_norm", "self_attn.q_proj.weight": "wq",
    "self_attn.k_proj.weight": "wk", "self_attn.v_proj.weight": "wv",
    "self_attn.q_proj.bias": "bq", "self_attn.k_proj.bias": "bk", "self_attn.v_proj.bias": "bv",
    "self_attn.q_norm.weight": "q_norm", "self_attn.k_norm.weight": "k_norm",
    "self_attn.o_proj.weight": "wo", "post_attention_layernorm.weight": "ffn_norm",
    "mlp.gate_proj.weight": "w_gate", "mlp.up_proj.weight": "w_up", "mlp.down_proj.weight": "w_down",
}


def weights_struct(spec: ModelSpec, ptr: Dict[str, int]):
    """Build a qie_model_weights from {full tensor name: pointer}.  Returns (struct, keepalive)."""
    layers = (_lib.LayerWeightsC * spec.n_layers)()
    for l in range(spec.n_layers):
        for short, field in _ROLE_FIELDS.items():
            setattr(layers[l], field, ptr.get(f"model.layers.{l}.{short}"))
    w = _lib.ModelWeightsC()
    w.embed = ptr["model.embed_tokens.weight"]
    w.final_norm = ptr["model.norm.weight"]
    w.lm_head = ptr["model.embed_tokens.weight"] if spec.tie_embeddings else ptr["lm_head.weight"]
    w.n_layers = spec.n_layers
    w.layers = C.cast(layers, C.POINTER(_lib.LayerWeightsC))
    return w, layers


class Comm:
    """Tensor-parallel communicator (qie_comm).  ``Comm.rccl(uid, world, rank, device)`` for
    one process per GPU (rank 0 makes ``Comm.unique_id()`` and ships the bytes to the others);
    ``Comm.local(world)`` for `world` in-process ranks on one device, one host thread each
    (the test backend; engines on it run without hipGraphs)."""

    def __init__(self, handle: int, lib, owner=None):
        self.h, self.lib, self._owner = handle, lib, owner
        w, r = C.c_int32(), C.c_int32()
        _lib.check(lib.qie_comm_rank(handle, C.byref(w), C.byref(r)), "qie_comm_rank")
        self.world, self.rank = w.value, r.value

    @staticmethod
    def unique_id() -> bytes:
        lib = _lib.load()
        buf = C.create_string_buffer(_lib.QIE_COMM_ID_BYTES)
        _lib.check(lib.qie_comm_unique_id(buf), "qie_comm_unique_id")
        return buf.raw

    @staticmethod
    def rccl(uid: bytes, world: int, rank: int, device: int) -> "Comm":
        lib = _lib.load()
        buf = C.create_string_buffer(uid, _lib.QIE_COMM_ID_BYTES)
        h = C.c_void_p()
        _lib.check(lib.qie_comm_create_rccl(buf, world, rank, device, C.byref(h)), "qie_comm_create_rccl")
        return Comm(h.value, lib)

    @staticmethod
    def peer(world: int, rank: int, device: int, exchange) -> "Comm":
        """Peer backend across processes: `exchange(handle_bytes) -> [handle of rank r for r
        in range(world)]` is the host channel (e.g. dist.FileGroup.allgather)."""
        lib = _lib.load()
        h = C.c_void_p()
        buf = C.create_string_buffer(_lib.QIE_COMM_PEER_HANDLE_BYTES)
        _lib.check(lib.qie_comm_create_peer(world, rank, device, C.byref(h), buf), "qie_comm_create_peer")
        comm = Comm(h.value, lib)
        hs = exchange(buf.raw)
        allh = C.create_string_buffer(b"".join(hs), _lib.QIE_COMM_PEER_HANDLE_BYTES * world)
        _lib.check(lib.qie_comm_peer_connect(h, allh), "qie_comm_peer_connect")
        return comm

    @staticmethod
    def peer_local(world: int) -> List["Comm"]:
        """Peer backend for `world` ranks of this process on one device (graph-capturable)."""
        lib = _lib.load()
        hs = (C.c_void_p * world)()
        _lib.check(lib.qie_comm_create_peer_local(world, hs), "qie_comm_create_peer_local")
        return [Comm(hs[r], lib) for r in range(world)]

    def peer_error(self) -> int:
        e = C.c_int32()
        _lib.check(self.lib.qie_comm_peer_error(self.h, C.byref(e)), "qie_comm_peer_error")
        return e.value

    def set_peer_mode(self, tagged: bool = True, push: bool = True) -> None:
        """Peer backend exchange form (qie_comm_peer_set_mode): tagged words polled by the
        readers, pushed by the producing GEMV (defaults), or the flagged form; the same on
        every rank, before the decode graph that should use it is captured."""
        _lib.check(self.lib.qie_comm_peer_set_mode(self.h, int(bool(tagged)), int(bool(push))),
                   "qie_comm_peer_set_mode")

    @staticmethod
    def local(world: int) -> List["Comm"]:
        lib = _lib.load()
        hs = (C.c_void_p * world)()
        _lib.check(lib.qie_comm_create_local(world, hs), "qie_comm_create_local")
        return [Comm(hs[r], lib) for r in range(world)]

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.qie_comm_destroy(self.h)
            self.h = None


class Engine:
    def __init__(self, spec: ModelSpec, device: int = 0, max_ctx: int = 4096, use_graph: bool = True,
                 comm: Optional[Comm] = None, weight_fp8: bool = False, comm_always: bool = False,
                 prefill_fp8: bool = False):
        self.lib = _lib.load()
        self.spec = spec
        self._spec_c = spec.to_c()
        opts = _lib.EngineOptsC()
        opts.device, opts.max_ctx, opts.use_graph = device, max_ctx, int(use_graph)
        opts.tp_rank, opts.tp_size = (comm.rank, comm.world) if comm else (0, 1)
        opts.tp_comm = comm.h if comm else None
        opts.weight_fp8 = int(weight_fp8)
        opts.comm_always = int(comm_always)   # exchange steps through comm even at world 1 (tests)
        # numerics flag: prefill projections on the block-scaled fp8 MFMA (activations quantised
        # per row to e4m3; needs weight_fp8) — the oracle's Model(prefill_act_fp8=True)
        opts.prefill_fp8 = int(prefill_fp8)
        self.comm = comm
        self._fp8 = weight_fp8
        h = C.c_void_p()
        _lib.check(self.lib.qie_engine_create(C.byref(self._spec_c), C.byref(opts), C.byref(h)),
                   "qie_engine_create")
        self.h = h
        self.max_ctx = max_ctx
        self._keep = None

    def init_synthetic(self, p: SynthParams = SynthParams()) -> "Engine":
        _lib.check(self.lib.qie_engine_init_synthetic(self.h, p.seed, p.w_scale, p.norm_scale, p.bias_scale),
                   "qie_engine_init_synthetic")
        if p.head_boost_every > 0 and p.head_boost_log2 != 0:
            self.boost_head(p.head_boost_every, p.head_boost_log2)
        return self

    def boost_head(self, every: int, log2f: int) -> None:
        """lm_head rows r % every == 0 times 2^log2f, in place on device (SynthParams'
        peaked head; same values as HostWeights.boost_head).  bf16 engines; under tensor
        parallelism each rank scales its vocab slice (rows rank*V/tp ..), untied heads only
        (a tied head's slice is a view of the replicated embedding)."""
        if getattr(self, "_fp8", False):
            raise ValueError("boost_head: bf16 engines only")
        rows, row0 = self.spec.vocab, 0
        if self.comm is not None and self.comm.world > 1:
            if self.spec.tie_embeddings:
                raise ValueError("boost_head: tensor-parallel engines with an untied head only")
            rows = self.spec.vocab // self.comm.world
            row0 = self.comm.rank * rows
        w = _lib.ModelWeightsC()
        _lib.check(self.lib.qie_engine_weights(self.h, C.byref(w), None), "qie_engine_weights")
        _lib.check(self.lib.qie_scale_rows_pow2(w.lm_head, rows, self.spec.hidden, row0, every, log2f,
                                                self.stream), "qie_scale_rows_pow2")
        self.sync()

    def load_weights_bin(self, bin_path: str, meta_path: str, chunk_bytes: int = 1 << 28) -> "Engine":
        _lib.check(self.lib.qie_engine_load_weights_bin(self.h, bin_path.encode(), meta_path.encode(),
                                                        chunk_bytes), "qie_engine_load_weights_bin")
        return self

    def set_weights(self, dev_ptrs: Dict[str, int], keepalive=None) -> "Engine":
        w, layers = weights_struct(self.spec, dev_ptrs)
        _lib.check(self.lib.qie_engine_set_weights(self.h, C.byref(w)), "qie_engine_set_weights")
        self._keep = (w, layers, keepalive)
        return self

    @property
    def stream(self) -> int:
        return self.lib.qie_engine_stream(self.h)

    def sync(self) -> None:
        _lib.check(self.lib.qie_engine_sync(self.h), "qie_engine_sync")

    def batch(self, batch: int = 1, max_ctx: Optional[int] = None, page_tokens: Optional[int] = None,
              n_pages: int = 0) -> "Batch":
        """B sequence slots.  page_tokens selects the paged KV cache (device block table over
        a pool of n_pages pages, 0 = enough for every slot at max_ctx); None = contiguous."""
        return Batch(self, batch, max_ctx or self.max_ctx, page_tokens, n_pages)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.qie_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    def __init__(self, engine: Engine, batch: int, max_ctx: int, page_tokens: Optional[int] = None,
                 n_pages: int = 0):
        self.e = engine
        self.lib = engine.lib
        self.B = batch
        self.max_ctx = max_ctx
        self.paged = page_tokens is not None
        h = C.c_void_p()
        if self.paged:
            _lib.check(self.lib.qie_batch_create_paged(engine.h, batch, max_ctx, page_tokens, n_pages, C.byref(h)),
                       "qie_batch_create_paged")
        else:
            _lib.check(self.lib.qie_batch_create(engine.h, batch, max_ctx, C.byref(h)), "qie_batch_create")
        self.h = h

    def prefill(self, seq: int, ids: Sequence[int], sampling: Sampling = GREEDY) -> int:
        arr = (C.c_int32 * len(ids))(*[int(i) for i in ids])
        out = C.c_int32(-1)
        sc = sampling.to_c()
        _lib.check(self.lib.qie_prefill(self.h, seq, arr, len(ids), C.byref(sc), C.byref(out)), "qie_prefill")
        return out.value

    def prefill_batch(self, seq0: int, prompts: Sequence[Sequence[int]], sampling: Sampling = GREEDY) -> List[int]:
        """Equal-length prompts into slots seq0, seq0+1, ... in one pass (qie_prefill_batch)."""
        n = len(prompts)
        length = len(prompts[0]) if n else 0
        if n == 0 or any(len(p) != length for p in prompts):
            raise ValueError("prefill_batch: needs one or more prompts of equal length")
        flat = np.ascontiguousarray(np.asarray(prompts, dtype=np.int32).reshape(-1))
        out = (C.c_int32 * n)()
        sc = sampling.to_c()
        _lib.check(self.lib.qie_prefill_batch(self.h, seq0, n, flat.ctypes.data_as(C.POINTER(C.c_int32)), length,
                                              C.byref(sc), out), "qie_prefill_batch")
        return list(out)

    def decode_step(self, sampling: Sampling = GREEDY) -> List[int]:
        out = (C.c_int32 * self.B)()
        sc = sampling.to_c()
        _lib.check(self.lib.qie_decode_step(self.h, C.byref(sc), out), "qie_decode_step")
        return list(out)

    def decode(self, n_steps: int, sampling: Sampling = GREEDY, want_ids: bool = True) -> Optional[np.ndarray]:
        out = np.zeros((max(n_steps, 1), self.B), dtype=np.int32)
        sc = sampling.to_c()
        ptr = out.ctypes.data_as(C.POINTER(C.c_int32)) if want_ids else None
        _lib.check(self.lib.qie_decode(self.h, n_steps, C.byref(sc), ptr), "qie_decode")
        return out[:n_steps] if want_ids else None

    def logits(self) -> np.ndarray:
        out = np.zeros((self.B, self.e.spec.vocab), dtype=np.uint16)
        _lib.check(self.lib.qie_batch_logits(self.h, out.ctypes.data), "qie_batch_logits")
        return out

    def positions(self) -> np.ndarray:
        out = np.zeros(self.B, dtype=np.int32)
        _lib.check(self.lib.qie_batch_positions(self.h, out.ctypes.data_as(C.POINTER(C.c_int32))),
                   "qie_batch_positions")
        return out

    def history(self, seq: int, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.int32)
        _lib.check(self.lib.qie_batch_history(self.h, seq, out.ctypes.data_as(C.POINTER(C.c_int32)), n),
                   "qie_batch_history")
        return out

    def set_position(self, seq: int, pos: int, token: int) -> None:
        _lib.check(self.lib.qie_batch_set_position(self.h, seq, pos, token), "qie_batch_set_position")

    def release(self, seq: int) -> None:
        """End sequence `seq`: its KV pages return to the pool; the slot idles until the next prefill."""
        _lib.check(self.lib.qie_batch_release(self.h, seq), "qie_batch_release")

    def page_stats(self):
        """(free pages, pages held per slot, page_tokens); zeros for a contiguous batch."""
        free, pt = C.c_int32(), C.c_int32()
        per = np.zeros(self.B, dtype=np.int32)
        _lib.check(self.lib.qie_batch_page_stats(self.h, C.byref(free), per.ctypes.data_as(C.POINTER(C.c_int32)),
                                                 C.byref(pt)), "qie_batch_page_stats")
        return free.value, per, pt.value

    def block_table(self, seq: int, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.int32)
        _lib.check(self.lib.qie_batch_block_table(self.h, seq, out.ctypes.data_as(C.POINTER(C.c_int32)), n),
                   "qie_batch_block_table")
        return out

    def reserve(self, seq: int, n_tokens: int) -> None:
        """Operator tier: make `seq` live and hold KV pages for positions [0, n_tokens)."""
        _lib.check(self.lib.qie_batch_reserve(self.h, seq, n_tokens), "qie_batch_reserve")

    def kv_cache(self, seq: int) -> _lib.KvCacheC:
        """KV descriptor of slot `seq` (kernels address it as sequence 0)."""
        c = _lib.KvCacheC()
        _lib.check(self.lib.qie_batch_kv_cache(self.h, seq, C.byref(c)), "qie_batch_kv_cache")
        return c

    def kv_rows(self, seq: int, layer: int, n: int):
        """Host copy of the cached K and V rows [n_kv_heads][n][head_dim] (bf16 bits) of
        positions [0, n) of `seq` at `layer` (diagnostics / tests)."""
        c = self.kv_cache(seq)
        hd, nkv, L = c.head_dim, c.n_kv_heads, c.n_layers
        out = [np.zeros((nkv, n, hd), np.uint16), np.zeros((nkv, n, hd), np.uint16)]
        if c.block_table:
            T = c.page_tokens
            pages = self.block_table(seq, (n + T - 1) // T)
            runs = [(t0, min(n, t0 + T), int(pages[t0 // T]) * c.seq_stride, T) for t0 in range(0, n, T)]
        else:
            runs = [(0, n, 0, c.max_ctx)]
        for which, base in enumerate((c.k, c.v)):
            for t0, t1, off, run in runs:
                for g in range(nkv):
                    src = base + 2 * (off + ((layer * nkv + g) * run + (t0 % run if c.block_table else t0)) * hd)
                    buf = np.zeros((t1 - t0, hd), np.uint16)
                    _lib.check(self.lib.qie_memcpy_d2h(buf.ctypes.data, src, buf.nbytes), "kv_rows")
                    out[which][g, t0:t1] = buf
        return out

    def debug_step(self, sampling: Sampling = GREEDY):
        """One eager decode step; returns (ids, residual snapshots bf16 [2L + 1][B][H]):
        slot 0 the input row, 2l + 1 after layer l's attention block, 2l + 2 after its MLP."""
        L, H = self.e.spec.n_layers, self.e.spec.hidden
        xs = np.zeros((2 * L + 1, self.B, H), np.uint16)
        out = (C.c_int32 * self.B)()
        sc = sampling.to_c()
        _lib.check(self.lib.qie_batch_debug_step(self.h, C.byref(sc), out, xs.ctypes.data), "qie_batch_debug_step")
        return list(out), xs

    def set_decode_mode(self, mode: int) -> None:
        """0: five launches per layer; 1: the persistent layer stack (qie_batch_set_decode_mode)."""
        _lib.check(self.lib.qie_batch_set_decode_mode(self.h, mode), "qie_batch_set_decode_mode")

    @property
    def decode_mode(self) -> int:
        return int(self.lib.qie_batch_decode_mode(self.h))

    def time_kernel(self, which: int = 0, iters: int = 20):
        us, by = C.c_double(), C.c_double()
        _lib.check(self.lib.qie_batch_time_kernel(self.h, which, iters, C.byref(us), C.byref(by)),
                   "qie_batch_time_kernel")
        return us.value, by.value

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.qie_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
