"""ctypes binding of libqie.so — the MI355X (gfx950) HIP engine's C ABI.

The declarations mirror include/qie/qie_types.h, qie_ops.h and qie_engine.h.
The library is built in-tree (qwen_inference_engine_amd/lib/libqie.so) by
``__graft_entry__.build()`` / ``make -C qwen_inference_engine_amd/csrc``.
There is deliberately no CPU fallback: if the library cannot be loaded, every
product entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QIE_LIB") or os.path.join(_HERE, "lib", "libqie.so")   # QIE_LIB: dev A/B builds

QIE_NUMERICS_REF = 0
QIE_NUMERICS_HF = 1
QIE_EPI_STORE = 0
QIE_EPI_RESIDUAL = 1
QIE_EPI_SWIGLU = 2
QIE_EPI_F32 = 3
QIE_LINEAR_FP8 = 1
QIE_LINEAR_TILE256 = 2
QIE_LINEAR_TILE128 = 4
QIE_LINEAR_STREAMK = 8
QIE_LINEAR_FP8_T16 = 16
QIE_LINEAR_ACT_FP8 = 32
QIE_ATTN_PREROPED = 0x100   # qie_attention_decode numerics flag: q / new k arrive rotated
QIE_COMM_ID_BYTES = 128
QIE_COMM_PEER_HANDLE_BYTES = 128


class ModelSpecC(C.Structure):
    _fields_ = [
        ("n_layers", C.c_int32), ("hidden", C.c_int32), ("n_heads", C.c_int32),
        ("n_kv_heads", C.c_int32), ("head_dim", C.c_int32), ("ffn", C.c_int32),
        ("vocab", C.c_int32), ("tie_embeddings", C.c_int32), ("qkv_bias", C.c_int32),
        ("qk_norm", C.c_int32), ("rms_eps", C.c_float), ("rope_theta", C.c_float),
        ("numerics", C.c_int32), ("reserved", C.c_int32 * 7),
    ]


class LayerWeightsC(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "attn_norm", "wq", "wk", "wv", "bq", "bk", "bv", "q_norm", "k_norm", "wo",
        "ffn_norm", "w_gate", "w_up", "w_down")]


class ModelWeightsC(C.Structure):
    _fields_ = [("embed", C.c_void_p), ("final_norm", C.c_void_p), ("lm_head", C.c_void_p),
                ("n_layers", C.c_int32), ("layers", C.POINTER(LayerWeightsC))]


class SamplingC(C.Structure):
    _fields_ = [("top_k", C.c_int32), ("temperature", C.c_float), ("top_p", C.c_float),
                ("seed", C.c_uint64)]


class LinearArgsC(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("ldx", C.c_int64), ("w", C.c_void_p * 3), ("bias", C.c_void_p * 3),
        ("seg_rows", C.c_int64 * 3), ("M", C.c_int64), ("K", C.c_int64), ("N", C.c_int64),
        ("y", C.c_void_p), ("ldy", C.c_int64), ("epilogue", C.c_int32), ("numerics", C.c_int32),
        ("norm_w", C.c_void_p), ("norm_eps", C.c_float), ("flags", C.c_int32),
        ("argmax_keys", C.c_void_p), ("key_col0", C.c_int64), ("x_exps", C.c_void_p),
    ]


class KvCacheC(C.Structure):
    _fields_ = [("k", C.c_void_p), ("v", C.c_void_p), ("seq_stride", C.c_int64),
                ("n_layers", C.c_int32), ("n_kv_heads", C.c_int32), ("head_dim", C.c_int32),
                ("max_ctx", C.c_int32), ("block_table", C.c_void_p), ("page_tokens", C.c_int32),
                ("max_pages", C.c_int32)]


class EngineOptsC(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_ctx", C.c_int32), ("use_graph", C.c_int32),
                ("tp_rank", C.c_int32), ("tp_size", C.c_int32), ("tp_comm", C.c_void_p),
                ("weight_fp8", C.c_int32), ("comm_always", C.c_int32), ("prefill_fp8", C.c_int32),
                ("reserved", C.c_int32 * 5)]


# (name, restype, argtypes) — every symbol the public headers declare.
_P = C.c_void_p
_I32, _I64, _U32, _U64, _F = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
_PI32 = C.POINTER(C.c_int32)
_PI64 = C.POINTER(C.c_int64)
_PF = C.POINTER(C.c_float)
_PD = C.POINTER(C.c_double)
_PCC = C.POINTER(C.c_char_p)
SIGNATURES = [
    # qie_ops.h
    ("qie_last_error", C.c_char_p, []),
    ("qie_abi_version", C.c_int, []),
    ("qie_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("qie_set_device", C.c_int, [C.c_int]),
    ("qie_malloc", C.c_int, [C.POINTER(_P), _I64]),
    ("qie_free", C.c_int, [_P]),
    ("qie_memcpy_h2d", C.c_int, [_P, _P, _I64]),
    ("qie_memcpy_d2h", C.c_int, [_P, _P, _I64]),
    ("qie_memset", C.c_int, [_P, C.c_int, _I64]),
    ("qie_synchronize", C.c_int, []),
    ("qie_stream_create", C.c_int, [C.POINTER(_P)]),
    ("qie_stream_synchronize", C.c_int, [_P]),
    ("qie_stream_destroy", C.c_int, [_P]),
    ("qie_rope_table_host", C.c_int, [_PF, _PF, _I32, _I32, _F, _I32]),
    ("qie_embedding", C.c_int, [_P, _P, _P, _I64, _I64, _P]),
    ("qie_rmsnorm", C.c_int, [_P, _P, _P, _I64, _I64, _F, _I32, _P]),
    ("qie_linear", C.c_int, [C.POINTER(LinearArgsC), _P]),
    ("qie_qkv_post", C.c_int, [_P, _I64, _P, _I32, _P, _P, _P, _P, _I32, C.POINTER(KvCacheC),
                               _I32, _F, _I32, _P, _P]),
    ("qie_attention_workspace_bytes", C.c_int64, [_I64, _I32, _I32, _I32]),
    ("qie_attention", C.c_int, [_P, _I64, _P, _I32, C.POINTER(KvCacheC), _I32, _I32, _P, _P, _P]),
    ("qie_attention_decode_workspace_bytes", C.c_int64, [_I64, _I32, _I32, _I32, _I32]),
    ("qie_attention_decode", C.c_int, [_P, _I64, _P, _P, _P, _P, _P, _I32, C.POINTER(KvCacheC), _I32, _F, _I32,
                                       _P, _P, _P]),
    ("qie_debug_tr16_probe", C.c_int, [_P]),
    ("qie_qknorm", C.c_int, [_P, _I64, _I64, _I32, _I32, _P, _F, _I32, _P]),
    ("qie_rope", C.c_int, [_P, _I64, _I64, _I32, _I32, _P, _I32, _P, _P, _I32, _P]),
    ("qie_kv_write", C.c_int, [_P, _P, _I64, _I64, _I32, C.POINTER(KvCacheC), _I32, _I32, _P]),
    ("qie_silu", C.c_int, [_P, _I64, _P]),
    ("qie_mul", C.c_int, [_P, _P, _P, _I64, _P]),
    ("qie_memcpy_d2d", C.c_int, [_P, _P, _I64, _P]),
    ("qie_silu_mul", C.c_int, [_P, _P, _P, _I64, _P]),
    ("qie_residual_add", C.c_int, [_P, _P, _I64, _P]),
    ("qie_residual_add_f32", C.c_int, [_P, _P, _I64, _P]),
    ("qie_sample_workspace_bytes", C.c_int64, [_I64, _I64]),
    ("qie_sample", C.c_int, [_P, _I64, _I64, _I64, C.POINTER(SamplingC), _P, _P, _P, _P]),
    ("qie_keys_to_ids", C.c_int, [_P, _I64, _P, _P]),
    ("qie_tensor_id", C.c_uint32, [C.c_char_p]),
    ("qie_synthetic_fill", C.c_int, [_P, _I64, _U32, _U64, _F, _F, _P]),
    ("qie_synthetic_fill_host", C.c_int, [_P, _I64, _U32, _U64, _F, _F]),
    ("qie_synthetic_fill_slice", C.c_int, [_P, _I64, _I64, _I64, _I64, _I64, _U32, _U64, _F, _F, _P]),
    ("qie_scale_rows_pow2", C.c_int, [_P, _I64, _I64, _I64, _I64, _I32, _P]),
    ("qie_fp8_weight_bytes", C.c_int64, [_I64, _I64]),
    ("qie_quantize_fp8", C.c_int, [_P, _I64, _I64, _P, _P]),
    ("qie_quantize_rows_fp8", C.c_int, [_P, _I64, _I64, _I64, _P, _I64, _P, _P]),
    ("qie_quantize_fp8_host", C.c_int, [_P, _I64, _I64, _P]),
    ("qie_dequantize_fp8", C.c_int, [_P, _I64, _I64, _P, _P]),
    ("qie_fp8_tile16", C.c_int, [_P, _I64, _I64, _P, _P]),
    ("qie_debug_fp8_decode", C.c_int, [_P]),
    ("qie_debug_fp8_decode_bf16", C.c_int, [_P]),
    # qie_engine.h
    ("qie_comm_unique_id", C.c_int, [_P]),
    ("qie_comm_create_rccl", C.c_int, [_P, _I32, _I32, _I32, C.POINTER(_P)]),
    ("qie_comm_create_local", C.c_int, [_I32, C.POINTER(_P)]),
    ("qie_comm_create_peer", C.c_int, [_I32, _I32, _I32, C.POINTER(_P), _P]),
    ("qie_comm_peer_connect", C.c_int, [_P, _P]),
    ("qie_comm_create_peer_local", C.c_int, [_I32, C.POINTER(_P)]),
    ("qie_comm_peer_error", C.c_int, [_P, _PI32]),
    ("qie_comm_allreduce_residual_bf16", C.c_int, [_P, _P, _P, _I64, _P]),
    ("qie_comm_peer_set_mode", C.c_int, [_P, _I32, _I32]),
    ("qie_comm_time_exchange", C.c_int, [_P, _P, _P, _I64, _I32, _I32, _I32, _P, C.POINTER(C.c_float)]),
    ("qie_comm_rank", C.c_int, [_P, _PI32, _PI32]),
    ("qie_comm_allreduce_sum_f32", C.c_int, [_P, _P, _I64, _P]),
    ("qie_comm_allreduce_max_u64", C.c_int, [_P, _P, _I64, _P]),
    ("qie_comm_destroy", None, [_P]),
    ("qie_index_load_meta", C.c_int, [C.c_char_p, C.POINTER(_P)]),
    ("qie_index_synthetic", C.c_int, [C.POINTER(ModelSpecC), C.POINTER(_P)]),
    ("qie_index_count", C.c_int, [_P]),
    ("qie_index_get", C.c_int, [_P, C.c_int, _PCC, _PCC, _PI32, _PI64, _PI64, _PI32, _PI64]),
    ("qie_index_total_bytes", C.c_int64, [_P]),
    ("qie_index_write_meta", C.c_int, [_P, C.c_char_p]),
    ("qie_index_destroy", None, [_P]),
    ("qie_engine_create", C.c_int, [C.POINTER(ModelSpecC), C.POINTER(EngineOptsC), C.POINTER(_P)]),
    ("qie_engine_init_synthetic", C.c_int, [_P, _U64, _F, _F, _F]),
    ("qie_engine_load_weights_bin", C.c_int, [_P, C.c_char_p, C.c_char_p, _I64]),
    ("qie_engine_set_weights", C.c_int, [_P, C.POINTER(ModelWeightsC)]),
    ("qie_engine_weights", C.c_int, [_P, C.POINTER(ModelWeightsC), C.POINTER(C.POINTER(LayerWeightsC))]),
    ("qie_engine_spec", C.c_int, [_P, C.POINTER(ModelSpecC)]),
    ("qie_engine_stream", _P, [_P]),
    ("qie_engine_sync", C.c_int, [_P]),
    ("qie_engine_destroy", None, [_P]),
    ("qie_batch_create", C.c_int, [_P, _I32, _I32, C.POINTER(_P)]),
    ("qie_batch_destroy", None, [_P]),
    ("qie_batch_create_paged", C.c_int, [_P, _I32, _I32, _I32, _I32, C.POINTER(_P)]),
    ("qie_batch_release", C.c_int, [_P, _I32]),
    ("qie_batch_page_stats", C.c_int, [_P, _PI32, _PI32, _PI32]),
    ("qie_batch_block_table", C.c_int, [_P, _I32, _PI32, _I32]),
    ("qie_prefill", C.c_int, [_P, _I32, _PI32, _I32, C.POINTER(SamplingC), _PI32]),
    ("qie_prefill_batch", C.c_int, [_P, _I32, _I32, _PI32, _I32, C.POINTER(SamplingC), _PI32]),
    ("qie_decode_step", C.c_int, [_P, C.POINTER(SamplingC), _PI32]),
    ("qie_decode", C.c_int, [_P, _I32, C.POINTER(SamplingC), _PI32]),
    ("qie_batch_logits", C.c_int, [_P, _P]),
    ("qie_batch_positions", C.c_int, [_P, _PI32]),
    ("qie_batch_history", C.c_int, [_P, _I32, _PI32, _I32]),
    ("qie_batch_set_position", C.c_int, [_P, _I32, _I32, _I32]),
    ("qie_batch_dims", C.c_int, [_P, _PI32, _PI32]),
    ("qie_batch_set_decode_mode", C.c_int, [_P, _I32]),
    ("qie_batch_decode_mode", C.c_int, [_P]),
    ("qie_batch_pk_trace", C.c_int, [_P, _I32, _P, C.c_int64]),
    ("qie_batch_kv_cache", C.c_int, [_P, _I32, C.POINTER(KvCacheC)]),
    ("qie_batch_reserve", C.c_int, [_P, _I32, _I32]),
    ("qie_engine_arena", C.c_int, [_P, C.POINTER(_P), _PI64]),
    ("qie_engine_rope_tables", C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), _PI32]),
    ("qie_batch_time_kernel", C.c_int, [_P, _I32, _I32, _PD, _PD]),
    ("qie_batch_debug_step", C.c_int, [_P, _P, _PI32, _P]),
]

_lib = None


class QieError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libqie.so (raises if it is missing — no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise QieError(f"{path} not built; run __graft_entry__.build() or make -C "
                       f"qwen_inference_engine_amd/csrc")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = _lib.qie_last_error().decode() if _lib is not None else ""
        raise QieError(f"{what} failed (rc={rc}): {msg}")
