"""Helpers for GPU tests: torch is only device-memory plumbing; all compute is libqie."""
import ctypes as C

import numpy as np

from qwen_inference_engine_amd import _lib


def torch():
    import torch as T
    assert T.cuda.is_available(), "gpu test without a visible GPU"
    return T


def dev(a: np.ndarray):
    T = torch()
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        return T.from_numpy(a.view(np.int16).copy()).cuda()
    if a.dtype == np.uint64:
        return T.from_numpy(a.view(np.int64).copy()).cuda()
    return T.from_numpy(a.copy()).cuda()


def zeros_bf16(*shape):
    T = torch()
    return T.zeros(*shape, dtype=T.int16, device="cuda")


def host_bf16(t) -> np.ndarray:
    torch().cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def host(t) -> np.ndarray:
    torch().cuda.synchronize()
    return t.cpu().numpy()


def p(t) -> int:
    return t.data_ptr()


def bf(a):
    return (np.asarray(a, np.uint16).astype(np.uint32) << 16).view(np.float32)


def ulp_diff(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Distance in bf16 ulps between two bf16 arrays (sign-magnitude aware)."""
    def key(x):
        x = x.astype(np.int32)
        return np.where(x & 0x8000, -(x & 0x7FFF), x & 0x7FFF)
    return np.abs(key(a) - key(b))


def assert_bf16_close(got, want, max_ulp=1, min_exact=0.98, what=""):
    d = ulp_diff(np.asarray(got), np.asarray(want))
    exact = float((d == 0).mean())
    assert d.max() <= max_ulp and exact >= min_exact, \
        f"{what}: max ulp {d.max()}, exact fraction {exact:.4f}"


def assert_sum_close(got, want, abs_scale, rel=1e-5, what=""):
    """|got - want| <= max(1 bf16 ulp of want, rel * sum|a*w|) element-wise."""
    g, w = bf(got).astype(np.float64), bf(want).astype(np.float64)
    ulp = np.maximum(np.abs(w), 1e-30) * 2.0 ** -7
    tol = np.maximum(ulp, rel * abs_scale)
    bad = np.abs(g - w) > tol
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} outside tolerance; worst " \
        f"{np.abs(g - w)[bad].max() if bad.any() else 0}"


def check(rc, what=""):
    _lib.check(rc, what)
