"""Helpers for GPU tests.  Device memory comes from libqie (qie_malloc & co): a process
must not host two HIP runtimes, and the PyTorch wheel ships its own (ROCm 7.0) while
libqie links /opt/rocm (7.2) — so torch.cuda is never touched in-process."""
import ctypes as C

import numpy as np

from qwen_inference_engine_amd import _lib


def L():
    return _lib.load()


def check(rc, what=""):
    _lib.check(rc, what)


class DBuf:
    """A device allocation with a numpy dtype/shape (freed with the object)."""

    def __init__(self, shape, dtype):
        self.shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        check(L().qie_malloc(C.byref(p), self.nbytes), "qie_malloc")
        self.ptr = p.value

    def upload(self, a: np.ndarray) -> "DBuf":
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes
        check(L().qie_memcpy_h2d(self.ptr, a.ctypes.data, self.nbytes), "h2d")
        return self

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        check(L().qie_memcpy_d2h(out.ctypes.data, self.ptr, self.nbytes), "d2h")
        return out

    def data_ptr(self) -> int:
        return self.ptr

    def __del__(self):
        try:
            if self.ptr:
                L().qie_free(self.ptr)
        except Exception:
            pass


# Every buffer made by dev()/zeros() stays alive until release_all() (called after each
# test): `p(dev(x))` would otherwise free the allocation before the kernel runs and let
# the next allocation reuse its address.
_LIVE = []


def release_all():
    _LIVE.clear()


def dev(a: np.ndarray) -> DBuf:
    a = np.ascontiguousarray(a)
    b = DBuf(a.shape, a.dtype).upload(a)
    _LIVE.append(b)
    return b


def zeros(shape, dtype=np.uint16) -> DBuf:
    b = DBuf(shape, dtype)
    check(L().qie_memset(b.ptr, 0, b.nbytes), "memset")
    _LIVE.append(b)
    return b


def zeros_bf16(*shape) -> DBuf:
    return zeros(shape, np.uint16)


def zeros_bytes(n) -> DBuf:
    return zeros((max(int(n), 16),), np.uint8)


def host_bf16(t: DBuf) -> np.ndarray:
    return t.numpy().view(np.uint16)


def host(t: DBuf) -> np.ndarray:
    return t.numpy()


def to_bf16(a: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bits, round to nearest even (finite values)."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def stream() -> int:
    """A new non-blocking stream (qie_stream_create), kept alive with the test's buffers."""
    import ctypes as C
    h = C.c_void_p()
    check(L().qie_stream_create(C.byref(h)), "stream")
    _LIVE.append(_Stream(h.value))
    return h.value


class _Stream:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            L().qie_stream_destroy(self.h)
        except Exception:
            pass


def p(t) -> int:
    return None if t is None else t.ptr


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


def assert_sum_close(got, want, abs_scale, rel=1e-5, ulps=1, what=""):
    """|got - want| <= max(ulps bf16 ulps of want, rel * sum|a*w|) element-wise."""
    g, w = bf(got).astype(np.float64), bf(want).astype(np.float64)
    ulp = ulps * np.maximum(np.abs(w), 1e-30) * 2.0 ** -7
    tol = np.maximum(ulp, rel * abs_scale)
    bad = np.abs(g - w) > tol
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} outside tolerance; worst " \
        f"{np.abs(g - w)[bad].max() if bad.any() else 0}"
