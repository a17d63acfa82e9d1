"""CPU: the C-ABI library loads, exports every symbol include/qie/*.h declares, and its
host-side pieces (synthetic generator, weights.bin writer/loader index) behave."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, rng

from qwen_inference_engine_amd import _lib, weights as W, spec as S

HEADERS = [os.path.join(ROOT, "include", "qie", h) for h in ("qie_ops.h", "qie_engine.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(qie_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol(qlib):
    names = declared_functions()
    assert len(names) >= 40
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = sorted(n for n in names if n not in exported)
    assert not missing, missing
    # the Python binding covers every declared function with an explicit signature
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert names <= bound, sorted(names - bound)


def test_built_libraries_leave_no_kernel_undefined():
    """Every built libqie (release and the development build, when present) defines all of
    its own qie:: symbols.  A device-only builtin reached by the host pass can drop a
    kernel's launch stub without a compile error: the library then links, but fails to load
    (undefined symbol) on the GPU box."""
    libs = [_lib.LIB_PATH] + [p for p in [os.path.join(ROOT, "qwen_inference_engine_amd", "lib", "dev", "libqie.so")]
                              if os.path.exists(p)]
    for path in libs:
        out = subprocess.check_output(["nm", "-D", "--undefined-only", path]).decode()
        undef = [l.split()[-1] for l in out.splitlines() if "_ZN3qie" in l or " qie_" in l]
        assert not undef, (path, undef[:5])


def test_abi_version_and_error_channel(qlib):
    assert qlib.qie_abi_version() == 1
    # invalid call reports through qie_last_error without touching a GPU
    rc = qlib.qie_embedding(None, None, None, 1, 8, None)
    assert rc == -22
    assert b"qie_embedding" in qlib.qie_last_error()


def test_no_oracle_or_cpu_fallback_in_product():
    """The product package never imports the oracle and libqie never links it."""
    pkg = os.path.join(ROOT, "qwen_inference_engine_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".hpp")):
                t = open(os.path.join(dp, f)).read()
                assert "import oracle" not in t and "liboracle" not in t and "or_forward" not in t, f
    out = subprocess.check_output(["ldd", _lib.LIB_PATH]).decode()
    assert "oracle" not in out


def _np_splitmix(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def test_synthetic_generator_matches_its_definition(qlib, oracle):
    """qie_synthetic_fill_host == the documented formula (qie_ops.h), restated in numpy."""
    name, seed, scale, off = "model.layers.3.mlp.up_proj.weight", 7, 0.0346, 0.0
    n = 4099 * 2
    got = W.synthetic_tensor(name, "mlp.up_proj.weight", n, W.SynthParams(seed=seed))
    with np.errstate(over="ignore"):
        tid = np.uint64(W.tensor_id(name))
        base = _np_splitmix(np.array([np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) ^ (tid << np.uint64(32))],
                                     dtype=np.uint64))[0]
        r = _np_splitmix(base + np.arange(n, dtype=np.uint64))
    u = ((r >> np.uint64(40)).astype(np.int64) - 8388608).astype(np.float32) * np.float32(1.0 / 8388608.0)
    want = oracle.f32_to_bf16(np.float32(off) + u * np.float32(scale))
    assert np.array_equal(got, want)
    assert W.tensor_id(name) == qlib.qie_tensor_id(name.encode())


def test_weights_bin_roundtrip(tmp_path):
    spec = S.tiny(n_layers=3, tie=True)
    hw = W.HostWeights.synthetic(spec, W.SynthParams(seed=3, norm_scale=0.2))
    idx = hw.write_weights_bin(str(tmp_path / "weights.bin"), str(tmp_path / "meta_data.txt"))
    assert [t.tensor_name for t in idx] == [t.tensor_name for t in W.synthetic_index(spec)]
    back = W.HostWeights.from_weights_bin(spec, str(tmp_path / "weights.bin"), str(tmp_path / "meta_data.txt"))
    for k, v in hw.tensors.items():
        assert np.array_equal(back.tensors[k], v), k


def test_convert_safetensors(tmp_path):
    """safetensors shards -> weights.bin + meta_data.txt (reference parser semantics)."""
    import json
    import struct
    r = rng(9)
    shards = []
    expect = {}
    for si, keys in enumerate([["model.b.weight", "lm_head.weight", "model.a.weight"],
                               ["model.layers.1.x.weight", "model.layers.0.x.weight", "other.bias"]]):
        hdr, blobs, off = {"__metadata__": {"format": "pt"}}, [], 0
        for k in keys:
            a = r.integers(0, 65535, (3, 5), dtype=np.uint16)
            expect[k] = a
            hdr[k] = {"dtype": "BF16", "shape": [3, 5], "data_offsets": [off, off + a.nbytes]}
            blobs.append(a.tobytes())
            off += a.nbytes
        hb = json.dumps(hdr).encode()
        p = tmp_path / f"model-{si}.safetensors"
        p.write_bytes(struct.pack("<Q", len(hb)) + hb + b"".join(blobs))
        shards.append(str(p))
    idx = W.convert_safetensors(shards, str(tmp_path / "w.bin"), str(tmp_path / "m.txt"))
    assert [t.tensor_name for t in idx] == ["lm_head.weight", "model.a.weight", "model.b.weight",
                                            "model.layers.0.x.weight", "model.layers.1.x.weight"]
    assert [t.short_name for t in idx] == ["logits", "a.weight", "b.weight", "x.weight", "x.weight"]
    assert [t.layer_index for t in idx] == [-1, -1, -1, 0, 1]
    data = np.fromfile(tmp_path / "w.bin", dtype=np.uint16)
    for t in idx:
        assert np.array_equal(data[t.data_offsets[0] // 2:t.data_offsets[1] // 2].reshape(3, 5), expect[t.tensor_name])


class _FakeBatch:
    """Records the engine calls the ContinuousBatcher makes (host logic only)."""

    def __init__(self, slots, max_ctx, n_pages):
        self.B, self.max_ctx, self.free = slots, max_ctx, n_pages - 1
        self.calls = []

    def page_stats(self):
        return self.free, [0] * self.B, 128

    def prefill(self, seq, ids, sampling=None):
        self.calls.append(("prefill", seq, len(ids)))
        return 1000 + seq

    def prefill_batch(self, seq0, prompts, sampling=None):
        assert len({len(p) for p in prompts}) == 1
        self.calls.append(("prefill_batch", seq0, len(prompts)))
        return [1000 + seq0 + z for z in range(len(prompts))]

    def decode_step(self, sampling=None):
        self.calls.append(("decode",))
        return [2000 + i for i in range(self.B)]

    def release(self, seq):
        self.calls.append(("release", seq))


class _FakeEngine:
    def __init__(self, fb):
        self.fb = fb

    def batch(self, slots, max_ctx, page_tokens=None, n_pages=0):
        return self.fb


def test_batcher_groups_equal_length_admissions():
    """Requests admitted in one step with equal prompt lengths into consecutive slots go
    through one qie_prefill_batch call; a length change or a slot gap starts a new run;
    first tokens are emitted in admission order."""
    from qwen_inference_engine_amd.scheduler import ContinuousBatcher, prefill_runs, Request
    fb = _FakeBatch(6, 512, 64)
    cb = ContinuousBatcher(_FakeEngine(fb), slots=6, max_ctx=512)
    lens = [16, 16, 16, 9, 16, 16]
    rids = [cb.submit(list(range(n)), 4) for n in lens]
    out = cb.step()
    assert fb.calls[:3] == [("prefill_batch", 0, 3), ("prefill", 3, 9), ("prefill_batch", 4, 2)]
    assert [rid for rid, _ in out[:6]] == rids
    assert [t for _, t in out[:6]] == [1000 + s for s in range(6)]
    # a gap: slots 0 and 2 free, slot 1 busy -> two single runs even with equal lengths
    rs = [Request(i, [0] * 8, 1, slot=s) for i, s in enumerate([0, 2, 3])]
    assert [[r.slot for r in run] for run in prefill_runs(rs)] == [[0], [2, 3]]
    assert prefill_runs([]) == []


@pytest.mark.parametrize("fp8,tiny_widths", [(False, False), (True, True)])
def test_prefill_fp8_refused_where_it_cannot_hold(qlib, fp8, tiny_widths):
    """qie_engine_create refuses prefill_fp8 without fp8 weights, or when a projection width
    (hidden, this rank's q width, ffn / tp) is not a multiple of the fp8 MFMA's 128-k block,
    instead of silently running the bf16-activation model.  The check precedes
    every HIP call, so it runs without a GPU."""
    spec = S.tiny(n_layers=1, hidden=192, ffn=320) if tiny_widths else S.QWEN2_7B
    if tiny_widths:
        assert spec.hidden % 128 or spec.ffn % 128 or (spec.n_heads * spec.head_dim) % 128
    sc = spec.to_c()
    opts = _lib.EngineOptsC()
    opts.max_ctx, opts.use_graph, opts.tp_size = 64, 0, 1
    opts.weight_fp8, opts.prefill_fp8 = int(fp8), 1
    h = C.c_void_p()
    rc = qlib.qie_engine_create(C.byref(sc), C.byref(opts), C.byref(h))
    assert rc == -22 and not h.value
    assert b"prefill_fp8" in qlib.qie_last_error()
