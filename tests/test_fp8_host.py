"""Host fp8 quantiser (libqie's qie_quantize_fp8_host, the bit-exact twin of the device
one): e4m3fn table, exact bf16 dequantisation, round-to-nearest-even, power-of-two
row scales and saturation — no GPU needed."""
import numpy as np

from qwen_inference_engine_amd import weights as W


def _bf16(a):
    return (np.ascontiguousarray(a, np.float32).view(np.uint32) >> 16).astype(np.uint16)


def test_e4m3_table():
    t = W.e4m3_table()
    assert t[0x7E] == 448.0 and t[0x01] == 2.0 ** -9 and t[0x08] == 2.0 ** -6 and t[0x38] == 1.0
    finite = t[~np.isnan(t)]
    assert len(finite) == 254 and np.all(np.diff(np.sort(finite[finite > 0])) > 0)


def test_quantize_roundtrip_properties():
    rng = np.random.default_rng(0)
    rows = [rng.standard_normal(256) * s for s in (1.0, 1e-3, 100.0, 3e4)] + [np.zeros(256)]
    w = _bf16(np.stack(rows))
    codes, scales = W.quantize_fp8(w)
    for s in scales:                                   # powers of two
        m, e = np.frexp(s)
        assert m == 0.5
    assert scales[-1] == 1.0 and not codes[-1].any()   # all-zero row
    t = W.e4m3_table()
    f = (w.astype(np.uint32) << 16).view(np.float32)
    for r in range(4):
        v = f[r] / scales[r]
        assert np.abs(v).max() <= 448.0 and np.abs(v).max() > 224.0   # smallest scale that fits
        q = t[codes[r]]
        # nearest representable (ties to even are exact midpoints: allow equality)
        grid = np.sort(t[~np.isnan(t)])
        nearest = grid[np.abs(grid[None, :] - v[:, None]).argmin(axis=1)]
        assert np.all(np.abs(q - v) <= np.abs(nearest - v) + 0.0)
    dq = W.dequantize_fp8(codes, scales)               # exact bf16 (asserts inside)
    assert dq.dtype == np.uint16


def test_quantize_ties_to_even():
    # 1 + 1/16 lies halfway between 1.0 (mantissa 0, even) and 1.125 (mantissa 1)
    w = _bf16(np.array([[448.0, 1.0625, 1.1875, -1.0625] + [0.0] * 12], np.float32))
    codes, scales = W.quantize_fp8(w)
    assert scales[0] == 1.0
    t = W.e4m3_table()
    assert list(t[codes[0, :4]]) == [448.0, 1.0, 1.25, -1.0]


def test_oracle_activation_quantiser_equals_libqie_row_quantiser(oracle):
    """The oracle's fp8-activation restatement (or_quant_rows_fp8: e4m3 rounding from the
    value set, ties to the even code) and libqie's host row quantiser (e4m3_encode,
    e4m3_row_scale) agree on every row — scales and dequantised values, including rows
    with ties, subnormal codes and zeros."""
    rng = np.random.default_rng(7)
    rows = [rng.standard_normal(512) * s for s in (1.0, 3e-3, 77.0, 2.5e4, 1e-30)]
    ties = np.array([t * 2.0 ** k for k in range(-9, 9) for t in (1.0625, 1.1875, 0.0068359375, 447.0, 448.0)])
    rows.append(np.resize(np.concatenate([ties, -ties]), 512))
    rows.append(np.zeros(512))
    w = _bf16(np.stack(rows))
    codes, scales = W.quantize_fp8(w)
    dq_lib = W.dequantize_fp8(codes, scales)
    dq_or, e = oracle.quant_rows_fp8(w)
    assert np.array_equal(2.0 ** e.astype(np.float64), scales.astype(np.float64))
    assert np.array_equal(dq_or, dq_lib)
