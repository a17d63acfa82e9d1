"""Debug dump for the fp8 batched-decode kernel: SwiGLU M=8 K=896 with / without the fused
norm, gate-only (STORE) too; writes gpurun_out/dbg_dec8.npz."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import gpu_util as G
from conftest import rng
from test_gpu_ops import _linear, rand_bf16
from test_gpu_fp8 import _fp8_dev
from qwen_inference_engine_amd import _lib
import oracle
oracle.lib()
qlib = _lib.load()
M, K, I = 8, 896, 640
x = rand_bf16(oracle, (M, K), seed=M + K)
nw = oracle.f32_to_bf16((1 + 0.2 * rng(12).standard_normal(K)).astype(np.float32))
xn = oracle.rmsnorm(x, nw, 1e-4, "ref")
(dg, qg), (du, qu) = _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=7)), \
    _fp8_dev(qlib, rand_bf16(oracle, (I, K), 0.08, seed=8))
out = {"x": x, "nw": nw, "xn": xn, "qg": qg, "qu": qu}
for name, xin, nwin in (("fused", x, nw), ("pre", xn, None)):
    y = G.zeros_bf16(M, I)
    _linear(qlib, G.dev(xin), [(dg, I), (du, I)], [], M, K, I, y, _lib.QIE_EPI_SWIGLU,
            norm_w=G.dev(nwin) if nwin is not None else None, eps=1e-4, num=0, flags=_lib.QIE_LINEAR_FP8)
    out["swiglu_" + name] = G.host_bf16(y)
    yg = G.zeros_bf16(M, I)
    _linear(qlib, G.dev(xin), [(dg, I)], [], M, K, I, yg, _lib.QIE_EPI_STORE,
            norm_w=G.dev(nwin) if nwin is not None else None, eps=1e-4, num=0, flags=_lib.QIE_LINEAR_FP8)
    out["gate_" + name] = G.host_bf16(yg)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dbg_dec8.npz"), **out)
print("saved")
# identity weights: the STORE output is the kernel's normalised activations themselves
eye = oracle.f32_to_bf16(np.eye(K, dtype=np.float32))
de, _ = _fp8_dev(qlib, eye)
ye = G.zeros_bf16(M, K)
_linear(qlib, G.dev(x), [(de, K)], [], M, K, K, ye, _lib.QIE_EPI_STORE, norm_w=G.dev(nw), eps=1e-4, num=0,
        flags=_lib.QIE_LINEAR_FP8)
out["xn_fused"] = G.host_bf16(ye)
np.savez(os.path.join(ROOT, "gpurun_out", "dbg_dec8.npz"), **out)
print("saved eye")
