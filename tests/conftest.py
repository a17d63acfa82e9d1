import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels in libqie.so)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def qlib():
    from qwen_inference_engine_amd import _lib
    return _lib.load()


@pytest.fixture(autouse=True)
def _release_device_buffers():
    yield
    import gpu_util
    gpu_util.release_all()


def rng(seed=0):
    return np.random.default_rng(seed)


def pytest_sessionfinish(session, exitstatus):
    """On the GPU box, keep every end-to-end parity step's (engine error, bar) as evidence."""
    import json
    try:
        import parity
    except Exception:
        return
    if parity.REPORT and os.environ.get("GRAFT_REPO_ROOT"):
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_report.json"), "w") as f:
            json.dump([{"step": w, "norm_rel": r, "bar": b} for w, r, b in parity.REPORT], f, indent=0)
