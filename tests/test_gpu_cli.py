"""GPU: the native driver (qie_cli, the reference's `layers/engine` main replaced,
iengine.cu:226-481) over compat.hpp — prompt ids from a file, streamed ids, and the paged
KV cache give the same greedy tokens as the contiguous run."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "qwen_inference_engine_amd", "lib", "qie_cli")


def _run(*args):
    r = subprocess.run([CLI, "--model", "Qwen2-0.5B", "--synthetic", "5", "--greedy", "--gen", "140", *args],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _tokens(out):
    line = [l for l in out.splitlines() if l.startswith("tokens:")][0]
    return [int(t) for t in line.split()[1:]]


def test_cli_prompt_file_stream_and_paged(tmp_path):
    ids = [151643, 785, 4767, 315, 279, 3639, 4180, 374] * 3
    f = tmp_path / "ids.txt"
    f.write_text(" ".join(map(str, ids[:10])) + "\n" + ",".join(map(str, ids[10:])) + "\n")
    base = _tokens(_run("--prompt", ",".join(map(str, ids))))
    out = _run("--prompt-file", str(f), "--stream", "--page-tokens", "128")
    streamed = [int(l) for l in out.splitlines() if l.strip().isdigit()]
    assert _tokens(out) == base          # 24 + 140 tokens: crosses a 128-token page
    assert streamed == base
