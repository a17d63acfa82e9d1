#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the reference's OWN files and code.

Container-only (needs /root/reference and oracle/_ref/, neither of which is on the GPU
box: oracle/_ref/ is listed in .gpurunignore).  The fixtures are data — inputs and
expected outputs — never reference source:

* rope_ref.npz     cos/sin tables produced by the reference's precompute_cos_sin
                   (layers/src/include.cpp) — built beforehand by ``make -C oracle ref``
                   into oracle/_ref/libref_rope.so and executed here — for head_dim 64
                   and 128 at positions up to the reference CONTEXT_SIZE (32786,
                   iengine.cuh:19).
* qwen3_14b_index.json   the reference's model_files/meta_data.txt (443 tensors) as
                   JSON: the re-based weights.bin layout its parser produced.
* qwen3_14b_shards.json  the raw per-shard safetensors entries of
                   model_files/meta_data_nooffsetsadjustment.txt (a shard starts where
                   the sorted key order descends; lm_head.weight, which that older dump omits,
                   is placed in the shard where meta_data.txt shows it, with its size).

Usage:  make -C oracle ref && python tools/make_golden.py [--ref /root/reference]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qwen_inference_engine_amd.weights import parse_meta  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_rope.so")
CONTEXT_SIZE = 32786


def rope_fixture():
    if not os.path.exists(REF_LIB):
        raise SystemExit(f"{REF_LIB} missing: run `make -C oracle ref` first")
    lib = C.CDLL(REF_LIB)
    f = getattr(lib, "_Z18precompute_cos_sinPfS_ii")   # precompute_cos_sin(float*, float*, int, int)
    f.restype = None
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    pos = np.unique(np.concatenate([np.arange(0, 1024), np.arange(1024, CONTEXT_SIZE, 61),
                                    [CONTEXT_SIZE - 1]])).astype(np.int32)
    out = {"positions": pos}
    for hd in (64, 128):
        c = np.zeros(CONTEXT_SIZE * hd // 2, np.float32)
        s = np.zeros_like(c)
        f(c.ctypes.data, s.ctypes.data, CONTEXT_SIZE, hd)
        out[f"cos_hd{hd}"] = c.reshape(CONTEXT_SIZE, hd // 2)[pos]
        out[f"sin_hd{hd}"] = s.reshape(CONTEXT_SIZE, hd // 2)[pos]
    np.savez_compressed(os.path.join(GOLD, "rope_ref.npz"), **out)


def index_fixtures(ref):
    with open(os.path.join(ref, "model_files", "meta_data.txt")) as f:
        idx = parse_meta(f.read())
    with open(os.path.join(GOLD, "qwen3_14b_index.json"), "w") as f:
        json.dump([[t.tensor_name, t.layer_index, t.short_name, t.shape, t.data_offsets] for t in idx], f)

    with open(os.path.join(ref, "model_files", "meta_data_nooffsetsadjustment.txt")) as f:
        raw = parse_meta(f.read())
    # The dump lists shards in order, each shard's keys sorted: a shard starts where the
    # key order descends.
    shards, cur = [], []
    for t in raw:
        if cur and t.tensor_name < cur[-1][0]:
            shards.append(cur)
            cur = []
        cur.append([t.tensor_name, t.shape, t.data_offsets])
    shards.append(cur)
    # lm_head: sorted first in its shard, so meta_data.txt lists it right before the
    # first model.* tensor of that shard.
    names = [t.tensor_name for t in idx]
    li = names.index("lm_head.weight")
    nxt = names[li + 1]
    lm = idx[li]
    for sh in shards:
        if sorted(e[0] for e in sh)[0] == nxt:
            end = max(e[2][1] for e in sh)
            sh.insert(0, ["lm_head.weight", lm.shape, [end, end + lm.data_offsets[1] - lm.data_offsets[0]]])
            break
    else:
        raise SystemExit("could not place lm_head.weight")
    with open(os.path.join(GOLD, "qwen3_14b_shards.json"), "w") as f:
        json.dump(shards, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    rope_fixture()
    index_fixtures(a.ref)
    print("wrote", sorted(os.listdir(GOLD)))


if __name__ == "__main__":
    main()
