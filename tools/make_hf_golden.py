#!/usr/bin/env python3
"""Generate tests/golden/hf_*.npz: the HF numerics mode's pin (SURVEY §8(c) "HF-mode second
oracle"; verdict r04 item 6).

The reference engine itself has no HF numerics; the engine's and the oracle's ``hf`` mode
follow transformers' Qwen2 / Qwen3 modelling code, so the fixtures come from the locally
installed ``transformers`` (5.15.0 in this container): ``Qwen2ForCausalLM`` and
``Qwen3ForCausalLM`` built offline from an in-memory config (no checkpoint, no network),
eager attention, parameters in bf16 with the rotary inv_freq buffer kept fp32 as
``from_pretrained(torch_dtype=bfloat16)`` leaves it, and their weights set to the
repository's counter-based synthetic weights (weights.HostWeights.synthetic — the same
values the engine's qie_engine_init_synthetic generates on the device), so a fixture holds
no weights: only the config, the synthetic parameters, a prompt, the model's greedy
continuation (16 tokens, KV-cached decode) and the bf16 logits of every decision.

Usage:  python tools/make_hf_golden.py      (CPU, ~10 s)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

SYN = dict(seed=7, w_scale=0.08, norm_scale=0.25, bias_scale=0.05)
CASES = {
    "hf_qwen2_tiny": dict(model_type="qwen2", vocab_size=1024, hidden_size=256, intermediate_size=512,
                          num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                          max_position_embeddings=512, rope_theta=1e6, rms_norm_eps=1e-6,
                          tie_word_embeddings=False),
    "hf_qwen3_tiny": dict(model_type="qwen3", vocab_size=1024, hidden_size=256, intermediate_size=512,
                          num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
                          max_position_embeddings=512, rope_theta=1e6, rms_norm_eps=1e-6,
                          tie_word_embeddings=False),
    # tied embedding (Qwen2-0.5B's layout), 14 / 2 heads of 64 like Qwen2-0.5B
    "hf_qwen2_tied": dict(model_type="qwen2", vocab_size=1536, hidden_size=448, intermediate_size=640,
                          num_hidden_layers=2, num_attention_heads=7, num_key_value_heads=1,
                          max_position_embeddings=512, rope_theta=1e6, rms_norm_eps=1e-6,
                          tie_word_embeddings=True),
}
PROMPT_LEN, N_NEW = 12, 16
ATTN = "eager"   # eager_attention_forward: bf16 scores and probabilities (the oracle's or_set_hf_eager form)


def to_bf16_bits(t):
    import torch
    return t.detach().to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def make(name, cfg):
    import torch
    import transformers
    from qwen_inference_engine_amd import spec as S, weights as W
    Cfg = transformers.Qwen2Config if cfg["model_type"] == "qwen2" else transformers.Qwen3Config
    Mdl = transformers.Qwen2ForCausalLM if cfg["model_type"] == "qwen2" else transformers.Qwen3ForCausalLM
    kw = {k: v for k, v in cfg.items() if k != "model_type"}
    c = Cfg(attn_implementation=ATTN, **kw)
    spec = S.ModelSpec.from_hf_config(dict(cfg), name=name, numerics="hf")
    hw = W.HostWeights.synthetic(spec, W.SynthParams(**SYN))
    torch.manual_seed(0)
    m = Mdl(c).eval()
    for p in m.parameters():          # bf16 parameters, fp32 rotary buffer
        p.data = p.data.to(torch.bfloat16)
    sd = m.state_dict()
    for k in sd:
        src = k if k in hw.tensors else ("model.embed_tokens.weight" if k == "lm_head.weight" else None)
        assert src is not None, f"{name}: no synthetic tensor for {k}"
        sd[k] = torch.from_numpy(np.ascontiguousarray(hw.tensors[src]).view(np.int16).copy()) \
            .view(torch.bfloat16).reshape(sd[k].shape)
    m.load_state_dict(sd)
    prompt = [int(t) for t in np.random.default_rng(3).integers(0, spec.vocab, PROMPT_LEN)]
    ids, logits = [], []
    with torch.no_grad():
        out = m(torch.tensor([prompt]), use_cache=True)
        for i in range(N_NEW):
            lg = out.logits[0, -1]
            logits.append(to_bf16_bits(lg))
            ids.append(int(torch.argmax(lg.float())))
            if i + 1 < N_NEW:
                out = m(torch.tensor([[ids[-1]]]), past_key_values=out.past_key_values, use_cache=True)
    path = os.path.join(GOLD, name + ".npz")
    np.savez_compressed(path, config=json.dumps(cfg), synth=json.dumps(SYN), prompt=np.array(prompt, np.int32),
                        ids=np.array(ids, np.int32), logits=np.stack(logits),
                        transformers_version=transformers.__version__, torch_version=torch.__version__)
    print(f"{path}: ids {ids}")


if __name__ == "__main__":
    for n, c in CASES.items():
        make(n, c)
