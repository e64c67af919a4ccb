"""Hugging Face Llama <-> framework parameter naming (full, unsharded tensors).

Framework layout (models/llama/modeling_llama.py): one fused QKV weight per attention block
(`self_attn.qkv_proj.weight_qkv` = [q; k; v] rows) and one fused `mlp.gate_up_proj.weight`
([gate; up] rows).  Tensor-parallel sharding of the full tensors is done separately from the
parameters' attributes (parallel_layers/sharding.py).  Reference equivalents:
scripts/checkpoint_converter.py:238-532 (gate/up fusion, fused QKV) and the inference
`convert_hf_to_neuron_state_dict` hooks (examples/inference/llama3/neuron_modeling_llama.py).
"""

from __future__ import annotations

import re
from typing import Dict, Mapping

import torch

_LAYER = re.compile(r"^model\.layers\.(\d+)\.(.+)$")


def hf_to_nxd(hf_sd: Mapping[str, torch.Tensor], config) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {}
    L = config.num_hidden_layers
    for k, v in hf_sd.items():
        if "rotary_emb" in k:
            continue
        m = _LAYER.match(k)
        if m and any(s in m.group(2) for s in ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj")):
            continue
        out[k] = v
    for i in range(L):
        p = f"model.layers.{i}."
        for suffix in ("weight", "bias"):
            q = hf_sd.get(p + f"self_attn.q_proj.{suffix}")
            if q is not None:
                k = hf_sd[p + f"self_attn.k_proj.{suffix}"]
                v = hf_sd[p + f"self_attn.v_proj.{suffix}"]
                out[p + f"self_attn.qkv_proj.{suffix}_qkv"] = torch.cat([q, k, v], dim=0)
        g = hf_sd.get(p + "mlp.gate_proj.weight")
        if g is not None:
            out[p + "mlp.gate_up_proj.weight"] = torch.cat([g, hf_sd[p + "mlp.up_proj.weight"]], dim=0)
    if "lm_head.weight" not in out and getattr(config, "tie_word_embeddings", False):
        out["lm_head.weight"] = out["model.embed_tokens.weight"]
    return out


def nxd_to_hf(sd: Mapping[str, torch.Tensor], config) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {}
    nq = config.num_attention_heads
    nkv = getattr(config, "num_key_value_heads", None) or nq
    D = getattr(config, "head_dim", None) or config.hidden_size // nq
    for k, v in sd.items():
        m = _LAYER.match(k)
        if m and m.group(2).startswith("self_attn.qkv_proj."):
            p = f"model.layers.{m.group(1)}.self_attn."
            suffix = "weight" if m.group(2).endswith("weight_qkv") else "bias"
            q, kk, vv = torch.split(v, [nq * D, nkv * D, nkv * D], dim=0)
            out[p + f"q_proj.{suffix}"], out[p + f"k_proj.{suffix}"], out[p + f"v_proj.{suffix}"] = q, kk, vv
        elif m and m.group(2) == "mlp.gate_up_proj.weight":
            p = f"model.layers.{m.group(1)}.mlp."
            g, u = v.chunk(2, dim=0)
            out[p + "gate_proj.weight"], out[p + "up_proj.weight"] = g, u
        else:
            out[k] = v
    if getattr(config, "tie_word_embeddings", False):
        out.pop("lm_head.weight", None)
    return out
