"""Hugging Face Mixtral / DBRX -> framework MoE parameter naming (full, unsharded tensors).

Framework layout (models/mixtral/modeling_mixtral.py, modules/moe): per layer one fused QKV
(`self_attn.qkv_proj.weight_qkv`), the router `block_sparse_moe.router.linear_router.weight` [E, H]
and expert-fused 3-D weights `block_sparse_moe.expert_mlps.mlp_op.gate_up_proj.weight` [E, H, 2I]
(gate columns then up columns) and `...down_proj.weight` [E, I, H].  TP sharding of the full
tensors follows the parameters' attributes (parallel_layers/sharding.py; gate_up with stride 2).

Reference equivalents: examples/inference/mixtral/neuron_modeling_mixtral.py:61-112
(`convert_mixtral_to_neuron_state_dict`) and examples/inference/dbrx/neuron_modeling_dbrx.py:60-108
(`convert_dbrx_to_neuron_state_dict`).  DBRX runs on the same MoE decoder with LayerNorm
(no bias) instead of RMSNorm and clipped QKV; `dbrx_to_mixtral_config` translates its config.
"""

from __future__ import annotations

import re
from typing import Dict, Mapping

import torch

from ..llama.convert import hf_to_nxd as _llama_attn_to_nxd

_MOE = "block_sparse_moe."
_EXPERTS = _MOE + "expert_mlps.mlp_op."


def mixtral_hf_to_nxd(hf_sd: Mapping[str, torch.Tensor], config) -> Dict[str, torch.Tensor]:
    """Accepts both the on-disk hub layout (`block_sparse_moe.gate`, `experts.{e}.w1/w2/w3`) and
    the transformers>=5 in-memory layout (`mlp.gate`, `mlp.experts.gate_up_proj` [E, 2I, H],
    `mlp.experts.down_proj` [E, H, I])."""
    L, E = config.num_hidden_layers, config.num_local_experts
    moe_keys = re.compile(r"^model\.layers\.\d+\.(block_sparse_moe|mlp)\.")
    out = _llama_attn_to_nxd({k: v for k, v in hf_sd.items() if not moe_keys.match(k)}, config)
    for i in range(L):
        p = f"model.layers.{i}."
        gate = hf_sd.get(p + "block_sparse_moe.gate.weight", hf_sd.get(p + "mlp.gate.weight"))
        if gate is None:
            continue
        out[p + _MOE + "router.linear_router.weight"] = gate
        if p + "mlp.experts.gate_up_proj" in hf_sd:
            gu = hf_sd[p + "mlp.experts.gate_up_proj"]                     # [E, 2I, H], gate rows first
            out[p + _EXPERTS + "gate_up_proj.weight"] = gu.transpose(1, 2).contiguous()
            out[p + _EXPERTS + "down_proj.weight"] = hf_sd[p + "mlp.experts.down_proj"].transpose(1, 2).contiguous()
        else:
            ex = p + "block_sparse_moe.experts."
            out[p + _EXPERTS + "gate_up_proj.weight"] = torch.stack(
                [torch.cat([hf_sd[f"{ex}{e}.w1.weight"].t(), hf_sd[f"{ex}{e}.w3.weight"].t()], dim=1)
                 for e in range(E)])
            out[p + _EXPERTS + "down_proj.weight"] = torch.stack([hf_sd[f"{ex}{e}.w2.weight"].t() for e in range(E)])
    return out


def mixtral_nxd_to_hf(sd: Mapping[str, torch.Tensor], config) -> Dict[str, torch.Tensor]:
    """Framework -> on-disk hub layout (per-expert w1/w2/w3)."""
    from ..llama.convert import nxd_to_hf

    L = config.num_hidden_layers
    rest = {k: v for k, v in sd.items() if _MOE not in k}
    out = nxd_to_hf(rest, config)
    for i in range(L):
        p = f"model.layers.{i}."
        r = sd.get(p + _MOE + "router.linear_router.weight")
        if r is None:
            continue
        out[p + "block_sparse_moe.gate.weight"] = r
        gu = sd[p + _EXPERTS + "gate_up_proj.weight"]
        dn = sd[p + _EXPERTS + "down_proj.weight"]
        inter = gu.shape[2] // 2
        for e in range(gu.shape[0]):
            out[f"{p}block_sparse_moe.experts.{e}.w1.weight"] = gu[e, :, :inter].t().contiguous()
            out[f"{p}block_sparse_moe.experts.{e}.w3.weight"] = gu[e, :, inter:].t().contiguous()
            out[f"{p}block_sparse_moe.experts.{e}.w2.weight"] = dn[e].t().contiguous()
    return out


# ---------------------------------------------------------------------------------------- DBRX
def _cfg_get(obj, key, default=None):
    if isinstance(obj, dict):
        return obj.get(key, default)
    return getattr(obj, key, default)


def dbrx_to_mixtral_config(dbrx_cfg, **overrides):
    """DbrxConfig (or its dict) -> the MixtralConfig the MoE decoder is built from, tagged with
    `norm_type="layernorm"`, `clip_qkv` and `source_model_type="dbrx"`."""
    from transformers import MixtralConfig

    g = (lambda k, d=None: dbrx_cfg.get(k, d)) if isinstance(dbrx_cfg, dict) else \
        (lambda k, d=None: getattr(dbrx_cfg, k, d))
    attn, ffn = g("attn_config") or {}, g("ffn_config") or {}
    act = _cfg_get(ffn, "ffn_act_fn") or {"name": "silu"}
    if (act.get("name") if isinstance(act, dict) else act) != "silu":
        raise NotImplementedError(f"DBRX ffn activation {act} (only silu GLU experts are supported)")
    norm_p = _cfg_get(ffn, "moe_normalize_expert_weights", 1.0)
    if norm_p not in (None, 1, 1.0):
        raise NotImplementedError(f"moe_normalize_expert_weights={norm_p} (only L1 / None supported)")
    rope = _cfg_get(attn, "rope_theta") or g("rope_theta") or _cfg_get(g("rope_parameters") or {}, "rope_theta") \
        or 10000.0
    kw = dict(hidden_size=g("d_model"), num_attention_heads=g("n_heads"), num_hidden_layers=g("n_layers"),
              num_key_value_heads=_cfg_get(attn, "kv_n_heads", 1), intermediate_size=_cfg_get(ffn, "ffn_hidden_size"),
              num_local_experts=_cfg_get(ffn, "moe_num_experts"), num_experts_per_tok=_cfg_get(ffn, "moe_top_k", 1),
              vocab_size=g("vocab_size"), max_position_embeddings=g("max_seq_len", 2048),
              rope_theta=float(rope), rms_norm_eps=1e-5,
              tie_word_embeddings=bool(g("tie_word_embeddings", False)), initializer_range=g("initializer_range", 0.02),
              pad_token_id=g("pad_token_id"), eos_token_id=g("eos_token_id"), bos_token_id=g("bos_token_id"))
    kw.update(overrides)
    cfg = MixtralConfig(**kw)
    cfg.norm_type = "layernorm"
    cfg.clip_qkv = _cfg_get(attn, "clip_qkv")
    cfg.normalize_top_k_affinities = norm_p is not None
    cfg.source_model_type = "dbrx"
    return cfg


def dbrx_hf_to_nxd(hf_sd: Mapping[str, torch.Tensor], config) -> Dict[str, torch.Tensor]:
    """HF DBRX names (`transformer.blocks.{l}.norm_attn_norm.*`, `ffn.experts.mlp.{w1,v1,w2}`
    [E*I, H]) -> framework MoE names; `config` is the translated MixtralConfig."""
    E, inter, H = config.num_local_experts, config.intermediate_size, config.hidden_size
    out = {"model.embed_tokens.weight": hf_sd["transformer.wte.weight"],
           "model.norm.weight": hf_sd["transformer.norm_f.weight"]}
    if "lm_head.weight" in hf_sd:
        out["lm_head.weight"] = hf_sd["lm_head.weight"]
    elif getattr(config, "tie_word_embeddings", False):
        out["lm_head.weight"] = out["model.embed_tokens.weight"]
    for i in range(config.num_hidden_layers):
        b, p = f"transformer.blocks.{i}.", f"model.layers.{i}."
        out[p + "input_layernorm.weight"] = hf_sd[b + "norm_attn_norm.norm_1.weight"]
        out[p + "post_attention_layernorm.weight"] = hf_sd[b + "norm_attn_norm.norm_2.weight"]
        out[p + "self_attn.qkv_proj.weight_qkv"] = hf_sd[b + "norm_attn_norm.attn.Wqkv.weight"]
        out[p + "self_attn.o_proj.weight"] = hf_sd[b + "norm_attn_norm.attn.out_proj.weight"]
        out[p + _MOE + "router.linear_router.weight"] = hf_sd[b + "ffn.router.layer.weight"]
        w1 = hf_sd[b + "ffn.experts.mlp.w1"].view(E, inter, H)
        v1 = hf_sd[b + "ffn.experts.mlp.v1"].view(E, inter, H)
        out[p + _EXPERTS + "gate_up_proj.weight"] = torch.cat([w1, v1], dim=1).transpose(1, 2).contiguous()
        out[p + _EXPERTS + "down_proj.weight"] = hf_sd[b + "ffn.experts.mlp.w2"].view(E, inter, H).contiguous()
    return out
