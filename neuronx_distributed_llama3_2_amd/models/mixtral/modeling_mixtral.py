"""Mixtral (sparse MoE) causal LM for TP + SP + EP training (reference example:
examples/training/mixtral/modeling_mixtral_moe_nxd.py; inference: examples/inference/mixtral/).

Same block structure as the Llama model (fused add+RMSNorm, fused QKV + RoPE + flash attention)
with the dense MLP replaced by the MoE layer (modules/moe): top-k router, expert-fused TP-sharded
GLU experts, capacity-factor or dropless dispatch, EP all-to-all.  The loss adds
`router_aux_loss_coef * load_balancing_loss` over all layers' router logits.
"""

from __future__ import annotations

import math
from functools import partial
from typing import Optional

import torch
from torch import nn
from torch.utils.checkpoint import checkpoint

from ...modules.moe import ExpertMLPs, MoE, RouterSinkhorn, RouterTopK, load_balancing_loss_func
from ...parallel_layers.layer_norm import RMSNorm
from ...parallel_layers.layers import ColumnParallelLinear, ParallelEmbedding
from ...parallel_layers.loss_functions import parallel_cross_entropy
from ...parallel_layers.parallel_state import get_tensor_model_parallel_size
from ..llama.modeling_llama import CausalLMOutput, LlamaAttention, RopeCache, _init_normal


class MixtralDecoderLayer(nn.Module):
    def __init__(self, config, dtype, device, rope_cache):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False) and get_tensor_model_parallel_size() > 1
        self.self_attn = LlamaAttention(config, dtype, device, rope_cache)
        init = partial(_init_normal, config.initializer_range)
        E, k = config.num_local_experts, config.num_experts_per_tok
        if getattr(config, "moe_router", "topk") == "sinkhorn":
            router = RouterSinkhorn(E, 1, config.hidden_size, dtype=torch.float32, device=device)
        else:
            router = RouterTopK(E, k, config.hidden_size, dtype=torch.float32, device=device)
        mlps = ExpertMLPs(E, k, config.hidden_size, config.intermediate_size, "silu", True,
                          getattr(config, "capacity_factor", None), normalize_top_k_affinities=k > 1,
                          init_method=init, output_layer_init_method=init, dtype=dtype, device=device)
        self.block_sparse_moe = MoE(router, mlps, sequence_parallel_enabled=sp, return_router_logits=True)
        self.input_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps, sequence_parallel_enabled=sp,
                                       dtype=dtype, device=device)
        self.post_attention_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps,
                                                sequence_parallel_enabled=sp, dtype=dtype, device=device)

    def forward(self, hidden_states, residual=None):
        if residual is None:
            normed = self.input_layernorm(hidden_states)
            residual = hidden_states
        else:
            normed, residual = self.input_layernorm(hidden_states, residual)
        attn = self.self_attn(normed)
        normed, residual = self.post_attention_layernorm(attn, residual)
        out, router_logits = self.block_sparse_moe(normed)
        return out, residual, router_logits


class MixtralModel(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = config
        sp = getattr(config, "sequence_parallel_enabled", False) and get_tensor_model_parallel_size() > 1
        head_dim = getattr(config, "head_dim", None) or config.hidden_size // config.num_attention_heads
        self.rope_cache = RopeCache(config, head_dim)
        init = partial(_init_normal, config.initializer_range)
        self.embed_tokens = ParallelEmbedding(config.vocab_size, config.hidden_size, init_method=init, dtype=dtype,
                                              device=device, sequence_parallel_enabled=sp)
        self.layers = nn.ModuleList([MixtralDecoderLayer(config, dtype, device, self.rope_cache)
                                     for _ in range(config.num_hidden_layers)])
        self.norm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps, sequence_parallel_enabled=sp, dtype=dtype,
                            device=device)
        self.activation_checkpoint = getattr(config, "activation_checkpoint", None)

    def forward(self, input_ids):
        hidden = self.embed_tokens(input_ids.t().contiguous())
        residual = None
        logits_all = []
        for layer in self.layers:
            if self.activation_checkpoint == "full" and self.training:
                res = checkpoint(layer, hidden, residual, use_reentrant=False)
            else:
                res = layer(hidden, residual)
            hidden, residual = res[0], res[1]
            logits_all.append(res[2])
        return self.norm(hidden, residual)[0], torch.cat(logits_all, 0)


class MixtralForCausalLM(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = config
        self.model = MixtralModel(config, dtype, device)
        sp = getattr(config, "sequence_parallel_enabled", False) and get_tensor_model_parallel_size() > 1
        init = partial(_init_normal, config.initializer_range)
        self.lm_head = ColumnParallelLinear(config.hidden_size, config.vocab_size, bias=False, gather_output=False,
                                           init_method=init, sequence_parallel_enabled=sp, dtype=dtype, device=device)

    def forward(self, input_ids, attention_mask=None, labels=None, **unused):
        hidden, router_logits = self.model(input_ids)
        logits = self.lm_head(hidden)
        loss = None
        if labels is not None:
            lab = labels.t()
            nxt = lab[1:]
            if attention_mask is not None:
                nxt = torch.where(attention_mask.t()[1:] > 0, nxt, torch.full_like(nxt, -100))
            shifted = torch.cat([nxt, torch.full_like(lab[:1], -100)], dim=0)
            per_tok = parallel_cross_entropy(logits, shifted, inplace_backward=True)
            loss = per_tok.sum() / (shifted != -100).sum().clamp(min=1)
            coef = float(getattr(self.config, "router_aux_loss_coef", 0.02))
            if coef > 0:
                aux = load_balancing_loss_func(router_logits, self.config.num_local_experts,
                                               self.config.num_experts_per_tok)
                loss = loss + coef * aux.to(loss.dtype)
        return CausalLMOutput(loss=loss, logits=logits)


def mixtral_config(name: str = "mixtral-8x7b", **overrides):
    from transformers import MixtralConfig

    presets = {
        "mixtral-8x7b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                             num_key_value_heads=8, vocab_size=32000, rope_theta=1e6, max_position_embeddings=32768,
                             num_local_experts=8, num_experts_per_tok=2, rms_norm_eps=1e-5),
        "tiny": dict(hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
                     num_key_value_heads=2, vocab_size=512, rope_theta=1e6, max_position_embeddings=512,
                     num_local_experts=4, num_experts_per_tok=2, rms_norm_eps=1e-5),
    }
    kw = dict(presets[name])
    kw.setdefault("initializer_range", 0.02)
    kw.setdefault("router_aux_loss_coef", 0.02)
    extra = {k: overrides.pop(k) for k in list(overrides) if k in ("sequence_parallel_enabled", "capacity_factor",
                                                                   "moe_router", "activation_checkpoint")}
    kw.update(overrides)
    cfg = MixtralConfig(**kw)
    for k, v in extra.items():
        setattr(cfg, k, v)
    return cfg
