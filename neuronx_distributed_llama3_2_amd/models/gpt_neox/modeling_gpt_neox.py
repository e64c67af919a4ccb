"""GPT-NeoX causal LM (6.9B / 20B pretraining examples) with tensor + sequence parallelism
(reference: examples/training/tp_dp_gpt_neox_hf_pretrain/tp_dp_gpt_neox_20b_hf_pretrain/
modeling_gpt_neox_nxd.py:53-560 — HF GPTNeoX with NxD parallel layers substituted).

Same parameter names as HF `GPTNeoXForCausalLM` (gpt_neox.embed_in, layers.N.attention.
query_key_value / dense, mlp.dense_h_to_4h / dense_4h_to_h, input/post_attention_layernorm,
final_layer_norm, embed_out), so HF checkpoints load after TP sharding.  The fused
query_key_value output is laid out per head ([h0: q k v][h1: q k v]...), so a contiguous split of
its rows over TP ranks keeps whole heads on a rank.  Partial rotary embedding (rotary_pct),
parallel residual (x + attn(ln1 x) + mlp(ln2 x)), vocab-parallel embed_in / embed_out / CE.
Activations are [S, B, H] (SP shards = contiguous sequence slabs).
"""

from __future__ import annotations

from functools import partial
from typing import Optional

import torch
from torch import nn
from torch.utils.checkpoint import checkpoint

from ...parallel_layers.layer_norm import LayerNorm
from ...parallel_layers.layers import ColumnParallelLinear, ParallelEmbedding, RowParallelLinear
from ...parallel_layers.loss_functions import parallel_cross_entropy
from ...parallel_layers.parallel_state import get_tensor_model_parallel_size
from ...parallel_layers.utils import divide
from ..attention import attention
from ..llama.modeling_llama import CausalLMOutput


def _init_normal(std, w):
    return nn.init.normal_(w, mean=0.0, std=std)


def _act(name):
    from transformers.activations import ACT2FN

    return ACT2FN[name]


class NeoXRotary:
    def __init__(self, rot_dims: int, base: float, max_pos: int):
        self.rot_dims, self.base, self.max_pos = rot_dims, base, max_pos
        self._cache = {}

    def tables(self, S: int, device):
        key = (S, str(device))
        if key not in self._cache:
            inv = 1.0 / (self.base ** (torch.arange(0, self.rot_dims, 2, dtype=torch.float32) / self.rot_dims))
            t = torch.arange(S, dtype=torch.float32)
            f = torch.outer(t, inv)
            emb = torch.cat([f, f], -1)
            self._cache[key] = (emb.cos().to(device), emb.sin().to(device))
        return self._cache[key]

    def apply(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        """x [S, B, H, D]: rotate the first rot_dims features (rotate-half convention)."""
        r = self.rot_dims
        xr, xp = x[..., :r].float(), x[..., r:]
        c, s = cos[:, None, None, :], sin[:, None, None, :]
        x1, x2 = xr[..., : r // 2], xr[..., r // 2:]
        rot = torch.cat([-x2, x1], -1)
        return torch.cat([(xr * c + rot * s).to(x.dtype), xp], -1)


class GPTNeoXAttention(nn.Module):
    def __init__(self, config, dtype, device, rotary):
        super().__init__()
        tp = get_tensor_model_parallel_size()
        self.num_heads = config.num_attention_heads
        self.head_dim = config.hidden_size // self.num_heads
        self.heads_local = divide(self.num_heads, tp)
        sp = getattr(config, "sequence_parallel_enabled", False)
        init = partial(_init_normal, config.initializer_range)
        bias = getattr(config, "attention_bias", True)
        self.query_key_value = ColumnParallelLinear(config.hidden_size, 3 * config.hidden_size, bias=bias,
                                                    gather_output=False, init_method=init,
                                                    sequence_parallel_enabled=sp, dtype=dtype, device=device)
        self.dense = RowParallelLinear(config.hidden_size, config.hidden_size, bias=bias, input_is_parallel=True,
                                       init_method=init, sequence_parallel_enabled=sp, dtype=dtype, device=device)
        self.rotary = rotary

    def forward(self, x):
        qkv = self.query_key_value(x)                 # [S, B, 3 H/tp]
        S, B = qkv.shape[:2]
        qkv = qkv.view(S, B, self.heads_local, 3, self.head_dim)
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        cos, sin = self.rotary.tables(S, x.device)
        q, k = self.rotary.apply(q, cos, sin), self.rotary.apply(k, cos, sin)
        o = attention(q.transpose(0, 1).contiguous(), k.transpose(0, 1).contiguous(), v.transpose(0, 1).contiguous(),
                      causal=True)                    # [B, S, h, D]
        return self.dense(o.transpose(0, 1).reshape(S, B, self.heads_local * self.head_dim))


class GPTNeoXMLP(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False)
        init = partial(_init_normal, config.initializer_range)
        self.dense_h_to_4h = ColumnParallelLinear(config.hidden_size, config.intermediate_size, bias=True,
                                                  gather_output=False, init_method=init, sequence_parallel_enabled=sp,
                                                  dtype=dtype, device=device)
        self.dense_4h_to_h = RowParallelLinear(config.intermediate_size, config.hidden_size, bias=True,
                                               input_is_parallel=True, init_method=init, sequence_parallel_enabled=sp,
                                               dtype=dtype, device=device)
        self.act = _act(config.hidden_act)

    def forward(self, x):
        return self.dense_4h_to_h(self.act(self.dense_h_to_4h(x)))


class GPTNeoXLayer(nn.Module):
    def __init__(self, config, dtype, device, rotary):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False)
        self.use_parallel_residual = getattr(config, "use_parallel_residual", True)
        self.input_layernorm = LayerNorm(config.hidden_size, eps=config.layer_norm_eps, sequence_parallel_enabled=sp,
                                         dtype=dtype, device=device)
        self.post_attention_layernorm = LayerNorm(config.hidden_size, eps=config.layer_norm_eps,
                                                  sequence_parallel_enabled=sp, dtype=dtype, device=device)
        self.attention = GPTNeoXAttention(config, dtype, device, rotary)
        self.mlp = GPTNeoXMLP(config, dtype, device)

    def forward(self, x):
        a = self.attention(self.input_layernorm(x))
        if self.use_parallel_residual:
            return x + a + self.mlp(self.post_attention_layernorm(x))
        h = x + a
        return h + self.mlp(self.post_attention_layernorm(h))


class GPTNeoXModel(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False) and get_tensor_model_parallel_size() > 1
        self.sequence_parallel_enabled = sp
        head_dim = config.hidden_size // config.num_attention_heads
        rot = int(head_dim * getattr(config, "rotary_pct", 0.25))
        self.rotary = NeoXRotary(rot, float(getattr(config, "rotary_emb_base", 10000)), config.max_position_embeddings)
        init = partial(_init_normal, config.initializer_range)
        self.embed_in = ParallelEmbedding(config.vocab_size, config.hidden_size, init_method=init, dtype=dtype,
                                          device=device, sequence_parallel_enabled=sp)
        self.layers = nn.ModuleList([GPTNeoXLayer(config, dtype, device, self.rotary)
                                     for _ in range(config.num_hidden_layers)])
        self.final_layer_norm = LayerNorm(config.hidden_size, eps=config.layer_norm_eps, sequence_parallel_enabled=sp,
                                          dtype=dtype, device=device)
        self.activation_checkpoint = getattr(config, "activation_checkpoint", None)

    def forward(self, input_ids):
        h = self.embed_in(input_ids.t().contiguous())     # [S(/tp), B, H]
        for layer in self.layers:
            if self.activation_checkpoint == "full" and self.training:
                h = checkpoint(layer, h, use_reentrant=False)
            else:
                h = layer(h)
        return self.final_layer_norm(h)


class GPTNeoXForCausalLM(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = config
        self.gpt_neox = GPTNeoXModel(config, dtype, device)
        init = partial(_init_normal, config.initializer_range)
        self.embed_out = ColumnParallelLinear(config.hidden_size, config.vocab_size, bias=False, gather_output=False,
                                              init_method=init,
                                              sequence_parallel_enabled=self.gpt_neox.sequence_parallel_enabled,
                                              dtype=dtype, device=device)

    def forward(self, input_ids, attention_mask: Optional[torch.Tensor] = None, labels=None, **unused):
        logits = self.embed_out(self.gpt_neox(input_ids))   # [S, B, V/tp]
        loss = None
        if labels is not None:
            lab = labels.t()
            nxt = lab[1:]
            if attention_mask is not None:
                nxt = torch.where(attention_mask.t()[1:] > 0, nxt, torch.full_like(nxt, -100))
            shifted = torch.cat([nxt, torch.full_like(lab[:1], -100)], 0)
            per_tok = parallel_cross_entropy(logits, shifted)
            loss = per_tok.sum() / (shifted != -100).sum().clamp(min=1)
        return CausalLMOutput(loss=loss, logits=logits)


def hf_to_nxd(sd):
    """HF GPT-NeoX state dict -> this model's names (transformers >= 5 calls the output projection
    `lm_head`; NxD / transformers 4 call it `embed_out`)."""
    return {("embed_out.weight" if k == "lm_head.weight" else k): v for k, v in sd.items()}


def gpt_neox_config(name: str = "gpt-neox-20b", **overrides):
    from transformers import GPTNeoXConfig

    presets = {
        "gpt-neox-20b": dict(vocab_size=50432, hidden_size=6144, num_hidden_layers=44, num_attention_heads=64,
                             intermediate_size=24576, hidden_act="gelu_fast", rotary_pct=0.25,
                             rotary_emb_base=10000, max_position_embeddings=2048, layer_norm_eps=1e-5,
                             use_parallel_residual=True),
        "pythia-6.9b": dict(vocab_size=50432, hidden_size=4096, num_hidden_layers=32, num_attention_heads=32,
                            intermediate_size=16384, hidden_act="gelu", rotary_pct=0.25, rotary_emb_base=10000,
                            max_position_embeddings=2048, layer_norm_eps=1e-5, use_parallel_residual=True),
        "tiny": dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=512, hidden_act="gelu", rotary_pct=0.25, rotary_emb_base=10000,
                     max_position_embeddings=256, layer_norm_eps=1e-5, use_parallel_residual=True),
    }
    kw = dict(presets[name])
    kw.setdefault("initializer_range", 0.02)
    kw.update(overrides)
    cfg = GPTNeoXConfig(**kw)
    for k in ("sequence_parallel_enabled", "activation_checkpoint"):
        if k in overrides:
            setattr(cfg, k, overrides[k])
    return cfg
