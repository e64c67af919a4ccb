"""Llama-2/3/3.1/3.2 causal LM for tensor + sequence parallel training on MI355X.

Capability parity with the reference training model (examples/training/llama/modeling_llama_nxd.py:134-774):
GQA QKV column-parallel projection with KV replication, fused gate_up (stride=2) / down MLP,
vocab-parallel embedding + lm_head + cross entropy, Megatron sequence parallelism, flash
attention, selective / full activation checkpointing.  MI355X-first structure:

* activations are [S, B, H] (sequence-major) so the SP shard of a rank is one contiguous slab;
* each decoder block is: fused (residual add + RMSNorm) kernel -> ONE QKV GEMM into a fused
  buffer -> in-place RoPE + GQA flash attention on strided views of that buffer (no transposes,
  no repeat_kv) -> o_proj (reduce-scatter) -> fused add+norm -> gate_up GEMM -> SwiGLU kernel ->
  down GEMM (reduce-scatter);
* the embedding reduce-scatters straight into the SP layout and the lm_head all-gathers from it
  (one collective each way), the loss is the fused vocab-parallel cross entropy whose backward
  overwrites the logits buffer in place; no fp64 anywhere (the reference upcasts logits and norms
  to fp64 only to survive XLA_DOWNCAST_BF16).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from functools import partial
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn
from torch.utils.checkpoint import checkpoint

from ... import ops
from ...modules.qkv_linear import GQAQKVColumnParallelLinear
from ...parallel_layers.layer_norm import RMSNorm
from ...parallel_layers.layers import ColumnParallelLinear, ParallelEmbedding, RowParallelLinear
from ...parallel_layers.loss_functions import parallel_cross_entropy
from ...parallel_layers.mappings import gather_from_sequence_parallel_region, scatter_to_sequence_parallel_region
from ...parallel_layers import stream_split
from ...parallel_layers.parallel_state import (get_data_parallel_size, get_pipeline_model_parallel_size,
                                                      get_tensor_model_parallel_size)
from ...parallel_layers.utils import divide


class CausalLMOutput(dict):
    """{loss, logits} with attribute access (a dict, so torch.fx can return it from a traced graph)."""

    def __init__(self, loss=None, logits=None):
        super().__init__(loss=loss, logits=logits)

    @property
    def loss(self):
        return self["loss"]

    @property
    def logits(self):
        return self["logits"]


def _init_normal(std, w):
    return nn.init.normal_(w, mean=0.0, std=std)


class LlamaMLP(nn.Module):
    def __init__(self, config, dtype, device):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False)
        init = partial(_init_normal, config.initializer_range)
        self.gate_up_proj = ColumnParallelLinear(config.hidden_size, 2 * config.intermediate_size, stride=2, bias=False,
                                                 gather_output=False, init_method=init, sequence_parallel_enabled=sp,
                                                 dtype=dtype, device=device)
        self.down_proj = RowParallelLinear(config.intermediate_size, config.hidden_size, bias=False,
                                           input_is_parallel=True, init_method=init, sequence_parallel_enabled=sp,
                                           dtype=dtype, device=device)
        self.selective_checkpoint = getattr(config, "selective_checkpoint_enabled", False)

    def forward(self, x):
        gu = self.gate_up_proj(x)
        if self.selective_checkpoint and self.training:
            h = checkpoint(ops.swiglu, gu, True, use_reentrant=False)
        else:
            h = ops.swiglu(gu, token_major=True)   # token-major copies feed the TN weight gradients
        return self.down_proj(h)


class LlamaAttention(nn.Module):
    def __init__(self, config, dtype, device, rope_cache):
        super().__init__()
        self.config = config
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.num_kv_heads = getattr(config, "num_key_value_heads", None) or self.num_heads
        self.head_dim = getattr(config, "head_dim", None) or self.hidden_size // self.num_heads
        tp = get_tensor_model_parallel_size()
        kv_mult = getattr(config, "kv_shared_group_size", 1)
        if self.num_kv_heads * kv_mult < tp or (self.num_kv_heads * kv_mult) % tp:
            kv_mult = max(kv_mult, tp // math.gcd(tp, self.num_kv_heads))
        self.kv_mult = kv_mult
        self.num_heads_local = divide(self.num_heads, tp)
        self.num_kv_heads_local = divide(self.num_kv_heads * kv_mult, tp)
        sp = getattr(config, "sequence_parallel_enabled", False)
        init = partial(_init_normal, config.initializer_range)
        self.qkv_proj = GQAQKVColumnParallelLinear(
            self.hidden_size, [self.num_heads * self.head_dim, self.num_kv_heads * self.head_dim],
            bias=getattr(config, "attention_bias", False), gather_output=False, init_method=init,
            sequence_parallel_enabled=sp, kv_size_multiplier=kv_mult, fuse_qkv=True, dtype=dtype, device=device)
        self.o_proj = RowParallelLinear(self.num_heads * self.head_dim, self.hidden_size,
                                        bias=getattr(config, "attention_bias", False), input_is_parallel=True,
                                        init_method=init, sequence_parallel_enabled=sp, dtype=dtype, device=device,
                                        keep_master_weight=kv_mult > 1)
        if kv_mult > 1:
            # replicated kv heads: this rank's q heads are head group q_group_order[rank] (see
            # qkv_proj), so its o_proj input columns are that group's (reference
            # scripts/checkpoint_converter.py:463-481 reshuffles o_proj the same way)
            _regroup_row_parallel(self.o_proj, tp, kv_mult)
        self.rope_cache = rope_cache

    def forward(self, x):
        qkv = self.qkv_proj.forward_fused(x)  # [S, B, (nq + 2 nkv) D]
        cos_t, sin_t = self.rope_cache.tables(qkv.device)
        o = ops.rope_attention(qkv, cos_t, sin_t, self.num_heads_local, self.num_kv_heads_local, self.head_dim,
                               causal=True)
        return self.o_proj(o)


def _regroup_row_parallel(layer, tp: int, mult: int) -> None:
    from ...parallel_layers.parallel_state import get_tensor_model_parallel_rank
    from ...parallel_layers.sharding import q_group_order

    layer.weight.qkv_qgroup_mult = mult
    master = getattr(layer, "master_weight", None)
    if master is not None and layer.weight.device.type != "meta":
        g = q_group_order(tp, mult)[get_tensor_model_parallel_rank()]
        with torch.no_grad():
            layer.weight.copy_(torch.chunk(master, tp, dim=1)[g])
    layer.master_weight = None


class RopeCache:
    """fp32 cos/sin tables shared by every layer (one per device)."""

    def __init__(self, config, head_dim):
        self.inv_freq = ops.inv_freq_from_config(config, head_dim)
        self.max_pos = int(getattr(config, "max_position_embeddings", 8192))
        self._cache = {}

    def tables(self, device):
        key = str(device)
        if key not in self._cache:
            self._cache[key] = ops.rope_tables(self.inv_freq, self.max_pos, device=device)
        return self._cache[key]


class LlamaDecoderLayer(nn.Module):
    def __init__(self, config, dtype, device, rope_cache):
        super().__init__()
        sp = getattr(config, "sequence_parallel_enabled", False)
        self.self_attn = LlamaAttention(config, dtype, device, rope_cache)
        self.mlp = LlamaMLP(config, dtype, device)
        self.input_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps, sequence_parallel_enabled=sp,
                                       dtype=dtype, device=device)
        self.post_attention_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps,
                                                sequence_parallel_enabled=sp, dtype=dtype, device=device)

    def forward(self, hidden_states, residual=None):
        """Pre-norm block on the un-added stream: returns (mlp_out, residual) where the true hidden
        state is mlp_out + residual (the add is fused into the next norm kernel)."""
        if residual is None:
            normed = self.input_layernorm(hidden_states)
            residual = hidden_states
        else:
            normed, residual = self.input_layernorm(hidden_states, residual)
        attn = self.self_attn(normed)
        normed, residual = self.post_attention_layernorm(attn, residual)
        return self.mlp(normed), residual

    def forward_stages(self, hidden_states, residual=None):
        """`forward` as a generator that yields after every op that issues a sequence-parallel
        collective (qkv all-gather, o_proj reduce-scatter, gate_up all-gather, down reduce-scatter),
        for the two-stream interleaving of parallel_layers/stream_split.py."""
        if residual is None:
            normed = self.input_layernorm(hidden_states)
            residual = hidden_states
        else:
            normed, residual = self.input_layernorm(hidden_states, residual)
        att = self.self_attn
        qkv = att.qkv_proj.forward_fused(normed)
        yield
        cos_t, sin_t = att.rope_cache.tables(qkv.device)
        o = ops.rope_attention(qkv, cos_t, sin_t, att.num_heads_local, att.num_kv_heads_local, att.head_dim,
                               causal=True)
        attn = att.o_proj(o)
        yield
        normed, residual = self.post_attention_layernorm(attn, residual)
        mlp = self.mlp
        gu = mlp.gate_up_proj(normed)
        yield
        if mlp.selective_checkpoint and self.training:
            h = checkpoint(ops.swiglu, gu, True, use_reentrant=False)
        else:
            h = ops.swiglu(gu, token_major=True)
        out = mlp.down_proj(h)
        yield
        return out, residual


class LlamaModel(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = config
        sp = getattr(config, "sequence_parallel_enabled", False)
        self.sequence_parallel_enabled = sp and get_tensor_model_parallel_size() > 1
        head_dim = getattr(config, "head_dim", None) or config.hidden_size // config.num_attention_heads
        self.rope_cache = RopeCache(config, head_dim)
        init = partial(_init_normal, config.initializer_range)
        self.embed_tokens = ParallelEmbedding(config.vocab_size, config.hidden_size, init_method=init, dtype=dtype,
                                              device=device, sequence_parallel_enabled=self.sequence_parallel_enabled)
        self.layers = nn.ModuleList([LlamaDecoderLayer(config, dtype, device, self.rope_cache)
                                     for _ in range(config.num_hidden_layers)])
        self.norm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps, sequence_parallel_enabled=sp, dtype=dtype,
                            device=device)
        self.activation_checkpoint = getattr(config, "activation_checkpoint", None)  # None | "full"

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        """input_ids [B, S] -> final hidden [S(/tp), B, H] (sequence-parallel shard if SP)."""
        ids = input_ids.t().contiguous()  # [S, B]
        hidden = self.embed_tokens(ids)
        residual = None
        for layer in self.layers:
            # index (not unpack) the (hidden, residual) pair: keeps the loop torch.fx-traceable for
            # pipeline partitioning, where each decoder layer is a leaf
            if self.activation_checkpoint == "full" and self.training:
                res = checkpoint(layer, hidden, residual, use_reentrant=False)
            else:
                res = layer(hidden, residual)
            hidden, residual = res[0], res[1]
        return self.norm(hidden, residual)[0]


class LlamaForCausalLM(nn.Module):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = config
        self.model = LlamaModel(config, dtype, device)
        sp = self.model.sequence_parallel_enabled
        init = partial(_init_normal, config.initializer_range)
        self.lm_head = ColumnParallelLinear(config.hidden_size, config.vocab_size, bias=False, gather_output=False,
                                           init_method=init, sequence_parallel_enabled=sp, dtype=dtype, device=device)
        if getattr(config, "tie_word_embeddings", False):
            assert self.lm_head.weight.shape == self.model.embed_tokens.weight.shape
            self.lm_head.weight = self.model.embed_tokens.weight
            self.lm_head.weight._nxd_tied = True   # grad buffers defer this bucket's reduction

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None, position_ids=None, **unused) -> CausalLMOutput:
        k = self._interleave(input_ids, labels)
        if k:
            return self._forward_interleaved(input_ids, attention_mask, labels, k)
        hidden = self.model(input_ids)
        logits = self.lm_head(hidden)  # [S, B, V/tp]
        loss = None
        if labels is not None:
            tok_sum, n = self._loss_terms(logits, labels, attention_mask)
            loss = tok_sum / n
        return CausalLMOutput(loss=loss, logits=logits)

    @staticmethod
    def _loss_terms(logits, labels, attention_mask):
        """(sum of per-token losses, token count) -- predict token s+1 at position s."""
        lab = labels.t()  # [S, B]
        nxt = lab[1:]
        if attention_mask is not None:
            nxt = torch.where(attention_mask.t()[1:] > 0, nxt, torch.full_like(nxt, -100))
        shifted = torch.cat([nxt, torch.full_like(lab[:1], -100)], dim=0)
        per_tok = parallel_cross_entropy(logits, shifted, inplace_backward=True)
        return per_tok.sum(), (shifted != -100).sum().clamp(min=1)

    def _interleave(self, input_ids, labels) -> int:
        """Parts of the micro-batch for the interleaved forward (0 = one pass)."""
        m = self.model
        if isinstance(input_ids, torch.fx.Proxy) or torch.fx._symbolic_trace.is_fx_tracing():
            return 0   # pipeline partitioning traces the one-pass forward
        if not (stream_split.enabled() and self.training and torch.is_grad_enabled() and labels is not None
                and get_pipeline_model_parallel_size() == 1
                and (m.sequence_parallel_enabled
                     or (stream_split.without_sp() and get_tensor_model_parallel_size() == 1))
                and m.activation_checkpoint != "full"
                and input_ids.dim() == 2 and get_data_parallel_size() == 1):
            return 0
        k = min(stream_split.parts(), input_ids.shape[0])
        while k > 1 and input_ids.shape[0] % k:
            k -= 1
        return k if k >= 2 else 0

    def _part(self, ids, labels, attention_mask):
        m = self.model
        hidden = m.embed_tokens(ids.t().contiguous())
        residual = None
        for layer in m.layers:
            hidden, residual = yield from layer.forward_stages(hidden, residual)
        hidden = m.norm(hidden, residual)[0]
        logits = self.lm_head(hidden)
        yield
        return self._loss_terms(logits, labels, attention_mask)

    def _forward_interleaved(self, input_ids, attention_mask, labels, k: int = 2) -> CausalLMOutput:
        """Training forward of TP + SP as k parts of the micro-batch on k streams, their collectives
        interleaved (parallel_layers/stream_split.py); same loss as the one-pass forward.

        Returns logits=None: the parts' logits are separate buffers that the fused cross-entropy
        backward overwrites in place (inplace_backward), and joining them would copy the whole
        vocab-parallel logits (~2 GiB per micro-batch at TP=8) only to be clobbered.  A caller that
        needs training logits runs with NXD_SP_STREAMS=1 (the one-pass path); that path is also the
        one that runs forward hooks registered on the decoder layers (this one calls
        `LlamaDecoderLayer.forward_stages`, not `forward`)."""
        n = input_ids.shape[0] // k
        sl = [slice(i * n, (i + 1) * n) for i in range(k)]
        self.model.rope_cache.tables(input_ids.device)   # built once on this stream, read by every part
        gens = [self._part(input_ids[s], labels[s], attention_mask[s] if attention_mask is not None else None)
                for s in sl]
        terms = stream_split.run_interleaved(gens, input_ids.device)
        if input_ids.is_cuda:
            for pair in terms:   # made on the parts' streams, read on this one
                for t in pair:
                    t.record_stream(torch.cuda.current_stream())
        loss = sum(t[0] for t in terms) / sum(t[1] for t in terms)
        return CausalLMOutput(loss=loss, logits=None)


def llama_config(name: str = "llama3-8b", **overrides):
    """HF `LlamaConfig` presets for the benchmark / examples (random-init architectures)."""
    from transformers import LlamaConfig

    presets = {
        "llama3-8b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                          num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0, max_position_embeddings=8192,
                          rms_norm_eps=1e-5),
        "llama3.1-8b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                            num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0,
                            max_position_embeddings=131072, rms_norm_eps=1e-5,
                            rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                          "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
        "llama3.2-1b": dict(hidden_size=2048, intermediate_size=8192, num_hidden_layers=16, num_attention_heads=32,
                            num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0,
                            max_position_embeddings=131072, rms_norm_eps=1e-5, tie_word_embeddings=True,
                            rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                                          "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
        "llama3-70b": dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                           num_key_value_heads=8, vocab_size=128256, rope_theta=500000.0, max_position_embeddings=8192,
                           rms_norm_eps=1e-5),
        "llama2-7b": dict(hidden_size=4096, intermediate_size=11008, num_hidden_layers=32, num_attention_heads=32,
                          num_key_value_heads=32, vocab_size=32000, rope_theta=10000.0, max_position_embeddings=4096,
                          rms_norm_eps=1e-5),
        # CodeGen2.5-7B is a Llama-architecture model (reference: examples/training/codegen25/config.json)
        "codegen25-7b": dict(hidden_size=4096, intermediate_size=11008, num_hidden_layers=32, num_attention_heads=32,
                             num_key_value_heads=32, vocab_size=51200, rope_theta=10000.0,
                             max_position_embeddings=2048, rms_norm_eps=1e-6),
        "tiny": dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                     num_key_value_heads=2, vocab_size=1024, rope_theta=10000.0, max_position_embeddings=512,
                     rms_norm_eps=1e-5),
        # Llama-3-8B's head geometry scaled down (32 / 8 heads of 128 -> 16 / 8 of 64): TP = 8 keeps one
        # KV head per rank as the headline config does (multi-rank rehearsals, tests)
        "tiny8": dict(hidden_size=1024, intermediate_size=2048, num_hidden_layers=2, num_attention_heads=16,
                      num_key_value_heads=8, vocab_size=1024, rope_theta=10000.0, max_position_embeddings=512,
                      rms_norm_eps=1e-5),
    }
    kw = dict(presets[name])
    kw.setdefault("initializer_range", 0.02)
    kw.update(overrides)
    cfg = LlamaConfig(**kw)
    for k in ("sequence_parallel_enabled", "selective_checkpoint_enabled", "kv_shared_group_size",
              "activation_checkpoint"):
        if k in overrides:
            setattr(cfg, k, overrides[k])
    return cfg
