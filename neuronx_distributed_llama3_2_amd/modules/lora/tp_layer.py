"""Tensor-parallel LoRA adapters (reference: src/neuronx_distributed/modules/lora/tp_layer.py:19-207).

The rank-r projection is placed on the cheap side of every collective:
* column-parallel base (incl. fused gate_up and the fused GQA QKV): A [r, in] is replicated and
  applied to the LOCAL sequence shard first, so sequence parallelism all-gathers a [S/tp, r] tensor
  instead of a second [S/tp, H] activation; B is sharded exactly like the base weight
  ([out/tp, r], same stride / QKV layout), so merge() is a local B @ A;
* row-parallel base: A [r, in/tp] is sharded like the base, its [S, r] partial sums are
  reduce-scattered (SP) or all-reduced, and the replicated B [out, r] produces the SP-local output.
Gradient bookkeeping follows the parallel attributes: shards are `tensor_model_parallel`,
replicated factors that see different tokens per TP rank are `sequence_parallel_enabled` (their
grads are summed over TP by the optimizer), the rest are plain replicated parameters.
"""

from __future__ import annotations

from typing import Any

import torch
from torch import nn

from ...parallel_layers import mappings
from ...parallel_layers import parallel_state as ps
from ...parallel_layers.layers import ColumnParallelLinear, RowParallelLinear
from ...parallel_layers.utils import set_tensor_model_parallel_attributes
from .config import LoraConfig
from .layer import LoraLayer


def _column_shard_B(base, full_B: torch.Tensor) -> torch.Tensor:
    """Shard a full [out, r] B like the base column weight (stride / fused-QKV aware)."""
    from ...parallel_layers.sharding import _attrs, shard_tensor

    return shard_tensor(full_B, _attrs(base.weight if hasattr(base, "weight") else base.weight_qkv),
                        ps.get_tensor_model_parallel_size(), ps.get_tensor_model_parallel_rank())


class LoraParallelLinear(LoraLayer):
    def __init__(self, base_layer: nn.Module, lora_config: LoraConfig) -> None:
        super().__init__(base_layer, lora_config)
        self.update_layer(lora_config)

    def update_layer(self, lora_config: LoraConfig):
        b = self.base_layer
        w = b.weight
        dt, dev = w.dtype, w.device
        self.is_row = isinstance(b, RowParallelLinear)
        self.sp = bool(getattr(b, "sequence_parallel_enabled", False)) and ps.get_tensor_model_parallel_size() > 1
        r = self.lora_rank
        if self.is_row:
            self.lora_A = nn.Linear(w.shape[1], r, bias=False, dtype=dt, device=dev)          # [r, in/tp]
            set_tensor_model_parallel_attributes(self.lora_A.weight, True, 1, 1)
            self.lora_B = nn.Linear(r, self.out_features, bias=False, dtype=dt, device=dev)  # [out, r]
            setattr(self.lora_B.weight, "sequence_parallel_enabled", self.sp)
        else:
            self.lora_A = nn.Linear(self.in_features, r, bias=False, dtype=dt, device=dev)   # [r, in]
            setattr(self.lora_A.weight, "sequence_parallel_enabled", self.sp)
            self.lora_B = nn.Linear(r, w.shape[0], bias=False, dtype=dt, device=dev)         # [out/tp, r]
            set_tensor_model_parallel_attributes(self.lora_B.weight, True, 0, getattr(b, "stride", 1))
        self.init_lora_parameters(lora_config.init_lora_weights)

    def get_delta_weight(self) -> torch.Tensor:
        return (self.lora_B.weight.float() @ self.lora_A.weight.float()) * self.scaling

    def _lora(self, x: torch.Tensor) -> torch.Tensor:
        x = self.lora_dropout(x)
        tp = ps.get_tensor_model_parallel_size()
        if self.is_row:
            if not self.base_layer.input_is_parallel:
                x = mappings.scatter_to_tensor_model_parallel_region(x)
            t = self.lora_A(x)                                                   # TP-partial [.., r]
            if self.sp:
                t = mappings.reduce_scatter_to_sequence_parallel_region(t)
            elif tp > 1:
                t = mappings.reduce_from_tensor_model_parallel_region(t)
            return self.lora_B(t)
        t = self.lora_A(x)                                                       # [.., r] on local tokens
        if self.sp:
            t = mappings.gather_from_sequence_parallel_region(t, to_model_parallel=True)
        elif tp > 1:
            t = mappings.copy_to_tensor_model_parallel_region(t)
        y = self.lora_B(t)
        if getattr(self.base_layer, "gather_output", False) and tp > 1:
            y = mappings.gather_from_tensor_model_parallel_region(y)
        return y

    def forward(self, x: torch.Tensor, *args: Any, **kwargs: Any):
        out = self.base_layer(x, *args, **kwargs)
        if self.merged:
            return out
        delta = self._lora(x) * self.scaling
        if isinstance(out, tuple):   # skip_bias_add
            return (out[0] + delta,) + tuple(out[1:])
        return out + delta


class LoraGQAQKVParallelLinear(LoraParallelLinear):
    """LoRA on the fused GQA QKV projection: B is laid out like weight_qkv ([q | k | v] local rows,
    K/V rows of replicated kv heads included)."""

    def update_layer(self, lora_config: LoraConfig):
        b = self.base_layer
        w, _ = b._fused_weight_bias()
        dt, dev = w.dtype, w.device
        self.is_row = False
        self.sp = bool(b.sequence_parallel_enabled) and ps.get_tensor_model_parallel_size() > 1
        r = self.lora_rank
        self.lora_A = nn.Linear(b.input_size, r, bias=False, dtype=dt, device=dev)
        setattr(self.lora_A.weight, "sequence_parallel_enabled", self.sp)
        self.lora_B = nn.Linear(r, w.shape[0], bias=False, dtype=dt, device=dev)
        set_tensor_model_parallel_attributes(self.lora_B.weight, True, 0, 1)
        setattr(self.lora_B.weight, "qkv_split", getattr(w, "qkv_split", None))
        self.in_features = b.input_size
        self.out_features = sum(b.output_sizes)
        self.init_lora_parameters(lora_config.init_lora_weights)
        if getattr(b, "kv_size_multiplier", 1) > 1:
            # K/V rows of B belong to replicated kv heads: keep the replicas identical by summing
            # their gradients over the kv-shared group (as the base projection does)
            q_l = b.q_output_size_per_partition

            def _sum_kv(grad, q_l=q_l):
                from ..qkv_linear import get_kv_shared_group
                import torch.distributed as dist

                g = grad.clone()
                kv = g[q_l:].contiguous()
                dist.all_reduce(kv, group=get_kv_shared_group())
                g[q_l:] = kv
                return g

            self.lora_B.weight.register_hook(_sum_kv)

    def _base_weight(self):
        return self.base_layer._fused_weight_bias()[0] if self.base_layer.fuse_qkv else None

    def merge(self, safe_merge: bool = False) -> None:
        if self.base_layer.fuse_qkv:
            return super().merge(safe_merge)
        d = self.get_delta_weight()
        q_l, kv_l = self.base_layer.q_output_size_per_partition, self.base_layer.kv_output_size_per_partition
        for wt, sl in ((self.base_layer.weight_q, d[:q_l]), (self.base_layer.weight_k, d[q_l:q_l + kv_l]),
                       (self.base_layer.weight_v, d[q_l + kv_l:])):
            wt.data.copy_((wt.data.float() + sl).to(wt.dtype))
        self.merged = True

    def unmerge(self) -> None:
        if self.base_layer.fuse_qkv:
            return super().unmerge()
        d = self.get_delta_weight()
        q_l, kv_l = self.base_layer.q_output_size_per_partition, self.base_layer.kv_output_size_per_partition
        for wt, sl in ((self.base_layer.weight_q, d[:q_l]), (self.base_layer.weight_k, d[q_l:q_l + kv_l]),
                       (self.base_layer.weight_v, d[q_l + kv_l:])):
            wt.data.copy_((wt.data.float() - sl).to(wt.dtype))
        self.merged = False

    def forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        out = self.base_layer.forward_fused(x)
        if self.merged:
            return out
        return out + self._lora(x) * self.scaling

    def forward(self, x: torch.Tensor, *args, **kwargs):
        fused = self.forward_fused(x)
        b = self.base_layer
        q_l, kv_l = b.q_output_size_per_partition, b.kv_output_size_per_partition
        q, k, v = fused[..., :q_l], fused[..., q_l:q_l + kv_l], fused[..., q_l + kv_l:]
        if b.gather_output and ps.get_tensor_model_parallel_size() > 1:
            q = mappings.gather_from_tensor_model_parallel_region(q)
            k = mappings.gather_from_tensor_model_parallel_region(k)
            v = mappings.gather_from_tensor_model_parallel_region(v)
        return q, k, v

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            if name == "base_layer":
                raise
            return getattr(self.base_layer, name)


class LoraParallelEmbedding(LoraLayer):
    """LoRA on a vocab-sharded ParallelEmbedding: A [r, V/tp] (sharded like the base), B [H, r]
    replicated; the masked lookup of A's columns is reduced over TP as a [.., r] tensor."""

    def __init__(self, base_layer: nn.Module, lora_config: LoraConfig) -> None:
        super().__init__(base_layer, lora_config)
        w = base_layer.weight
        self.sp = bool(getattr(base_layer, "sequence_parallel_enabled", False)) and \
            ps.get_tensor_model_parallel_size() > 1
        self.lora_embedding_A = nn.Parameter(torch.zeros(self.lora_rank, w.shape[0], dtype=w.dtype, device=w.device))
        set_tensor_model_parallel_attributes(self.lora_embedding_A, True, 1, 1)
        self.lora_embedding_B = nn.Parameter(torch.empty(w.shape[1], self.lora_rank, dtype=w.dtype, device=w.device))
        setattr(self.lora_embedding_B, "sequence_parallel_enabled", self.sp)
        nn.init.normal_(self.lora_embedding_B, std=1 / self.lora_rank
                        if str(lora_config.init_lora_weights).lower() == "gaussian" else 1.0)

    def get_delta_weight(self) -> torch.Tensor:
        return (self.lora_embedding_B.float() @ self.lora_embedding_A.float()).t() * self.scaling

    def forward(self, x: torch.Tensor, *args, **kwargs):
        out = self.base_layer(x, *args, **kwargs)
        if self.merged:
            return out
        b = self.base_layer
        local = x - b.start_index
        mask = (local >= 0) & (local < b.num_embeddings_per_partition)
        a = torch.nn.functional.embedding(local.clamp(0, b.num_embeddings_per_partition - 1),
                                          self.lora_embedding_A.t()) * mask.unsqueeze(-1).to(out.dtype)
        if self.sp:
            a = mappings.reduce_scatter_to_sequence_parallel_region(a)
        elif ps.get_tensor_model_parallel_size() > 1:
            a = mappings.reduce_from_tensor_model_parallel_region(a)
        return out + (a @ self.lora_embedding_B.t()) * self.scaling
