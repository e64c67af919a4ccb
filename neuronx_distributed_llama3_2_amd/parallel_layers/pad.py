"""Attention-head padding so #heads divides the TP degree (reference: parallel_layers/pad.py:10-107)."""

from __future__ import annotations

import torch
from torch import nn

from .layers import ColumnParallelLinear, RowParallelLinear
from .parallel_state import get_tensor_model_parallel_rank, get_tensor_model_parallel_size


def get_number_of_extra_heads(num_heads: int, tp_degree: int) -> int:
    return (tp_degree - num_heads % tp_degree) % tp_degree


def pad_model(model: nn.Module, tp_degree: int, n_heads: int, wrapped_classes=(), pad_hook_fn=None) -> nn.Module:
    """Zero-pad column-parallel output rows / row-parallel input columns of attention projections
    so a model with `n_heads` not divisible by `tp_degree` can be sharded.

    Each wrapped attention module (class in `wrapped_classes`) has its Column/Row linears' local
    shards extended by the per-rank share of `extra_heads * head_dim` zero rows (Column) / columns
    (Row); `pad_hook_fn(module, tgt_src_ratio)` lets a module update its own head counts.
    """
    extra = get_number_of_extra_heads(n_heads, tp_degree)
    if extra == 0:
        return model
    tgt_src_ratio = (n_heads + extra) / n_heads
    rank = get_tensor_model_parallel_rank()
    ws = get_tensor_model_parallel_size()

    def pad_linear(mod, dim):
        w = mod.weight
        full = w.shape[dim] * ws
        new_full = int(round(full * tgt_src_ratio))
        per_rank_new = new_full // ws
        add = per_rank_new - w.shape[dim]
        if add <= 0:
            return
        pad_shape = list(w.shape)
        pad_shape[dim] = add
        pad = torch.zeros(pad_shape, dtype=w.dtype, device=w.device)
        # padded heads live at the end of the global head range: ranks past the real heads get zeros
        new_w = torch.cat([w.data, pad], dim=dim)
        mod.weight = nn.Parameter(new_w, requires_grad=w.requires_grad)
        for a in ("tensor_model_parallel", "partition_dim", "partition_stride"):
            if hasattr(w, a):
                setattr(mod.weight, a, getattr(w, a))
        if dim == 0 and getattr(mod, "bias", None) is not None and mod.bias.shape[0] == w.shape[0]:
            b = mod.bias
            mod.bias = nn.Parameter(torch.cat([b.data, torch.zeros(add, dtype=b.dtype, device=b.device)]))
        if dim == 0:
            mod.output_size_per_partition = per_rank_new
        else:
            mod.input_size_per_partition = per_rank_new
        _ = rank

    for m in model.modules():
        if wrapped_classes and not isinstance(m, tuple(wrapped_classes)):
            continue
        for child in m.modules():
            if isinstance(child, ColumnParallelLinear):
                pad_linear(child, 0)
            elif isinstance(child, RowParallelLinear):
                pad_linear(child, 1)
        if pad_hook_fn is not None:
            pad_hook_fn(m, tgt_src_ratio)
    return model
