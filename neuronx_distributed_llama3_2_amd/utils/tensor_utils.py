"""Tensor helpers (reference: src/neuronx_distributed/utils/tensor_utils.py:4-62).

The reference computes a blocked fp64 cumsum through lower-triangular matmuls because its
compiler lacks an exact scan; on MI355X `torch.cumsum` is a native exact scan (int64 / fp32
accumulate), so `cumsum` keeps the reference signature but uses it directly (integer inputs such
as MoE expert-assignment masks are summed in int64, floating inputs in fp32 or wider)."""

from __future__ import annotations

import torch


def cumsum(tensor: torch.Tensor, dim: int = 0, tril_size: int = 2048) -> torch.Tensor:
    if tensor.dim() != 2:
        raise ValueError(f"Expected 2D input tensor, unsupported shape: {tuple(tensor.shape)}")
    if dim != 0:
        raise NotImplementedError(f"Only cumsum along dimension-0 is currently supported, unexpected dim={dim}")
    if tensor.dtype.is_floating_point:
        acc = torch.float64 if tensor.dtype == torch.float64 else torch.float32
        return torch.cumsum(tensor, dim=0, dtype=acc).to(tensor.dtype)
    return torch.cumsum(tensor, dim=0, dtype=torch.int64).to(tensor.dtype)
