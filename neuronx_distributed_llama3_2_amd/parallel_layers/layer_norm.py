"""Sequence-parallel-aware norms (reference: src/neuronx_distributed/parallel_layers/layer_norm.py:17-37).

`LayerNorm` tags its parameters `sequence_parallel_enabled` so their gradients are summed over TP
(grads.allreduce_sequence_parallel_gradients).  `RMSNorm` is the Llama norm on the fused CDNA4
kernel (optionally fused with the residual add: `forward(x, residual) -> (y, x + residual)`).
"""

from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .. import ops


class LayerNorm(nn.LayerNorm):
    def __init__(self, normalized_shape, eps: float = 1e-5, elementwise_affine: bool = True, bias: bool = True,
                 sequence_parallel_enabled: bool = False, device=None, dtype=None):
        super().__init__(normalized_shape, eps=eps, elementwise_affine=elementwise_affine, bias=bias, device=device,
                         dtype=dtype)
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if elementwise_affine:
            setattr(self.weight, "sequence_parallel_enabled", sequence_parallel_enabled)
            if self.bias is not None:
                setattr(self.bias, "sequence_parallel_enabled", sequence_parallel_enabled)


class RMSNorm(nn.Module):
    def __init__(self, hidden_size: int, eps: float = 1e-6, sequence_parallel_enabled: bool = False, dtype=torch.float32,
                 device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size, dtype=dtype, device=device))
        self.variance_epsilon = eps
        self.sequence_parallel_enabled = sequence_parallel_enabled
        setattr(self.weight, "sequence_parallel_enabled", sequence_parallel_enabled)

    def forward(self, hidden_states: torch.Tensor, residual: Optional[torch.Tensor] = None):
        y, h = ops.rms_norm(hidden_states, self.weight, self.variance_epsilon, residual)
        if residual is None:
            return y
        return y, h
