"""Vocab-parallel cross entropy (reference: src/neuronx_distributed/parallel_layers/loss_functions.py:11-135).

`parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing=0.0)` returns the per-token
loss for logits sharded along the vocabulary over the TP group.  On the GPU it runs the fused
CDNA4 kernels (ops/cross_entropy.py: one statistics pass + one all-gather of [N, 4] fp32 instead
of three all-reduces over an fp64 copy of the logits); on the CPU it runs the same math in torch.
"""

from __future__ import annotations

import torch

from ..ops.cross_entropy import vocab_parallel_cross_entropy
from .parallel_state import (
    get_tensor_model_parallel_group,
    get_tensor_model_parallel_rank,
    get_tensor_model_parallel_size,
    model_parallel_is_initialized,
)


def parallel_cross_entropy(vocab_parallel_logits: torch.Tensor, target: torch.Tensor, label_smoothing: float = 0.0,
                           ignore_index: int = -100, inplace_backward: bool = False) -> torch.Tensor:
    if model_parallel_is_initialized():
        group = get_tensor_model_parallel_group()
        world = get_tensor_model_parallel_size()
        rank = get_tensor_model_parallel_rank()
    else:
        group, world, rank = None, 1, 0
    return vocab_parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing, ignore_index, group, world, rank,
                                        inplace_backward)
