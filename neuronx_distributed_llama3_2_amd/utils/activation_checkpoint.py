"""Activation checkpointing (reference: src/neuronx_distributed/utils/activation_checkpoint.py:20-83).

Wraps modules matching `check_fn` so their forward is recomputed in backward
(torch.utils.checkpoint, non-reentrant).  On a 288 GB MI355X the Llama-3-8B TP=1 step fits without
any recompute, so the headline benchmark runs with checkpointing off; it is available for 70B /
long-sequence configurations.
"""

from __future__ import annotations

from typing import Callable

import torch
from torch import nn
from torch.utils.checkpoint import checkpoint


class NxDCheckpointWrapper(nn.Module):
    def __init__(self, module: nn.Module):
        super().__init__()
        self._checkpoint_wrapped_module = module

    def forward(self, *args, **kwargs):
        if not torch.is_grad_enabled():
            return self._checkpoint_wrapped_module(*args, **kwargs)
        return checkpoint(self._checkpoint_wrapped_module, *args, use_reentrant=False, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._checkpoint_wrapped_module, name)


def checkpoint_wrapper(module: nn.Module) -> nn.Module:
    return NxDCheckpointWrapper(module)


def apply_activation_checkpointing(model: nn.Module, check_fn: Callable[[nn.Module], bool] = lambda _: True) -> None:
    """Replace every submodule for which check_fn(m) is True by a checkpoint wrapper (in place)."""
    for name, child in list(model.named_children()):
        if isinstance(child, NxDCheckpointWrapper):
            continue
        if check_fn(child):
            setattr(model, name, checkpoint_wrapper(child))
        else:
            apply_activation_checkpointing(child, check_fn)
