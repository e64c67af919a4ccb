"""Per-channel symmetric abs-max observer (reference: src/neuronx_distributed/quantization/observer.py:12-166).

Tracks the running abs-max along every axis except `ch_axis` and produces symmetric int8
scales = absmax / 127 (zero point 0).  A plain nn.Module (no torch.ao quantized tensors)."""

from __future__ import annotations

from typing import Tuple

import torch
from torch import nn


class PerChannelAbsMaxObserver(nn.Module):
    def __init__(self, ch_axis: int = 0, dtype: torch.dtype = torch.int8, qscheme=torch.per_channel_symmetric,
                 quant_min: int = -127, quant_max: int = 127, eps: float = torch.finfo(torch.float32).eps, **kwargs):
        super().__init__()
        if qscheme != torch.per_channel_symmetric:
            raise NotImplementedError("only per_channel_symmetric is supported")
        self.ch_axis, self.dtype, self.qscheme = ch_axis, dtype, qscheme
        self.quant_min, self.quant_max, self.eps = quant_min, quant_max, eps
        self.register_buffer("max_val", torch.tensor([]))

    def forward(self, x_orig: torch.Tensor) -> torch.Tensor:
        if x_orig.numel() == 0:
            return x_orig
        x = x_orig.detach().float().movedim(self.ch_axis, 0).reshape(x_orig.shape[self.ch_axis], -1)
        cur = x.abs().amax(1)
        self.max_val = cur if self.max_val.numel() == 0 else torch.maximum(self.max_val, cur)
        return x_orig

    def calculate_qparams(self) -> Tuple[torch.Tensor, torch.Tensor]:
        scale = torch.clamp(self.max_val / ((self.quant_max - self.quant_min) / 2), min=self.eps)
        return scale, torch.zeros_like(scale, dtype=torch.int64)

    def reset_min_max_vals(self):
        self.max_val = torch.tensor([])

    def extra_repr(self):
        return f"ch_axis={self.ch_axis}, max_val={self.max_val}"

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "max_val"
        if key in state_dict:
            self.max_val = state_dict[key].clone()
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
