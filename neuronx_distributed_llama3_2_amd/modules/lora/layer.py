"""LoRA adapters for plain torch layers (reference: src/neuronx_distributed/modules/lora/layer.py:15-424).

y = base(x) + scaling * B(A(dropout(x))), scaling = alpha / r (or alpha / sqrt(r) with rsLoRA);
merge() folds scaling * B @ A into the base weight (and unmerge() takes it back out).
"""

from __future__ import annotations

import math
import warnings
from typing import Any

import torch
import torch.nn.functional as F
from torch import nn

from .config import LoraConfig


class LoraLayer(nn.Module):
    def __init__(self, base_layer: nn.Module, lora_config: LoraConfig) -> None:
        super().__init__()
        self.base_layer = base_layer
        self.lora_rank = int(lora_config.lora_rank)
        self.lora_alpha = lora_config.lora_alpha
        self.scaling = self.lora_alpha / (math.sqrt(self.lora_rank) if lora_config.use_rslora else self.lora_rank)
        self.merged = False
        self.lora_config = lora_config
        self.in_features, self.out_features = self._features(base_layer)
        self.lora_dropout = nn.Dropout(p=lora_config.lora_dropout) if lora_config.lora_dropout > 0 else nn.Identity()

    @staticmethod
    def _features(base):
        if hasattr(base, "output_sizes"):   # fused GQA QKV
            return base.input_size, sum(base.output_sizes) if isinstance(base.output_sizes, (list, tuple)) else 0
        for a, b in (("in_features", "out_features"), ("input_size", "output_size"),
                     ("num_embeddings", "embedding_dim"), ("in_channels", "out_channels")):
            if hasattr(base, a):
                return getattr(base, a), getattr(base, b)
        raise ValueError(f"unsupported LoRA base layer {type(base).__name__}")

    def get_base_layer(self) -> nn.Module:
        return self.base_layer

    @property
    def weight(self):
        return self.base_layer.weight

    def _base_weight(self) -> torch.Tensor:
        return self.base_layer.weight

    def merge(self, safe_merge: bool = False) -> None:
        if self.merged:
            warnings.warn("Already merged. Nothing to do.")
            return
        w = self._base_weight()
        delta = self.get_delta_weight()
        new = w.data.float() + delta
        if safe_merge and not torch.isfinite(new).all():
            raise ValueError("NaNs detected in the merged weights")
        w.data.copy_(new.to(w.dtype))
        self.merged = True

    def unmerge(self) -> None:
        if not self.merged:
            warnings.warn("Already unmerged. Nothing to do.")
            return
        w = self._base_weight()
        w.data.copy_((w.data.float() - self.get_delta_weight()).to(w.dtype))
        self.merged = False

    def get_delta_weight(self) -> torch.Tensor:
        raise NotImplementedError

    def init_lora_parameters(self, init_lora_weights: str = "default"):
        init = str(init_lora_weights).lower()
        if init == "default":
            nn.init.kaiming_uniform_(self.lora_A.weight, a=math.sqrt(5))
        elif init == "gaussian":
            nn.init.normal_(self.lora_A.weight, std=1 / self.lora_rank)
        else:
            raise ValueError(f"Unknown LoRA parameters initialization with {init_lora_weights}")
        nn.init.zeros_(self.lora_B.weight)

    def __repr__(self) -> str:
        return "lora." + super().__repr__()


class LoraLinear(LoraLayer):
    def __init__(self, base_layer: nn.Linear, lora_config: LoraConfig, is_conv_1d_layer: bool = False) -> None:
        super().__init__(base_layer, lora_config)
        self.is_conv_1d_layer = is_conv_1d_layer
        self.update_layer(lora_config)

    def update_layer(self, lora_config: LoraConfig):
        dt = self.base_layer.weight.dtype
        dev = self.base_layer.weight.device
        self.lora_A = nn.Linear(self.in_features, self.lora_rank, bias=False, dtype=dt, device=dev)
        self.lora_B = nn.Linear(self.lora_rank, self.out_features, bias=False, dtype=dt, device=dev)
        self.init_lora_parameters(lora_config.init_lora_weights)

    def get_delta_weight(self) -> torch.Tensor:
        d = (self.lora_B.weight.float() @ self.lora_A.weight.float()) * self.scaling
        return d.t() if self.is_conv_1d_layer else d

    def forward(self, x: torch.Tensor, *args: Any, **kwargs: Any) -> torch.Tensor:
        out = self.base_layer(x, *args, **kwargs)
        if self.merged:
            return out
        return out + self.lora_B(self.lora_A(self.lora_dropout(x))) * self.scaling


class LoraEmbedding(LoraLayer):
    """A: [r, num_embeddings], B: [embedding_dim, r] (peft convention); delta = (B @ A)^T."""

    def __init__(self, base_layer: nn.Embedding, lora_config: LoraConfig) -> None:
        super().__init__(base_layer, lora_config)
        self.update_layer(lora_config)

    def update_layer(self, lora_config: LoraConfig):
        w = self.base_layer.weight
        self.lora_embedding_A = nn.Parameter(torch.zeros(self.lora_rank, w.shape[0], dtype=w.dtype, device=w.device))
        self.lora_embedding_B = nn.Parameter(torch.empty(w.shape[1], self.lora_rank, dtype=w.dtype, device=w.device))
        if str(lora_config.init_lora_weights).lower() == "gaussian":
            nn.init.normal_(self.lora_embedding_B, std=1 / self.lora_rank)
        else:
            nn.init.normal_(self.lora_embedding_B)

    def get_delta_weight(self) -> torch.Tensor:
        return (self.lora_embedding_B.float() @ self.lora_embedding_A.float()).t() * self.scaling

    def _embed(self, x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
        b = self.base_layer
        return F.embedding(x, weight, padding_idx=getattr(b, "padding_idx", None), max_norm=getattr(b, "max_norm", None),
                           norm_type=getattr(b, "norm_type", 2.0),
                           scale_grad_by_freq=getattr(b, "scale_grad_by_freq", False), sparse=getattr(b, "sparse", False))

    def forward(self, x: torch.Tensor, *args: Any, **kwargs: Any) -> torch.Tensor:
        out = self.base_layer(x, *args, **kwargs)
        if self.merged:
            return out
        after_a = self._embed(x, self.lora_embedding_A.t())
        return out + (after_a @ self.lora_embedding_B.t()) * self.scaling


class LoraConv2d(LoraLayer):
    def __init__(self, base_layer: nn.Conv2d, lora_config: LoraConfig) -> None:
        super().__init__(base_layer, lora_config)
        self.update_layer(lora_config)

    def update_layer(self, lora_config: LoraConfig):
        b = self.base_layer
        dt, dev = b.weight.dtype, b.weight.device
        self.lora_A = nn.Conv2d(self.in_features, self.lora_rank, b.kernel_size, b.stride, b.padding, bias=False,
                                dtype=dt, device=dev)
        self.lora_B = nn.Conv2d(self.lora_rank, self.out_features, (1, 1), (1, 1), bias=False, dtype=dt, device=dev)
        self.init_lora_parameters(lora_config.init_lora_weights)

    def get_delta_weight(self) -> torch.Tensor:
        wa, wb = self.lora_A.weight.float(), self.lora_B.weight.float()
        if tuple(self.base_layer.weight.shape[2:4]) == (1, 1):
            d = (wb.squeeze(3).squeeze(2) @ wa.squeeze(3).squeeze(2)).unsqueeze(2).unsqueeze(3)
        else:
            d = F.conv2d(wa.permute(1, 0, 2, 3), wb).permute(1, 0, 2, 3)
        return d * self.scaling

    def forward(self, x: torch.Tensor, *args, **kwargs) -> torch.Tensor:
        out = self.base_layer(x, *args, **kwargs)
        if self.merged:
            return out
        return out + self.lora_B(self.lora_A(self.lora_dropout(x))) * self.scaling
