"""Dequantisation helpers (reference: src/neuronx_distributed/quantization/dequantize.py:3-32)."""

import torch


def direct_cast_dequantize(tensor: torch.Tensor, upcast_dtype: torch.dtype) -> torch.Tensor:
    return tensor.to(upcast_dtype)


def scale_dequantize(tensor: torch.Tensor, scale: torch.Tensor, upcast_dtype: torch.dtype) -> torch.Tensor:
    return (tensor.to(torch.float32) * scale.to(torch.float32)).to(upcast_dtype)
