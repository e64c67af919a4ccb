"""Quantization utilities (reference: src/neuronx_distributed/quantization/quantization_utils.py:11-126).

`quantize_pytorch_model_per_{tensor,channel}_symmetric` quantize a model's plain nn.Linear AND
tensor-parallel linears to int8 weight-only layers (the reference goes through torch.ao dynamic
quantization of CPU nn.Linear modules and then converts qint8 state dicts; here the int8 tensor and
its fp32 scale are produced directly)."""

from __future__ import annotations

import copy

import torch
from torch import nn

from .quantization_config import QuantizationType, get_default_custom_qconfig_dict, \
    get_default_per_channel_custom_qconfig_dict
from .quantization_layers import quantize_symmetric
from .quantize import convert


class QuantizedLinear(nn.Module):
    """Weight-only int8 replacement of a plain nn.Linear (single device)."""

    def __init__(self, lin: nn.Linear, per_channel: bool):
        super().__init__()
        q, s = quantize_symmetric(lin.weight, 0 if per_channel else None)
        self.weight = nn.Parameter(q, requires_grad=False)
        self.scale = nn.Parameter(s.reshape(-1, 1) if per_channel else s, requires_grad=False)
        self.bias = None if lin.bias is None else nn.Parameter(lin.bias.detach().clone(), requires_grad=False)
        self.dtype = lin.weight.dtype
        self.in_features, self.out_features = lin.in_features, lin.out_features

    def forward(self, x):
        from ..ops.gemv import skinny_linear

        return skinny_linear(x.to(self.dtype) if x.dtype != self.dtype else x, self.weight,
                             self.scale.reshape(-1), self.bias)


def _quantize_linears(model: nn.Module, per_channel: bool) -> nn.Module:
    for name, child in list(model.named_children()):
        if type(child) is nn.Linear:
            model._modules[name] = QuantizedLinear(child, per_channel)
        else:
            _quantize_linears(child, per_channel)
    return model


def quantize_pytorch_model_per_tensor_symmetric(model: nn.Module, inplace: bool = False) -> nn.Module:
    model = model if inplace else copy.deepcopy(model)
    convert(model, get_default_custom_qconfig_dict(), inplace=True)
    return _quantize_linears(model, per_channel=False)


def quantize_pytorch_model_per_channel_symmetric(model: nn.Module, inplace: bool = False) -> nn.Module:
    model = model if inplace else copy.deepcopy(model)
    convert(model, get_default_per_channel_custom_qconfig_dict(), inplace=True)
    return _quantize_linears(model, per_channel=True)


def extract_q_scale_per_tensor(q_tensor: torch.Tensor) -> torch.Tensor:
    assert q_tensor.qscheme() == torch.per_tensor_affine
    return torch.tensor([q_tensor.q_scale()])


def extract_q_scale_per_channel(q_tensor: torch.Tensor) -> torch.Tensor:
    assert q_tensor.qscheme() == torch.per_channel_affine
    axis = q_tensor.q_per_channel_axis()
    shape = [1] * q_tensor.dim()
    shape[axis] = q_tensor.shape[axis]
    return q_tensor.q_per_channel_scales().to(torch.float32).view(shape)


def extract_q_scale(q_tensor: torch.Tensor) -> torch.Tensor:
    if q_tensor.qscheme() == torch.per_tensor_affine:
        return extract_q_scale_per_tensor(q_tensor)
    if q_tensor.qscheme() == torch.per_channel_affine:
        return extract_q_scale_per_channel(q_tensor)
    raise ValueError(f"qscheme {q_tensor.qscheme()} is not supported")


def convert_qint8_to_int8_state_dict(state_dict: dict) -> dict:
    """torch qint8 tensors -> (int8 tensor, '<prefix>scale') in place."""
    for k in list(state_dict):
        v = state_dict[k]
        if isinstance(v, torch.Tensor) and v.is_quantized:
            prefix = k.rsplit("weight", 1)[0]
            state_dict[prefix + "scale"] = extract_q_scale(v)
            state_dict[k] = v.int_repr()
    return state_dict
