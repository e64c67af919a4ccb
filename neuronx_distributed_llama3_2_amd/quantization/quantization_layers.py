"""int8 weight-only quantized tensor-parallel linears
(reference: src/neuronx_distributed/quantization/quantization_layers.py:60-890).

Weights are stored as int8 shards with fp32 symmetric scales (per tensor [1], or per output
channel [out, 1] — sharded with the weight when the channel axis is the partition dim).  The matmul:
* token generation (<= 8 rows): the int8 skinny-GEMM kernel (csrc/gemv.hip) reads the int8 weight
  directly and applies the scale in the epilogue — half the HBM bytes of bf16 decode;
* prefill / training-size inputs: one int8 -> bf16 dequantisation kernel, then the tuned GEMM.
Same collectives as the float layers (TP all-reduce / SP reduce-scatter / gather_output).
"""

from __future__ import annotations

from typing import Any, Optional

import torch
from torch import nn
from torch.nn.parameter import Parameter

from ..modules.moe.moe_parallel_layers import ExpertFusedColumnParallelLinear, ExpertFusedRowParallelLinear
from ..ops.gemv import dequantize_weight, skinny_linear
from ..parallel_layers import mappings
from ..parallel_layers import parallel_state as ps
from ..parallel_layers import sp
from ..parallel_layers.layers import ColumnParallelLinear, RowParallelLinear
from ..parallel_layers.utils import divide, set_tensor_model_parallel_attributes
from .quantization_config import (
    BASE_QCONFIG_DICT_TYPE,
    QuantizationType,
    QuantizedDtype,
    get_default_custom_qconfig_dict,
)


def quantize_symmetric(w: torch.Tensor, per_channel_axis: Optional[int] = None):
    """float -> (int8, fp32 scale): scale = absmax / 127 over the tensor or per channel."""
    wf = w.detach().float()
    if per_channel_axis is None:
        scale = (wf.abs().max() / 127.0).clamp(min=1e-12).reshape(1)
        q = torch.round(wf / scale).clamp(-127, 127).to(torch.int8)
        return q, scale
    red = [d for d in range(wf.dim()) if d != per_channel_axis]
    amax = wf.abs().amax(dim=red, keepdim=True)
    scale = (amax / 127.0).clamp(min=1e-12)
    q = torch.round(wf / scale).clamp(-127, 127).to(torch.int8)
    return q, scale


class QuantizedParallelLinearLayerStateDictAdaptor:
    """Accepts float or int8 weights in a state dict; float ones are quantized on load."""

    @staticmethod
    def get_weight_from_state_dict(prefix: str, state_dict: dict) -> torch.Tensor:
        for k in (prefix + "weight", prefix + "_packed_params.weight"):
            if k in state_dict:
                return state_dict[k]
        raise RuntimeError(f"Cannot find weight in state dict for prefix {prefix}")

    @staticmethod
    def get_scale_from_state_dict(prefix: str, state_dict: dict) -> Optional[torch.Tensor]:
        return state_dict.get(prefix + "scale")


class BaseQuantizeParallelLinear(nn.Module):
    def _setup_q(self, q_config: Optional[BASE_QCONFIG_DICT_TYPE], weight_shape, partition_dim: int, stride: int,
                 device, is_expert: bool = False):
        q_config = q_config or get_default_custom_qconfig_dict()
        qt = q_config["quantization_type"]
        self.quantization_type = QuantizationType(qt) if not isinstance(qt, QuantizationType) else qt
        qd = q_config.get("quantized_dtype", QuantizedDtype.INT8)
        self.quantized_dtype = qd.value if isinstance(qd, QuantizedDtype) else qd
        assert self.quantized_dtype == torch.int8, "only int8 weight-only quantization is supported"
        self.per_channel_axis = q_config.get("quantization_per_channel_axis", 0) \
            if self.quantization_type == QuantizationType.PER_CHANNEL_SYMMETRIC else None
        self.weight = Parameter(torch.zeros(weight_shape, dtype=torch.int8, device=device), requires_grad=False)
        set_tensor_model_parallel_attributes(self.weight, True, partition_dim, stride)
        if self.per_channel_axis is None:
            self.scale = Parameter(torch.ones(1, dtype=torch.float32, device=device), requires_grad=False)
        else:
            shape = [1] * len(weight_shape)
            shape[self.per_channel_axis] = weight_shape[self.per_channel_axis]
            self.scale = Parameter(torch.ones(shape, dtype=torch.float32, device=device), requires_grad=False)
            if self.per_channel_axis == partition_dim:
                set_tensor_model_parallel_attributes(self.scale, True, partition_dim, stride)

    def quantize_from(self, w_float: torch.Tensor) -> None:
        """Quantise a float weight of this layer's (local) shape into the int8 weight + scale."""
        q, s = quantize_symmetric(w_float, self.per_channel_axis)
        with torch.no_grad():
            self.weight.copy_(q.to(self.weight.device))
            self.scale.copy_(s.reshape(self.scale.shape).to(self.scale.device))

    def _row_scale(self) -> torch.Tensor:
        """Scale as one fp32 value per output row of the [out, in] weight."""
        if self.per_channel_axis is None:
            return self.scale.reshape(1)
        assert self.per_channel_axis == 0, "per-channel scales must be along the output dim"
        return self.scale.reshape(-1)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        wk = prefix + "weight"
        if wk in state_dict and state_dict[wk].is_floating_point():
            q, s = quantize_symmetric(state_dict[wk], self.per_channel_axis)
            state_dict[wk] = q
            state_dict[prefix + "scale"] = s.reshape(self.scale.shape)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def _matmul(self, x: torch.Tensor) -> torch.Tensor:
        return skinny_linear(x, self.weight, self._row_scale())


class QuantizedColumnParallel(BaseQuantizeParallelLinear):
    def __init__(self, input_size: int, output_size: int, bias: bool = True, gather_output: bool = True,
                 dtype: torch.dtype = torch.bfloat16, device: Optional[torch.device] = None, stride: int = 1,
                 sequence_parallel_enabled: bool = False, keep_master_weight: bool = False,
                 quantization_type: Any = None, quantized_dtype: Any = QuantizedDtype.INT8,
                 quantization_per_channel_axis: Optional[int] = None, q_config: Optional[dict] = None, **kw):
        super().__init__()
        tp = ps.get_tensor_model_parallel_size()
        self.input_size, self.output_size = input_size, output_size
        self.output_size_per_partition = divide(output_size, tp)
        self.gather_output, self.stride, self.dtype = gather_output, stride, dtype
        self.sequence_parallel_enabled = sequence_parallel_enabled and tp > 1
        q_config = q_config or _qc(quantization_type, quantized_dtype, quantization_per_channel_axis)
        self._setup_q(q_config, (self.output_size_per_partition, input_size), 0, stride, device)
        if bias:
            self.bias = Parameter(torch.zeros(self.output_size if gather_output else self.output_size_per_partition,
                                              dtype=dtype, device=device), requires_grad=False)
            if not gather_output:
                set_tensor_model_parallel_attributes(self.bias, True, 0, stride)
        else:
            self.register_parameter("bias", None)

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        x = sp.sp_gather(input) if self.sequence_parallel_enabled else input
        out = self._matmul(x.to(self.dtype) if x.dtype != self.dtype else x)
        if self.gather_output and ps.get_tensor_model_parallel_size() > 1:
            out = mappings.gather_from_tensor_model_parallel_region(out)
        return out + self.bias if self.bias is not None else out

    @classmethod
    def from_float(cls, mod: ColumnParallelLinear, q_config: BASE_QCONFIG_DICT_TYPE = None):
        new = cls(mod.input_size, mod.output_size, bias=mod.bias is not None, gather_output=mod.gather_output,
                  dtype=mod.weight.dtype if mod.weight.is_floating_point() else torch.bfloat16,
                  device=mod.weight.device, stride=mod.stride,
                  sequence_parallel_enabled=mod.sequence_parallel_enabled, q_config=q_config)
        if mod.weight.device.type != "meta":
            new.quantize_from(mod.weight)
            if mod.bias is not None:
                with torch.no_grad():
                    new.bias.copy_(mod.bias)
        return new


class QuantizedRowParallel(BaseQuantizeParallelLinear):
    def __init__(self, input_size: int, output_size: int, bias: bool = True, input_is_parallel: bool = False,
                 dtype: torch.dtype = torch.bfloat16, device: Optional[torch.device] = None, stride: int = 1,
                 sequence_parallel_enabled: bool = False, keep_master_weight: bool = False,
                 quantization_type: Any = None, quantized_dtype: Any = QuantizedDtype.INT8,
                 quantization_per_channel_axis: Optional[int] = None, q_config: Optional[dict] = None, **kw):
        super().__init__()
        tp = ps.get_tensor_model_parallel_size()
        self.input_size, self.output_size = input_size, output_size
        self.input_size_per_partition = divide(input_size, tp)
        self.input_is_parallel, self.stride, self.dtype = input_is_parallel, stride, dtype
        self.sequence_parallel_enabled = sequence_parallel_enabled and tp > 1
        q_config = q_config or _qc(quantization_type, quantized_dtype, quantization_per_channel_axis)
        self._setup_q(q_config, (output_size, self.input_size_per_partition), 1, stride, device)
        if bias:
            self.bias = Parameter(torch.zeros(output_size, dtype=dtype, device=device), requires_grad=False)
        else:
            self.register_parameter("bias", None)

    def forward(self, input_: torch.Tensor) -> torch.Tensor:
        x = input_ if self.input_is_parallel else mappings.scatter_to_tensor_model_parallel_region(input_)
        out = self._matmul(x.to(self.dtype) if x.dtype != self.dtype else x)
        if self.sequence_parallel_enabled:
            out = sp.sp_reduce_scatter(out)
        elif ps.get_tensor_model_parallel_size() > 1:
            out = mappings.reduce_from_tensor_model_parallel_region(out)
        return out + self.bias if self.bias is not None else out

    @classmethod
    def from_float(cls, mod: RowParallelLinear, q_config: BASE_QCONFIG_DICT_TYPE = None):
        new = cls(mod.input_size, mod.output_size, bias=mod.bias is not None, input_is_parallel=mod.input_is_parallel,
                  dtype=mod.weight.dtype if mod.weight.is_floating_point() else torch.bfloat16,
                  device=mod.weight.device, stride=mod.stride,
                  sequence_parallel_enabled=mod.sequence_parallel_enabled, q_config=q_config)
        if mod.weight.device.type != "meta":
            new.quantize_from(mod.weight)
            if mod.bias is not None:
                with torch.no_grad():
                    new.bias.copy_(mod.bias)
        return new


class _QuantizedExpertFused(nn.Module):
    """int8 3-D expert weights [E, in, out] (+ scale per expert [E, 1, 1] or per out channel [E, 1, out])."""

    def _init_q(self, mod, q_config):
        q_config = q_config or get_default_custom_qconfig_dict()
        qt = q_config["quantization_type"]
        self.quantization_type = QuantizationType(qt) if not isinstance(qt, QuantizationType) else qt
        w = mod.weight
        self.num_experts = mod.num_experts
        self.weight = Parameter(torch.zeros(w.shape, dtype=torch.int8, device=w.device if w.device.type != "meta" else None),
                                requires_grad=False)
        for a in ("tensor_model_parallel", "partition_dim", "partition_stride", "expert_model_parallel"):
            if hasattr(w, a):
                setattr(self.weight, a, getattr(w, a))
        per_ch = self.quantization_type == QuantizationType.PER_CHANNEL_SYMMETRIC
        sshape = (w.shape[0], 1, w.shape[2]) if per_ch else (w.shape[0], 1, 1)
        self.scale = Parameter(torch.ones(sshape, dtype=torch.float32, device=self.weight.device), requires_grad=False)
        if w.device.type != "meta":
            wf = w.detach().float()
            amax = wf.abs().amax(dim=1, keepdim=True) if per_ch else wf.abs().amax(dim=(1, 2), keepdim=True)
            s = (amax / 127.0).clamp(min=1e-12)
            with torch.no_grad():
                self.weight.copy_(torch.round(wf / s).clamp(-127, 127).to(torch.int8))
                self.scale.copy_(s)
        self.dtype = w.dtype if w.is_floating_point() else torch.bfloat16

    def _w(self, expert_indices=None):
        w, s = (self.weight, self.scale) if expert_indices is None else (self.weight[expert_indices], self.scale[expert_indices])
        return (w.float() * s).to(self.dtype)


class QuantizedExpertFusedColumnParallel(_QuantizedExpertFused):
    def __init__(self, mod: ExpertFusedColumnParallelLinear, q_config=None):
        super().__init__()
        self._init_q(mod, q_config)
        self.async_tensor_model_parallel_allreduce = False

    def forward(self, input_, expert_indices=None):
        w = self._w(expert_indices)
        E = w.shape[0]
        x = input_.expand((E,) + tuple(input_.shape[1:])) if input_.shape[0] == 1 and E > 1 else input_
        return torch.bmm(x.reshape(E, -1, x.shape[-1]), w).view(tuple(x.shape[:-1]) + (w.shape[-1],))

    @classmethod
    def from_float(cls, mod, q_config=None):
        return cls(mod, q_config)


class QuantizedExpertFusedRowParallel(QuantizedExpertFusedColumnParallel):
    def __init__(self, mod: ExpertFusedRowParallelLinear, q_config=None):
        super().__init__(mod, q_config)
        self.reduce_output = getattr(mod, "reduce_output", True)

    def forward(self, input_, expert_indices=None):
        out = super().forward(input_, expert_indices)
        if self.reduce_output and ps.get_tensor_model_parallel_size() > 1:
            out = mappings.reduce_from_tensor_model_parallel_region(out)
        return out


def _qc(quantization_type, quantized_dtype, axis):
    if quantization_type is None:
        return get_default_custom_qconfig_dict()
    d = {"quantization_type": QuantizationType(quantization_type) if not isinstance(quantization_type, QuantizationType)
         else quantization_type, "quantized_dtype": quantized_dtype}
    if d["quantization_type"] == QuantizationType.PER_CHANNEL_SYMMETRIC:
        d["quantization_per_channel_axis"] = 0 if axis is None else axis
    return d
