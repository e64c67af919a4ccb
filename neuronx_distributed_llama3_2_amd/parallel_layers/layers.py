"""Tensor-parallel layers: ColumnParallelLinear, RowParallelLinear, ParallelEmbedding and the
channel-parallel Conv2d pair (reference: src/neuronx_distributed/parallel_layers/layers.py:101-1235).

Constructor kwargs and parameter attributes (`tensor_model_parallel`, `partition_dim`,
`partition_stride`, `sequence_parallel_enabled`) match the reference so checkpoints and
converters line up.  The compute path is MI355X-first:

* GEMMs go to hipBLASLt (torch.matmul on bf16, MFMA), the collectives to RCCL over xGMI;
* sequence parallel (activations sharded along dim 0 = sequence of [S, B, H]): the column layer
  all-gathers its input once in forward and KEEPS the gathered input for the weight-gradient GEMM
  (HBM is plentiful on a 288 GB part: this removes the reference's backward re-gather, X7), and its
  backward reduce-scatter of dX runs asynchronously on RCCL's stream while the dW GEMM runs;
* without SP the column backward all-reduce of dX likewise overlaps the dW GEMM;
* weight gradients accumulate straight into an fp32 `main_grad` buffer when the parameter has one
  (fp32-output GEMM `addmm(out_dtype=float32, beta=1)`), the hook that drives bucketed data-parallel
  reduction (parallel/grad_buffer.py) fires right after.
"""

from __future__ import annotations

import math
import os
import warnings
from typing import Any, Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel import comm
import torch.nn.functional as F
from torch import nn
from torch.nn.parameter import Parameter

from .. import ops
from ..ops import gemm as _gemm
from ..ops.activations import attached_token_major
from . import stream_split
from . import sp
from .mappings import (
    _gather_along_first_dim,
    copy_to_tensor_model_parallel_region,
    gather_from_tensor_model_parallel_region,
    reduce_from_tensor_model_parallel_region,
    reduce_scatter_to_sequence_parallel_region,
    scatter_input_channels_to_tensor_model_parallel_region,
    scatter_to_tensor_model_parallel_region,
)
from .parallel_state import get_tensor_model_parallel_group, get_tensor_model_parallel_rank, get_tensor_model_parallel_size
from .random import get_rng_tracker
from .utils import EmbeddingUtility, divide, get_padding_length, set_tensor_model_parallel_attributes

_SAVE_GATHERED_INPUT = os.environ.get("NXD_SP_SAVE_GATHERED_INPUT", "1") == "1"


def create_local_weight(full_weight: torch.Tensor, partition_dim: int, per_partition_size: int, stride: int,
                        out_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    """This rank's strided shard of a full weight (reference layers.py:58-66): split into
    `per_partition_size / stride` chunks and take chunks rank, rank + tp, ..."""
    per_stride = divide(per_partition_size, stride)
    chunks = torch.split(full_weight, per_stride, dim=partition_dim)
    rank, ws = get_tensor_model_parallel_rank(), get_tensor_model_parallel_size()
    mine = chunks[rank::ws]
    with torch.no_grad():
        if out_weight is not None:
            return torch.cat(mine, dim=partition_dim, out=out_weight)
        return torch.cat(mine, dim=partition_dim)


def _initialize_parameter(param: torch.Tensor, partition_dim: int, init_method: Callable, stride: int = 1,
                          return_master_param: bool = False) -> Optional[torch.Tensor]:
    """Initialise the FULL weight in fp32 (same values on every TP rank for a given seed) and keep
    this rank's shard — so results are independent of the TP degree."""
    set_tensor_model_parallel_attributes(param, True, partition_dim, stride)
    if param.device.type == "meta":
        return None
    shape = list(param.shape)
    shape[partition_dim] *= get_tensor_model_parallel_size()
    master = torch.empty(shape, dtype=torch.float32, device=param.device)
    init_method(master)
    create_local_weight(master.to(param.dtype), partition_dim, param.shape[partition_dim], stride, out_weight=param.data)
    return master if return_master_param else None


def _notify(param):
    cb = getattr(param, "_nxd_grad_ready", None)
    if cb is not None:
        cb(param)


def _accumulate_wgrad(weight: torch.Tensor, go2: torch.Tensor, x2, go_t: torch.Tensor = None,
                      x_t: torch.Tensor = None):
    """dW = go2^T @ x2; accumulated into weight.main_grad (fp32) if present, else returned.
    `go_t` / `x_t` are optional producer-written transposes of go2 / x2 (see ops/activations.py);
    x2 may be None when only x_t was saved."""
    mg = getattr(weight, "main_grad", None)
    if mg is None:
        return go2.t().matmul(x2 if x2 is not None else x_t.t())
    stream_split.accumulate_begin(weight)
    _gemm.wgrad_accumulate_(mg, go2, x2, go_t=go_t, x_t=x_t)
    stream_split.accumulate_end(weight)
    _notify(weight)
    return None


def _token_major_copy(x: torch.Tensor):
    """The producer-written [K, tokens] copy of activation x ([..., K]) if one is attached."""
    t = attached_token_major(x)
    if t is None or t.dim() != 2 or not t.is_contiguous() or x.dim() < 1:
        return None
    K = x.shape[-1]
    return t if t.shape == (K, x.numel() // max(K, 1)) else None


def _bias_grad(bias, go2):
    if bias is None:
        return None
    g = go2.sum(0)
    mg = getattr(bias, "main_grad", None)
    if mg is not None:
        stream_split.accumulate_begin(bias)
        mg.add_(g.float())
        stream_split.accumulate_end(bias)
        _notify(bias)
        return None
    return g.to(bias.dtype)


class LinearWithAsyncCommunication(torch.autograd.Function):
    """Y = X W^T (+ b) with the column-parallel input collectives fused into fwd/bwd.

    Sequence parallel: the input all-gather is chunk-pipelined with the GEMM (sp.gather_linear)
    and the backward input-gradient reduce-scatter is chunk-pipelined with the dgrad GEMM and
    overlapped with the weight-gradient GEMM (sp.matmul_reduce_scatter_start)."""

    @staticmethod
    def forward(ctx, input, weight, bias, async_grad_allreduce, sequence_parallel_enabled, save_for_backward=True,
                process_group=None):
        ctx.use_bias = bias is not None
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sequence_parallel_enabled = sequence_parallel_enabled
        ctx.process_group = process_group
        if sequence_parallel_enabled:
            output, total_input = sp.gather_linear(input, weight, process_group)
        else:
            total_input = input
            output = _gemm.linear(total_input, weight)
        ctx.saved_gathered = sequence_parallel_enabled and _SAVE_GATHERED_INPUT
        # a token-major copy of the input written by its producer (SwiGLU forward) is saved
        # INSTEAD of the input: the weight gradient is the only backward use of it
        x_t = _token_major_copy(input) if not sequence_parallel_enabled else None
        ctx.x_is_t = x_t is not None
        if save_for_backward:
            if ctx.x_is_t:
                ctx.save_for_backward(x_t, weight, bias)
            else:
                ctx.save_for_backward(total_input if (ctx.saved_gathered or not sequence_parallel_enabled) else input,
                                      weight, bias)
        if bias is not None:
            output = output + bias
        return output

    @staticmethod
    def backward(ctx, grad_output):
        inp, weight, bias = ctx.saved_tensors
        x_t = None
        if ctx.x_is_t:
            x_t, total_input = inp, None
        elif ctx.sequence_parallel_enabled and not ctx.saved_gathered:
            total_input = sp.sp_gather(inp, ctx.process_group)
        else:
            total_input = inp
        go_t = attached_token_major(grad_output)   # token-contiguous copy from the SwiGLU backward
        grad_output = grad_output.contiguous()
        group = ctx.process_group if ctx.process_group is not None else get_tensor_model_parallel_group()
        handles = []
        if ctx.sequence_parallel_enabled and dist.get_world_size(group=group) > 1:
            grad_input, handles = sp.matmul_reduce_scatter_start(grad_output, weight, group)
        else:
            grad_input = _gemm.dgrad(grad_output, weight)
            if not ctx.sequence_parallel_enabled and ctx.async_grad_allreduce and dist.get_world_size(group=group) > 1:
                handles = [dist.all_reduce(grad_input, group=group, async_op=True)]
        go2 = grad_output.reshape(-1, grad_output.shape[-1])
        x2 = total_input.reshape(-1, total_input.shape[-1]) if total_input is not None else None
        grad_weight = _accumulate_wgrad(weight, go2, x2, go_t=go_t, x_t=x_t) if ctx.needs_input_grad[1] else None
        grad_bias = _bias_grad(bias, go2) if ctx.use_bias else None
        for h in handles:
            h.wait()
        return grad_input, grad_weight, grad_bias, None, None, None, None


class RowParallelSPLinear(torch.autograd.Function):
    """Row-parallel linear with sequence parallelism: reduce_scatter(X W^T), the reduce-scatter of
    each sequence chunk overlapping the GEMM of the next; backward all-gathers the output grad
    chunk-pipelined with the dgrad GEMM."""

    @staticmethod
    def forward(ctx, input, weight, process_group=None):
        ctx.process_group = process_group
        local, hs = sp.linear_reduce_scatter_start(input, weight, process_group)
        x_t = _token_major_copy(input)
        ctx.x_is_t = x_t is not None
        ctx.save_for_backward(x_t if ctx.x_is_t else input, weight)
        for h in hs:
            h.wait()
        return local

    @staticmethod
    def backward(ctx, grad_output):
        inp, weight = ctx.saved_tensors
        grad_input, g_full = sp.gather_matmul(grad_output.contiguous(), weight, ctx.process_group)
        go2 = g_full.reshape(-1, g_full.shape[-1])
        x_t = inp if ctx.x_is_t else None
        x2 = None if ctx.x_is_t else inp.reshape(-1, inp.shape[-1])
        grad_weight = _accumulate_wgrad(weight, go2, x2, x_t=x_t) if ctx.needs_input_grad[1] else None
        return grad_input, grad_weight, None


def linear_with_async_allreduce(input, weight, bias, async_grad_allreduce, sequence_parallel_enabled,
                                autograd_func_class=LinearWithAsyncCommunication, save_for_backward=True,
                                process_group=None):
    return autograd_func_class.apply(input, weight, bias, async_grad_allreduce, sequence_parallel_enabled,
                                     save_for_backward, process_group)


class BaseParallelLinear(nn.Module):
    autograd_func_class = LinearWithAsyncCommunication

    def _init_weight(self, weight: torch.Tensor) -> None:
        if self.arg_init_method is None:
            nn.init.kaiming_uniform_(weight, a=math.sqrt(5))
        else:
            self.arg_init_method(weight)

    def _init_bias(self) -> None:
        fan_in = self.weight.shape[1] if self.weight.dim() > 1 else 1
        bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
        with torch.no_grad():
            nn.init.uniform_(self.bias, -bound, bound)


def _device_of(device):
    if device is None:
        return torch.device("cpu")
    return torch.device(device)


class ColumnParallelLinear(BaseParallelLinear):
    """Y = X A + b with A split along its output dim: weight [out/tp, in] (partition_dim 0)."""

    def __init__(self, input_size: int, output_size: int, bias: bool = True, gather_output: bool = True,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None, stride: int = 1,
                 init_method: Optional[Callable[..., Any]] = None, sequence_parallel_enabled: bool = False,
                 keep_master_weight: bool = False, skip_bias_add: bool = False, pad: bool = False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.add_bias = bias
        self.gather_output = gather_output
        self.arg_init_method = init_method
        ws = get_tensor_model_parallel_size()
        self.pad = pad
        self.pad_size = 0
        if pad:
            self.pad_size = get_padding_length(output_size, ws)
            self.output_size = output_size + self.pad_size
        self.output_size_per_partition = divide(self.output_size, ws)
        self.dtype = dtype
        self.device = _device_of(device)
        self.stride = stride
        self.keep_master_weight = keep_master_weight
        self.skip_bias_add = skip_bias_add
        self.async_tensor_model_parallel_allreduce = not sequence_parallel_enabled and ws > 1
        if sequence_parallel_enabled and ws <= 1:
            warnings.warn(f"`sequence_parallel_enabled` is set to `True`, but got world_size of {ws}")
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.initialize_weight_and_bias()
        self._forward_impl = linear_with_async_allreduce

    def set_weight_and_bias_config(self) -> None:
        self.weight_shape = (self.output_size_per_partition, self.input_size)
        self.weight_partition_dim = 0
        if self.add_bias:
            self.bias_shape = (self.output_size if self.gather_output else self.output_size_per_partition,)
        else:
            self.bias_shape = None

    def initialize_weight_and_bias(self) -> None:
        self.set_weight_and_bias_config()
        self.weight = Parameter(torch.empty(*self.weight_shape, device=self.device, dtype=self.dtype))
        with get_rng_tracker().fork():
            self.master_weight = _initialize_parameter(self.weight, self.weight_partition_dim, self._init_weight,
                                                       self.stride, self.keep_master_weight)
        if self.add_bias:
            self.bias = Parameter(torch.empty(*self.bias_shape, device=self.device, dtype=self.dtype))
            if self.device.type != "meta":
                self._init_bias()
            if not self.gather_output:
                set_tensor_model_parallel_attributes(self.bias, True, 0, stride=self.stride)
        else:
            self.register_parameter("bias", None)

    def forward(self, input: torch.Tensor):
        if self.pad and self.training:
            raise RuntimeError("`pad=True` is only supported for inference. Set model.eval()")
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled:
            input_parallel = input
        else:
            input_parallel = copy_to_tensor_model_parallel_region(input)
        output_parallel = self._forward_impl(input_parallel, self.weight, None, self.async_tensor_model_parallel_allreduce,
                                             self.sequence_parallel_enabled, self.autograd_func_class)
        if self.gather_output:
            assert not self.sequence_parallel_enabled
            output = gather_from_tensor_model_parallel_region(output_parallel)
            if self.pad and self.pad_size > 0:
                output = torch.narrow(output, -1, 0, self.output_size - self.pad_size)
        else:
            output = output_parallel
        if self.skip_bias_add:
            return output, self.bias
        return output + self.bias if self.bias is not None else output

    def preshard_hook(self, model_state_dict: Dict[str, Any], prefix: str) -> None:
        if not self.pad or self.pad_size == 0:
            return
        size = model_state_dict[prefix].shape[0]
        if self.output_size != size + self.pad_size:
            raise RuntimeError(f"State dict {prefix} is of an unexpected size {size} expected {size - self.pad_size}")
        model_state_dict[prefix] = F.pad(model_state_dict[prefix], (0, 0, 0, self.pad_size))


class RowParallelLinear(BaseParallelLinear):
    """Y = X A + b with A split along its input dim: weight [out, in/tp] (partition_dim 1); output is
    all-reduced over TP, or reduce-scattered along the sequence with sequence parallelism."""

    def __init__(self, input_size: int, output_size: int, bias: bool = True, input_is_parallel: bool = False,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None, stride: int = 1,
                 init_method: Optional[Callable[..., Any]] = None, sequence_parallel_enabled: bool = False,
                 keep_master_weight: bool = False, skip_bias_add: bool = False, pad: bool = False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.add_bias = bias
        self.input_is_parallel = input_is_parallel
        self.pad = pad
        self.pad_size = 0
        ws = get_tensor_model_parallel_size()
        if pad:
            self.pad_size = get_padding_length(input_size, ws)
            self.input_size = input_size + self.pad_size
        self.input_size_per_partition = divide(self.input_size, ws)
        self.arg_init_method = init_method
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if sequence_parallel_enabled and not input_is_parallel:
            raise RuntimeError("To enable `sequence_parallel_enabled`, `input_is_parallel` must be `True`")
        self.dtype = dtype
        self.device = _device_of(device)
        self.stride = stride
        self.keep_master_weight = keep_master_weight
        self.skip_bias_add = skip_bias_add
        self.initialize_weight_and_bias()
        self._forward_impl = linear_with_async_allreduce

    def set_weight_and_bias_config(self) -> None:
        self.weight_shape = (self.output_size, self.input_size_per_partition)
        self.weight_partition_dim = 1
        self.bias_shape = (self.output_size,) if self.add_bias else None

    def initialize_weight_and_bias(self) -> None:
        self.set_weight_and_bias_config()
        self.weight = Parameter(torch.empty(*self.weight_shape, device=self.device, dtype=self.dtype))
        with get_rng_tracker().fork():
            self.master_weight = _initialize_parameter(self.weight, self.weight_partition_dim, self._init_weight,
                                                       self.stride, self.keep_master_weight)
        if self.add_bias:
            self.bias = Parameter(torch.empty(*self.bias_shape, device=self.device, dtype=self.dtype))
            if self.device.type != "meta":
                bound = 1 / math.sqrt(self.input_size_per_partition) if self.input_size_per_partition > 0 else 0
                with torch.no_grad():
                    nn.init.uniform_(self.bias, -bound, bound)
            setattr(self.bias, "sequence_parallel_enabled", self.sequence_parallel_enabled)
        else:
            self.register_parameter("bias", None)

    def forward(self, input_: torch.Tensor):
        if self.pad and self.training:
            raise RuntimeError("`pad=True` is only supported for inference. Set model.eval()")
        if self.input_is_parallel:
            input_parallel = input_
        else:
            if self.pad and self.pad_size > 0:
                input_ = F.pad(input_, (0, self.pad_size))
            assert not self.sequence_parallel_enabled
            input_parallel = scatter_to_tensor_model_parallel_region(input_)
        if self.sequence_parallel_enabled and get_tensor_model_parallel_size() > 1 and \
                self.autograd_func_class is LinearWithAsyncCommunication:
            output_ = RowParallelSPLinear.apply(input_parallel, self.weight, None)
        else:
            output_parallel = self._forward_impl(input_parallel, self.weight, None, False, False,
                                                 self.autograd_func_class)
            if self.sequence_parallel_enabled:
                output_ = reduce_scatter_to_sequence_parallel_region(output_parallel)
            else:
                output_ = reduce_from_tensor_model_parallel_region(output_parallel)
        if self.skip_bias_add:
            return output_, self.bias
        return output_ + self.bias if self.bias is not None else output_

    def preshard_hook(self, model_state_dict: Dict[str, Any], prefix: str) -> None:
        if not self.pad or self.pad_size == 0:
            return
        size = model_state_dict[prefix].shape[1]
        if self.input_size != size + self.pad_size:
            raise RuntimeError(f"State dict {prefix} is of an unexpected size {size} expected {size - self.pad_size}")
        model_state_dict[prefix] = F.pad(model_state_dict[prefix], (0, self.pad_size))


class ParallelEmbedding(nn.Module):
    """Embedding sharded along the vocabulary (default) or the embedding dim.

    Vocab sharding uses the fused masked-gather kernel and a TP all-reduce of the output; with
    `sequence_parallel_enabled` and [S, B] ids the all-reduce becomes a reduce-scatter along the
    sequence (one collective instead of all-reduce + split)."""

    def __init__(self, num_embeddings: int, embedding_dim: int, padding_idx: Optional[int] = None,
                 max_norm: Optional[float] = None, norm_type: float = 2.0, scale_grad_by_freq: bool = False,
                 sparse: bool = False, init_method: Callable[..., torch.Tensor] = nn.init.normal_,
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.float32,
                 shard_across_embedding: bool = False, pad: bool = False, sequence_parallel_enabled: bool = False):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.max_norm = max_norm
        self.norm_type = norm_type
        self.scale_grad_by_freq = scale_grad_by_freq
        self.sparse = sparse
        self.tensor_model_parallel_size = get_tensor_model_parallel_size()
        self.shard_across_embedding = shard_across_embedding
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.stride = 1
        self.pad = pad
        self.pad_size = 0
        ws, rank = self.tensor_model_parallel_size, get_tensor_model_parallel_rank()
        if shard_across_embedding:
            self.num_embeddings_per_partition = num_embeddings
            if pad:
                self.pad_size = get_padding_length(embedding_dim, ws)
                self.embedding_dim = embedding_dim + self.pad_size
            self.embedding_dim_per_partition = divide(self.embedding_dim, ws)
            self.padding_idx = padding_idx
            self.weight_partition_dim = 1
            self.start_index, self.end_index = 0, num_embeddings
        else:
            if pad:
                self.pad_size = get_padding_length(num_embeddings, ws)
                self.num_embeddings = num_embeddings + self.pad_size
            self.start_index, self.end_index = EmbeddingUtility.range_from_global_vocab_size(self.num_embeddings, rank, ws)
            self.num_embeddings_per_partition = self.end_index - self.start_index
            self.embedding_dim_per_partition = embedding_dim
            if padding_idx is not None and self.start_index <= padding_idx < self.end_index:
                self.padding_idx = padding_idx - self.start_index
            else:
                self.padding_idx = None
            self.weight_partition_dim = 0
        self.init_method = init_method
        self.dtype = dtype
        self.device = _device_of(device)
        self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, self.embedding_dim_per_partition,
                                            device=self.device, dtype=dtype))
        with get_rng_tracker().fork():
            _initialize_parameter(self.weight, self.weight_partition_dim, self.init_method, 1)

    def init_weight_cpu(self) -> None:
        _initialize_parameter(self.weight, self.weight_partition_dim, self.init_method, 1)

    def _forward_shard_across_vocab(self, input_: torch.Tensor) -> torch.Tensor:
        if self.max_norm is None and not self.scale_grad_by_freq and self.padding_idx is None:
            out = ops.vocab_parallel_embedding(input_, self.weight, self.start_index)
        else:
            local = input_ - self.start_index
            mask = (local >= 0) & (local < self.num_embeddings_per_partition)
            out = F.embedding(local.clamp(0, self.num_embeddings_per_partition - 1), self.weight, self.padding_idx,
                              self.max_norm, self.norm_type, self.scale_grad_by_freq, self.sparse)
            out = out * mask.unsqueeze(-1).to(out.dtype)
        if self.sequence_parallel_enabled:
            return reduce_scatter_to_sequence_parallel_region(out)
        return reduce_from_tensor_model_parallel_region(out)

    def _forward_shard_across_embed(self, input_: torch.Tensor) -> torch.Tensor:
        out = F.embedding(input_.long(), self.weight, self.padding_idx, self.max_norm, self.norm_type,
                          self.scale_grad_by_freq, self.sparse)
        return gather_from_tensor_model_parallel_region(out)

    def forward(self, input_: torch.Tensor) -> torch.Tensor:
        if self.pad and self.training:
            raise RuntimeError("`pad=True` is only supported for inference. Set model.eval()")
        if self.shard_across_embedding:
            out = self._forward_shard_across_embed(input_)
            if self.pad and self.pad_size > 0:
                out = torch.narrow(out, -1, 0, self.embedding_dim - self.pad_size)
            return out
        return self._forward_shard_across_vocab(input_)

    def preshard_hook(self, model_state_dict: Dict[str, Any], prefix: str) -> None:
        if not self.pad or self.pad_size == 0:
            return
        dim = self.weight_partition_dim
        size = model_state_dict[prefix].shape[dim]
        if self.shard_across_embedding:
            if self.embedding_dim != size + self.pad_size:
                raise RuntimeError(f"State dict {prefix} is of an unexpected shape {size}")
            model_state_dict[prefix] = F.pad(model_state_dict[prefix], (0, self.pad_size))
        else:
            if self.num_embeddings != size + self.pad_size:
                raise RuntimeError(f"State dict {prefix} is of an unexpected shape {size}")
            model_state_dict[prefix] = F.pad(model_state_dict[prefix], (0, 0, 0, self.pad_size))


# ------------------------------------------------------------------------------------------------
# channel-parallel convolutions (reference layers.py:813-1235)
# ------------------------------------------------------------------------------------------------


class _ConvTPBase(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias, padding_mode,
                 partition_dim, dtype, device, init_method, keep_master_weight):
        super().__init__()
        if groups != 1:
            raise NotImplementedError("grouped channel-parallel convolutions are not supported")
        self.in_channels, self.out_channels = in_channels, out_channels
        ks = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.kernel_size = ks
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.padding_mode = padding_mode
        ws = get_tensor_model_parallel_size()
        self.partition_dim = partition_dim
        shape = [out_channels, in_channels] + list(ks)
        shape[partition_dim] = divide(shape[partition_dim], ws)
        self.dtype, self.device = dtype, _device_of(device)
        self.weight = Parameter(torch.empty(shape, dtype=dtype, device=self.device))
        self.arg_init_method = init_method

        def _init(w):
            if init_method is None:
                nn.init.kaiming_uniform_(w, a=math.sqrt(5))
            else:
                init_method(w)

        with get_rng_tracker().fork():
            self.master_weight = _initialize_parameter(self.weight, partition_dim, _init, 1, keep_master_weight)
        self.use_bias = bias

    def _conv(self, x, weight, bias):
        return F.conv2d(x, weight, bias, self.stride, self.padding, self.dilation, 1)


class OutputChannelParallelConv2d(_ConvTPBase):
    """Conv2d with out-channels split over TP (column-style); optional gather of the output channels."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 padding_mode="zeros", gather_output=True, dtype=torch.float32, device=None, init_method=None,
                 keep_master_weight=False):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias, padding_mode, 0,
                         dtype, device, init_method, keep_master_weight)
        self.gather_output = gather_output
        if bias:
            self.bias = Parameter(torch.zeros(self.weight.shape[0], dtype=dtype, device=self.device))
            set_tensor_model_parallel_attributes(self.bias, True, 0, 1)
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        x = copy_to_tensor_model_parallel_region(x)
        out = self._conv(x, self.weight, self.bias)
        if self.gather_output:
            from .mappings import gather_from_tensor_model_parallel_region_with_dim

            out = gather_from_tensor_model_parallel_region_with_dim(out, 1)
        return out


class InputChannelParallelConv2d(_ConvTPBase):
    """Conv2d with in-channels split over TP (row-style); partial outputs all-reduced."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 padding_mode="zeros", input_is_parallel=False, dtype=torch.float32, device=None, init_method=None,
                 keep_master_weight=False):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias, padding_mode, 1,
                         dtype, device, init_method, keep_master_weight)
        self.input_is_parallel = input_is_parallel
        if bias:
            self.bias = Parameter(torch.zeros(out_channels, dtype=dtype, device=self.device))
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_input_channels_to_tensor_model_parallel_region(x)
        out = reduce_from_tensor_model_parallel_region(self._conv(x, self.weight, None))
        if self.bias is not None:
            out = out + self.bias.view(1, -1, 1, 1)
        return out
