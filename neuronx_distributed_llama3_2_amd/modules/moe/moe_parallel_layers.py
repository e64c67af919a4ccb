"""Expert-fused tensor-parallel linears with 3-D weights, and the router linear
(reference: src/neuronx_distributed/modules/moe/moe_parallel_layers.py:13-394).

Weights are [E_local, in, out_local] (E_local = num_experts / EP; the out dim is TP-sharded for the
column layer, the in dim for the row layer) and tagged `expert_model_parallel` so the optimizer,
grad-norm and checkpoint code treat them as EP-sharded.  The expert GEMMs are batched
(one strided-batched hipBLASLt call over all local experts: torch.bmm / baddbmm).
"""

from __future__ import annotations

import math
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist
from torch import nn
from torch.nn.parameter import Parameter

from ...parallel_layers import parallel_state as ps
from ...parallel_layers.mappings import copy_to_tensor_model_parallel_region
from ...parallel_layers.random import get_rng_tracker
from ...parallel_layers.utils import divide, set_tensor_model_parallel_attributes


def _mark_ep(p: torch.Tensor) -> None:
    setattr(p, "expert_model_parallel", True)


class ExpertFusedLinearWithAsyncCommunication(torch.autograd.Function):
    """out[e] = in[e] @ W[e] for every local expert (in: [E, ..., H], W: [E, H, I])."""

    @staticmethod
    def forward(ctx, input, weight, bias, async_grad_allreduce, sequence_parallel_enabled, save_for_backward=True):
        if bias is not None:
            raise NotImplementedError("Bias is not currently supported for MoE")
        if sequence_parallel_enabled:
            raise NotImplementedError("exit sequence parallelism before the expert-fused linears")
        if input.shape[0] != weight.shape[0] and input.shape[0] > 1:
            raise RuntimeError(f"input/weight expert count mismatch: {tuple(input.shape)} vs {tuple(weight.shape)}")
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.compute_weight_gradient = weight.requires_grad
        ctx.save_for_backward(input, weight)
        E = weight.shape[0]
        x = input.expand((E,) + tuple(input.shape[1:])) if input.shape[0] == 1 and E > 1 else input
        ctx.in_shape = input.shape
        x3 = x.reshape(E, -1, x.shape[-1])
        out = torch.bmm(x3, weight)
        return out.view(tuple(x.shape[:-1]) + (weight.shape[-1],))

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        E = weight.shape[0]
        g3 = grad_output.reshape(E, -1, grad_output.shape[-1])
        grad_in = torch.bmm(g3, weight.transpose(1, 2)).view(tuple(grad_output.shape[:-1]) + (weight.shape[1],))
        if ctx.in_shape[0] == 1 and E > 1:
            grad_in = grad_in.sum(0, keepdim=True)
        handle = None
        if ctx.async_grad_allreduce and ps.get_tensor_model_parallel_size() > 1:
            grad_in = grad_in.contiguous()
            handle = dist.all_reduce(grad_in, group=ps.get_tensor_model_parallel_group(), async_op=True)
        grad_w = None
        if ctx.compute_weight_gradient:
            x = input.expand((E,) + tuple(input.shape[1:])) if input.shape[0] == 1 and E > 1 else input
            x3 = x.reshape(E, -1, x.shape[-1])
            grad_w = torch.bmm(x3.transpose(1, 2), g3)
            mg = getattr(weight, "main_grad", None)
            if mg is not None:
                mg.add_(grad_w.float())
                cb = getattr(weight, "_nxd_grad_ready", None)
                if cb is not None:
                    cb(weight)
                grad_w = None
        if handle is not None:
            handle.wait()
        return grad_in, grad_w, None, None, None, None


class _ExpertFusedBase(nn.Module):
    def _create(self, num_experts, in_size, out_size, partition_dim, stride, init_method, dtype, device, tp_dim_full):
        ep = ps.get_expert_model_parallel_size() if ps.model_parallel_is_initialized() else 1
        self.num_experts = num_experts
        self._n_local_experts = divide(num_experts, ep)
        ep_rank = ps.get_expert_model_parallel_rank() if ep > 1 else 0
        tp = ps.get_tensor_model_parallel_size()
        tp_rank = ps.get_tensor_model_parallel_rank()
        shape = [self._n_local_experts, in_size, out_size]
        shape[partition_dim] = divide(shape[partition_dim], tp)
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.weight = Parameter(torch.empty(*shape, dtype=dtype, device=device))
        set_tensor_model_parallel_attributes(self.weight, True, partition_dim, stride)
        _mark_ep(self.weight)
        if device.type == "meta":
            return
        # initialise every expert's FULL weight in fp32 (independent of TP/EP degree), keep ours
        with get_rng_tracker().fork():
            full_shape = [num_experts, in_size, out_size]
            full = torch.empty(full_shape, dtype=torch.float32)
            for e in range(num_experts):
                if init_method is None:
                    nn.init.kaiming_uniform_(full[e], a=math.sqrt(5))
                else:
                    init_method(full[e])
        full = full[ep_rank * self._n_local_experts:(ep_rank + 1) * self._n_local_experts]
        per = shape[partition_dim] // stride
        chunks = torch.split(full, per, dim=partition_dim)
        local = torch.cat(chunks[tp_rank::tp], dim=partition_dim)
        with torch.no_grad():
            self.weight.copy_(local.to(dtype))


class ExpertFusedColumnParallelLinear(_ExpertFusedBase):
    """[E, ..., H] -> [E, ..., I/tp] (weights [E_local, H, I/tp])."""

    autograd_func_class = ExpertFusedLinearWithAsyncCommunication

    def __init__(self, num_experts: int, input_size: int, output_size: int, dtype: torch.dtype = torch.float32,
                 device: Optional[torch.device] = None, stride: int = 1,
                 init_method: Optional[Callable[..., Any]] = None, keep_master_weight: bool = False):
        super().__init__()
        self.input_size, self.output_size, self.stride = input_size, output_size, stride
        self._create(num_experts, input_size, output_size, 2, stride, init_method, dtype, device, output_size)
        self.async_tensor_model_parallel_allreduce = ps.get_tensor_model_parallel_size() > 1
        self.skip_input_copy = False

    def forward(self, input_: torch.Tensor, expert_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = input_ if (self.async_tensor_model_parallel_allreduce or self.skip_input_copy) \
            else copy_to_tensor_model_parallel_region(input_)
        w = self.weight[expert_indices] if expert_indices is not None else self.weight
        return ExpertFusedLinearWithAsyncCommunication.apply(x, w, None, self.async_tensor_model_parallel_allreduce,
                                                             False)


class ExpertFusedRowParallelLinear(_ExpertFusedBase):
    """[E, ..., I/tp] -> [E, ..., H] partial sums (reduce over TP by the caller, or here when
    `reduce_output` is set)."""

    def __init__(self, num_experts: int, input_size: int, output_size: int, reduce_output: bool = True,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None, stride: int = 1,
                 init_method: Optional[Callable[..., Any]] = None, keep_master_weight: bool = False):
        super().__init__()
        self.input_size, self.output_size, self.stride = input_size, output_size, stride
        self.reduce_output = reduce_output
        self._create(num_experts, input_size, output_size, 1, stride, init_method, dtype, device, input_size)

    def forward(self, input_: torch.Tensor, expert_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        w = self.weight[expert_indices] if expert_indices is not None else self.weight
        out = ExpertFusedLinearWithAsyncCommunication.apply(input_, w, None, False, False)
        if self.reduce_output and ps.get_tensor_model_parallel_size() > 1:
            from ...parallel_layers.mappings import reduce_from_tensor_model_parallel_region

            out = reduce_from_tensor_model_parallel_region(out)
        return out


class LinearWithWeightGradAR(torch.autograd.Function):
    """y = x W^T whose weight gradient is all-reduced over TP (router fed by TP-sharded tokens)."""

    @staticmethod
    def forward(ctx, input, weight, reduce_weight_grad):
        ctx.save_for_backward(input, weight)
        ctx.reduce = reduce_weight_grad
        return torch.matmul(input, weight.t())

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        gi = grad_output.matmul(weight)
        gw = grad_output.reshape(-1, grad_output.shape[-1]).t().matmul(input.reshape(-1, input.shape[-1]))
        if ctx.reduce and ps.get_tensor_model_parallel_size() > 1:
            dist.all_reduce(gw, group=ps.get_tensor_model_parallel_group())
        return gi, gw, None


class LinearRouter(nn.Module):
    """Replicated router projection [E, H] (fp32 by default).  Inside a TP MoE layer the logits'
    gradients are TP-partial (each rank combines only its shard of every expert's output), so the
    weight gradient is all-reduced over TP (`reduce_weight_grad`, set by the MoE layer)."""

    def __init__(self, input_size: int, output_size: int, sequence_parallel_enabled: bool = False,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None):
        super().__init__()
        self.input_size, self.output_size = input_size, output_size
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.reduce_weight_grad = sequence_parallel_enabled
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.weight = Parameter(torch.empty(output_size, input_size, dtype=dtype, device=device))
        if device.type != "meta":
            self.init_weight_cpu()

    def init_weight_cpu(self):
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def forward(self, input_):
        x = input_.to(self.weight.dtype)
        return LinearWithWeightGradAR.apply(x, self.weight, self.reduce_weight_grad)
