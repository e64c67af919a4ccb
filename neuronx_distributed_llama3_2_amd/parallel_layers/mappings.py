"""Autograd-aware tensor-parallel / sequence-parallel / expert-parallel collectives.

Megatron "f/g" operators with the reference's names and semantics
(src/neuronx_distributed/parallel_layers/mappings.py:42-486).  Every collective is a
`torch.distributed` call on the NCCL backend, i.e. RCCL over xGMI on ROCm, issued on the current
HIP stream (RCCL orders it behind the producing kernel) — real all-gather / reduce-scatter /
all-to-all tensors, not the reference's XLA replica-group lowering.  Gathers and scatters along
a non-leading dim move that dim to the front first so the RCCL buffer is contiguous.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel import comm
from torch import Tensor

from .parallel_state import (
    get_expert_model_parallel_group,
    get_expert_model_parallel_size,
    get_tensor_model_parallel_group,
    get_tensor_model_parallel_rank,
    get_tensor_model_parallel_size,
)
from .sp import sp_gather, sp_reduce_scatter, sp_split
from .utils import split_tensor_along_dim


def _tp_group():
    return get_tensor_model_parallel_group()


def nonzero_partition_dim_swap(func):
    """Run `func` on `x` with `partition_dim` moved to dim 0 (reference mappings.py:24-39)."""

    def wrapped(x: Tensor, partition_dim: int, *args, **kwargs):
        partition_dim = partition_dim % x.dim()
        if partition_dim == 0:
            return func(x, 0, *args, **kwargs)
        xt = x.transpose(0, partition_dim).contiguous()
        out = func(xt, 0, *args, **kwargs)
        return out.transpose(0, partition_dim).contiguous()

    return wrapped


def _reduce(input_: Tensor, group=None) -> Tensor:
    group = group if group is not None else _tp_group()
    if dist.get_world_size(group=group) == 1:
        return input_
    x = input_.contiguous()
    dist.all_reduce(x, group=group)
    return x


def _split_along_dim(input_: Tensor, partition_dim: int, group=None) -> Tensor:
    group = group if group is not None else _tp_group()
    ws = dist.get_world_size(group=group)
    if ws == 1:
        return input_
    rank = dist.get_rank(group=group)
    return split_tensor_along_dim(input_, partition_dim % input_.dim(), ws)[rank].contiguous()


def _split_along_last_dim(input_: Tensor) -> Tensor:
    return _split_along_dim(input_, -1)


def _split_along_first_dim(input_: Tensor) -> Tensor:
    return _split_along_dim(input_, 0)


@nonzero_partition_dim_swap
def _gather_along_dim_0(x: Tensor, _dim: int, group=None) -> Tensor:
    ws = dist.get_world_size(group=group)
    out = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    comm.all_gather_into_tensor(out, x.contiguous(), group=group)
    return out


def _gather_along_dim(x: Tensor, partition_dim: int, group=None) -> Tensor:
    group = group if group is not None else _tp_group()
    if dist.get_world_size(group=group) == 1:
        return x
    return _gather_along_dim_0(x, partition_dim, group=group)


def _gather_along_first_dim(x: Tensor) -> Tensor:
    return _gather_along_dim(x, 0)


def _gather_along_last_dim(x: Tensor) -> Tensor:
    return _gather_along_dim(x, -1)


@nonzero_partition_dim_swap
def _reduce_scatter_dim_0(x: Tensor, _dim: int, group=None) -> Tensor:
    ws = dist.get_world_size(group=group)
    assert x.shape[0] % ws == 0, f"dim {x.shape[0]} not divisible by TP size {ws}"
    out = torch.empty((x.shape[0] // ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    comm.reduce_scatter_tensor(out, x.contiguous(), group=group)
    return out


def _reduce_scatter_along_dim(x: Tensor, partition_dim: int, group=None) -> Tensor:
    group = group if group is not None else _tp_group()
    if dist.get_world_size(group=group) == 1:
        return x
    return _reduce_scatter_dim_0(x, partition_dim, group=group)


def _reduce_scatter_along_first_dim(x: Tensor) -> Tensor:
    return _reduce_scatter_along_dim(x, 0)


def _reduce_scatter_along_last_dim(x: Tensor) -> Tensor:
    return _reduce_scatter_along_dim(x, -1)


def _all_to_all_in_expert_parallel_region(x: Tensor, split_dim: int, concat_dim: int) -> Tensor:
    """Split `x` along split_dim into EP chunks, exchange, concatenate received chunks on concat_dim."""
    group = get_expert_model_parallel_group()
    ws = get_expert_model_parallel_size()
    if ws == 1:
        return x
    split_dim %= x.dim()
    concat_dim %= x.dim()
    xs = x.movedim(split_dim, 0).contiguous()
    out = torch.empty_like(xs)
    comm.all_to_all_single(out, xs, group=group)
    chunks = out.chunk(ws, dim=0)
    chunks = [c.movedim(0, split_dim) for c in chunks]
    return torch.cat(chunks, dim=concat_dim).contiguous()


# ---------------------------------------------------------------------------------------------


class _CopyToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return input_

    @staticmethod
    def backward(ctx, grad_output):
        return _reduce(grad_output)


class _ReduceFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _reduce(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class _ScatterToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _split_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_last_dim(grad_output)


class _GatherFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _gather_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _split_along_last_dim(grad_output)


class _ScatterToSequenceParallelRegion(torch.autograd.Function):
    """Split along the sequence into this rank's (chunk-interleaved, see sp.py) SP shard."""

    @staticmethod
    def forward(ctx, input_):
        return sp_split(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return sp_gather(grad_output)


class _GatherFromSequenceParallelRegion(torch.autograd.Function):
    """All-gather along seq; backward reduce-scatters (to_model_parallel=True: the consumer is a TP
    region whose grads are partial sums) or just splits (to_model_parallel=False)."""

    @staticmethod
    def forward(ctx, input_, to_model_parallel=True):
        ctx.to_model_parallel = to_model_parallel
        return sp_gather(input_)

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.to_model_parallel:
            return sp_reduce_scatter(grad_output), None
        return sp_split(grad_output), None


class _ReduceScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return sp_reduce_scatter(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return sp_gather(grad_output)


class _ReduceScatterToTensorParallelRegionWithDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, partition_dim):
        ctx.partition_dim = partition_dim
        return _reduce_scatter_along_dim(input_, partition_dim)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_dim(grad_output, ctx.partition_dim), None


class _GatherFromTensorParallelRegionWithDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, partition_dim):
        ctx.partition_dim = partition_dim
        return _gather_along_dim(input_, partition_dim)

    @staticmethod
    def backward(ctx, grad_output):
        return _split_along_dim(grad_output, ctx.partition_dim), None


class _AllToAllInExpertParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, split_dim, concat_dim):
        ctx.split_dim, ctx.concat_dim = split_dim, concat_dim
        return _all_to_all_in_expert_parallel_region(input_, split_dim, concat_dim)

    @staticmethod
    def backward(ctx, grad_output):
        return _all_to_all_in_expert_parallel_region(grad_output, ctx.concat_dim, ctx.split_dim), None, None


class _ScatterInputChannelsToModelParallelRegion(torch.autograd.Function):
    """Split the channel dim (1) of an NCHW activation over TP; backward all-gathers."""

    @staticmethod
    def forward(ctx, input_):
        return _split_along_dim(input_, 1)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_dim(grad_output, 1)


def copy_to_tensor_model_parallel_region(input_: Tensor) -> Tensor:
    return _CopyToModelParallelRegion.apply(input_)


def reduce_from_tensor_model_parallel_region(input_: Tensor) -> Tensor:
    return _ReduceFromModelParallelRegion.apply(input_)


def scatter_input_channels_to_tensor_model_parallel_region(input_: Tensor) -> Tensor:
    return _ScatterInputChannelsToModelParallelRegion.apply(input_)


def scatter_to_tensor_model_parallel_region(input_: Tensor) -> Tensor:
    return _ScatterToModelParallelRegion.apply(input_)


def gather_from_tensor_model_parallel_region(input_: Tensor) -> Tensor:
    return _GatherFromModelParallelRegion.apply(input_)


def scatter_to_sequence_parallel_region(input_: Tensor) -> Tensor:
    return _ScatterToSequenceParallelRegion.apply(input_)


def gather_from_sequence_parallel_region(input_: Tensor, to_model_parallel: bool = True) -> Tensor:
    return _GatherFromSequenceParallelRegion.apply(input_, to_model_parallel)


def reduce_scatter_to_sequence_parallel_region(input_: Tensor) -> Tensor:
    return _ReduceScatterToSequenceParallelRegion.apply(input_)


def reduce_scatter_to_tensor_model_parallel_region_with_dim(input_: Tensor, partition_dim: int) -> Tensor:
    return _ReduceScatterToTensorParallelRegionWithDim.apply(input_, partition_dim)


def gather_from_tensor_model_parallel_region_with_dim(input_: Tensor, partition_dim: int) -> Tensor:
    return _GatherFromTensorParallelRegionWithDim.apply(input_, partition_dim)


def enter_expert_parallel_region(x: Tensor, scatter_gather: bool = False) -> Tensor:
    """[E, C, H] tokens grouped by expert -> [E/ep, ep*C, H] this rank's experts' tokens
    (reference mappings.py:412-449).  With `scatter_gather` the token dim is additionally
    gathered over TP first (SP inputs)."""
    if scatter_gather and get_tensor_model_parallel_size() > 1:
        x = gather_from_tensor_model_parallel_region_with_dim(x, 1)
    if get_expert_model_parallel_size() == 1:
        return x
    return _AllToAllInExpertParallelRegion.apply(x, 0, 1)


def exit_expert_parallel_region(x: Tensor, scatter_gather: bool = False) -> Tensor:
    """Inverse of `enter_expert_parallel_region` (reference mappings.py:452-486)."""
    if get_expert_model_parallel_size() > 1:
        x = _AllToAllInExpertParallelRegion.apply(x, 1, 0)
    if scatter_gather and get_tensor_model_parallel_size() > 1:
        x = reduce_scatter_to_tensor_model_parallel_region_with_dim(x, 1)
    return x


__all__ = [
    "copy_to_tensor_model_parallel_region",
    "reduce_from_tensor_model_parallel_region",
    "scatter_to_tensor_model_parallel_region",
    "gather_from_tensor_model_parallel_region",
    "scatter_to_sequence_parallel_region",
    "gather_from_sequence_parallel_region",
    "reduce_scatter_to_sequence_parallel_region",
    "reduce_scatter_to_tensor_model_parallel_region_with_dim",
    "gather_from_tensor_model_parallel_region_with_dim",
    "enter_expert_parallel_region",
    "exit_expert_parallel_region",
    "get_tensor_model_parallel_rank",
]
