"""GQA QKV column-parallel projection with KV-head replication
(reference: src/neuronx_distributed/modules/qkv_linear.py:34-772).

* `kv_size_multiplier` replicates the K/V heads so that (num_kv_heads * multiplier) is divisible by
  the TP degree (TP > #kv heads).  Ranks holding the same KV head form a "kv-shared group"; the
  K/V *output* gradients are summed over it before the K/V weight-gradient GEMM so replicas stay
  identical (the local, un-reduced gradients feed dX, which is exact).
* `fuse_qkv=True` keeps one [q_r | k_r | v_r] weight per rank and runs ONE GEMM whose output is the
  fused [S, B, (nq + 2 nkv) * D] buffer the flash-attention core reads in place
  (ops.rope_attention) — `forward_fused`.  `forward` returns (q, k, v) views for API parity.
* Sequence parallelism: the input is all-gathered once along the sequence and kept for dW;
  the dX reduce-scatter overlaps the weight-gradient GEMMs (same scheme as ColumnParallelLinear).
"""

from __future__ import annotations

import math
import warnings
from typing import Any, Callable, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel import comm
from ..ops import gemm as _gemm
from torch import nn
from torch.nn.parameter import Parameter

from ..parallel_layers.layers import (
    _SAVE_GATHERED_INPUT,
    BaseParallelLinear,
    _accumulate_wgrad,
    _bias_grad,
    _initialize_parameter,
    _device_of,
)
from ..parallel_layers import sp
from ..parallel_layers.mappings import copy_to_tensor_model_parallel_region, gather_from_tensor_model_parallel_region
from ..parallel_layers.parallel_state import (
    get_tensor_model_parallel_group,
    get_tensor_model_parallel_rank,
    get_tensor_model_parallel_size,
    model_parallel_is_initialized,
)
from ..parallel_layers.random import get_rng_tracker
from ..parallel_layers.utils import divide, set_tensor_model_parallel_attributes

_KV_SHARED_GROUP = None
_KV_SHARED_GROUP_MESH: Optional[List[List[int]]] = None
_KV_GROUP_SIZE: Optional[int] = None


def _initialize_kv_group(kv_shared_group_size: int = 1) -> None:
    """Ranks i, i + tp/m, i + 2 tp/m, ... of every TP group share a KV head (reference :34-72)."""
    global _KV_SHARED_GROUP, _KV_SHARED_GROUP_MESH, _KV_GROUP_SIZE
    if _KV_GROUP_SIZE is not None:
        assert kv_shared_group_size == _KV_GROUP_SIZE, "only one KV replication factor per process is supported"
        return
    _KV_GROUP_SIZE = kv_shared_group_size
    if kv_shared_group_size == 1 or not (dist.is_initialized() and model_parallel_is_initialized()):
        return
    tp = get_tensor_model_parallel_size()
    assert tp % kv_shared_group_size == 0
    world = dist.get_world_size()
    rank = dist.get_rank()
    mesh = []
    for i in range(world // tp):
        for j in range(tp // kv_shared_group_size):
            mesh.append(list(range(i * tp + j, (i + 1) * tp, tp // kv_shared_group_size)))
    _KV_SHARED_GROUP_MESH = mesh
    for ranks in mesh:
        g = dist.new_group(ranks)
        if rank in ranks:
            _KV_SHARED_GROUP = g


def get_kv_shared_group(as_list: bool = False):
    return _KV_SHARED_GROUP_MESH if as_list else _KV_SHARED_GROUP


def destroy_kv_group() -> None:
    global _KV_SHARED_GROUP, _KV_SHARED_GROUP_MESH, _KV_GROUP_SIZE
    _KV_SHARED_GROUP = _KV_SHARED_GROUP_MESH = _KV_GROUP_SIZE = None


class GQAQKVLinearWithAsyncCommunication(torch.autograd.Function):
    """Fused QKV GEMM; output [..., q_local + 2 kv_local]."""

    @staticmethod
    def forward(ctx, input, weight, bias, q_local, kv_local, async_grad_allreduce, sequence_parallel_enabled,
                kv_mult):
        ctx.use_bias = bias is not None
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sp = sequence_parallel_enabled
        ctx.q_local, ctx.kv_local, ctx.kv_mult = q_local, kv_local, kv_mult
        if sequence_parallel_enabled:
            out, total_input = sp.gather_linear(input, weight)   # chunk-pipelined all-gather + GEMM
        else:
            total_input = input
            out = _gemm.linear(total_input, weight)
        ctx.saved_gathered = (not sequence_parallel_enabled) or _SAVE_GATHERED_INPUT
        ctx.save_for_backward(total_input if ctx.saved_gathered else input, weight, bias)
        if bias is not None:
            out = out + bias
        return out

    @staticmethod
    def backward(ctx, grad_output):
        inp, weight, bias = ctx.saved_tensors
        total_input = inp if ctx.saved_gathered else sp.sp_gather(inp)
        grad_output = grad_output.contiguous()
        group = get_tensor_model_parallel_group() if model_parallel_is_initialized() else None
        ws = dist.get_world_size(group=group) if group is not None else 1
        handles = []
        if ctx.sp and ws > 1:
            # dgrad GEMM chunks with their reduce-scatters in flight behind them
            grad_input, handles = sp.matmul_reduce_scatter_start(grad_output, weight, group)
        else:
            grad_input = _gemm.dgrad(grad_output, weight)
            if ctx.async_grad_allreduce and ws > 1:
                handles = [dist.all_reduce(grad_input, group=group, async_op=True)]
        go2 = grad_output.reshape(-1, grad_output.shape[-1])
        if ctx.kv_mult > 1 and _KV_SHARED_GROUP is not None:
            # sum the K/V output grads over the replicas before the weight-gradient GEMM
            kv = go2[:, ctx.q_local:].contiguous()
            dist.all_reduce(kv, group=_KV_SHARED_GROUP)
            go2 = torch.cat([go2[:, :ctx.q_local], kv], dim=1)
        x2 = total_input.reshape(-1, total_input.shape[-1])
        grad_weight = _accumulate_wgrad(weight, go2, x2) if ctx.needs_input_grad[1] else None
        grad_bias = _bias_grad(bias, go2) if ctx.use_bias else None
        for h in handles:
            h.wait()
        return grad_input, grad_weight, grad_bias, None, None, None, None, None


def gqa_qkv_linear_with_async_allreduce(input, weight, bias, q_local, kv_local, async_grad_allreduce,
                                        sequence_parallel_enabled, kv_mult=1):
    return GQAQKVLinearWithAsyncCommunication.apply(input, weight, bias, q_local, kv_local, async_grad_allreduce,
                                                    sequence_parallel_enabled, kv_mult)


class GQAQKVColumnParallelLinear(BaseParallelLinear):
    def __init__(self, input_size: int, output_sizes: List[int], bias: bool = True, gather_output: bool = True,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None,
                 init_method: Optional[Callable[..., Any]] = None, sequence_parallel_enabled: bool = False,
                 keep_master_weight: bool = False, kv_size_multiplier: int = 1, fuse_qkv: bool = True):
        super().__init__()
        self.input_size = input_size
        self.output_sizes = list(output_sizes)
        self.gather_output = gather_output
        self.arg_init_method = init_method
        ws = get_tensor_model_parallel_size()
        self.kv_size_multiplier = kv_size_multiplier
        assert ws % kv_size_multiplier == 0, "tp_world_size should be divisible by kv_size_multiplier"
        assert (output_sizes[1] * kv_size_multiplier) % ws == 0, \
            "kv_output_dim*kv_size_multiplier should be divisible by tp_world_size"
        _initialize_kv_group(kv_size_multiplier)
        self.q_output_size_per_partition = divide(output_sizes[0], ws)
        self.kv_output_size_per_partition = divide(output_sizes[1] * kv_size_multiplier, ws)
        self.dtype = dtype
        self.device = _device_of(device)
        self.keep_master_weight = keep_master_weight
        self.use_bias = bias
        self.fuse_qkv = fuse_qkv
        self.async_tensor_model_parallel_allreduce = not sequence_parallel_enabled and ws > 1
        if sequence_parallel_enabled and ws <= 1:
            warnings.warn(f"`sequence_parallel_enabled` is set to `True`, but got world_size of {ws}")
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self._create_weights_biases()

    # full weights are generated deterministically (same on every rank) then sharded
    def _shard_full(self, full: torch.Tensor, is_kv: bool) -> torch.Tensor:
        """Same layout as parallel_layers.sharding.shard_tensor: replicated K/V, and with
        replication each rank's Q head group is the one that attends to its kv head."""
        from ..parallel_layers.sharding import q_group_order

        ws, rank = get_tensor_model_parallel_size(), get_tensor_model_parallel_rank()
        if is_kv and self.kv_size_multiplier > 1:
            full = torch.cat([full] * self.kv_size_multiplier, dim=0)
        per = full.shape[0] // ws
        g = q_group_order(ws, self.kv_size_multiplier)[rank] if not is_kv else rank
        return full[g * per:(g + 1) * per]

    def _init_full(self, rows: int) -> torch.Tensor:
        w = torch.empty(rows, self.input_size, dtype=torch.float32, device=self.device if self.device.type != "meta" else "cpu")
        if self.arg_init_method is None:
            nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        else:
            self.arg_init_method(w)
        return w

    def _create_weights_biases(self):
        q_l, kv_l = self.q_output_size_per_partition, self.kv_output_size_per_partition
        meta = self.device.type == "meta"
        with get_rng_tracker().fork():
            if meta:
                shards = [torch.empty(q_l, self.input_size, device="meta", dtype=self.dtype),
                          torch.empty(kv_l, self.input_size, device="meta", dtype=self.dtype),
                          torch.empty(kv_l, self.input_size, device="meta", dtype=self.dtype)]
            else:
                fq = self._init_full(self.output_sizes[0])
                fk = self._init_full(self.output_sizes[1])
                fv = self._init_full(self.output_sizes[1])
                shards = [self._shard_full(fq, False), self._shard_full(fk, True), self._shard_full(fv, True)]
                shards = [s.to(device=self.device, dtype=self.dtype) for s in shards]
        if self.fuse_qkv:
            self.weight_qkv = Parameter(torch.cat(shards, dim=0))
            set_tensor_model_parallel_attributes(self.weight_qkv, True, 0, 1)
            setattr(self.weight_qkv, "fused_qkv", True)
            setattr(self.weight_qkv, "num_partitions", get_tensor_model_parallel_size())
            # full-row layout needed to (un)shard checkpoints: (q rows, kv rows, kv replication)
            setattr(self.weight_qkv, "qkv_split", (self.output_sizes[0], self.output_sizes[1], self.kv_size_multiplier))
        else:
            self.weight_q = Parameter(shards[0])
            self.weight_k = Parameter(shards[1])
            self.weight_v = Parameter(shards[2])
            for w in (self.weight_q, self.weight_k, self.weight_v):
                set_tensor_model_parallel_attributes(w, True, 0, 1)
        if self.use_bias:
            if self.fuse_qkv:
                self.bias_qkv = Parameter(torch.zeros(q_l + 2 * kv_l, dtype=self.dtype, device=self.device))
                set_tensor_model_parallel_attributes(self.bias_qkv, True, 0, 1)
                setattr(self.bias_qkv, "qkv_split", (self.output_sizes[0], self.output_sizes[1], self.kv_size_multiplier))
            else:
                self.bias_q = Parameter(torch.zeros(q_l, dtype=self.dtype, device=self.device))
                self.bias_k = Parameter(torch.zeros(kv_l, dtype=self.dtype, device=self.device))
                self.bias_v = Parameter(torch.zeros(kv_l, dtype=self.dtype, device=self.device))
                for b in (self.bias_q, self.bias_k, self.bias_v):
                    set_tensor_model_parallel_attributes(b, True, 0, 1)
        else:
            self.bias_qkv = self.bias_q = self.bias_k = self.bias_v = None

    def _fused_weight_bias(self):
        if self.fuse_qkv:
            return self.weight_qkv, self.bias_qkv
        w = torch.cat([self.weight_q, self.weight_k, self.weight_v], dim=0)
        b = torch.cat([self.bias_q, self.bias_k, self.bias_v]) if self.use_bias else None
        return w, b

    def forward_fused(self, input: torch.Tensor) -> torch.Tensor:
        """[.., H] -> [.., q_local + 2 * kv_local] (one GEMM)."""
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled:
            x = input
        else:
            x = copy_to_tensor_model_parallel_region(input)
        w, b = self._fused_weight_bias()
        return gqa_qkv_linear_with_async_allreduce(x, w, b, self.q_output_size_per_partition,
                                                   self.kv_output_size_per_partition,
                                                   self.async_tensor_model_parallel_allreduce,
                                                   self.sequence_parallel_enabled, self.kv_size_multiplier)

    def forward(self, input: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        out = self.forward_fused(input)
        q_l, kv_l = self.q_output_size_per_partition, self.kv_output_size_per_partition
        q, k, v = out[..., :q_l], out[..., q_l:q_l + kv_l], out[..., q_l + kv_l:]
        if self.gather_output:
            q = gather_from_tensor_model_parallel_region(q)
            k = gather_from_tensor_model_parallel_region(k)
            v = gather_from_tensor_model_parallel_region(v)
        return q, k, v

    def get_parameter_names(self):
        return ["weight_qkv"] if self.fuse_qkv else ["weight_q", "weight_k", "weight_v"]
