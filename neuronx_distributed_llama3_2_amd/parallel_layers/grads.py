"""Gradient utilities: global grad norm / clipping over TP+PP(+EP) and bucketed DP reductions
(reference: src/neuronx_distributed/parallel_layers/grads.py:33-329).

* Norms are computed with fused multi-tensor reductions (`torch._foreach_norm`, or the flat-buffer
  HIP kernel when gradients live in one buffer) — not one `torch.norm` per tensor; the result stays
  on the device (no host sync) and clipping multiplies by a device-side coefficient.
* TP-duplicated parameters (norm weights, row-parallel biases) are counted once (on TP rank 0),
  TP-sharded ones on every rank, then the partial sums are all-reduced over TP and PP.  K/V rows
  of a GQA QKV projection whose kv heads are replicated on m ranks (`qkv_split[2] = m`) are the
  same parameter m times: their squares count 1/m on each replica, so the norm (and clipping) is
  the unsharded model's at every TP degree.  (The reference counts them m times.)
* DP reduction coalesces gradients into per-dtype buckets (default 128 MiB:
  `ALLREDUCE_BUCKET_CAP_MB`) — sized so each RCCL ring chunk over the 7 xGMI links stays in the
  bandwidth regime — reduced in reverse registration order.
"""

from __future__ import annotations

import os
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

from .parallel_state import (
    get_data_parallel_group,
    get_data_parallel_size,
    get_expert_data_parallel_group,
    get_expert_data_parallel_size,
    get_expert_model_parallel_group,
    get_expert_model_parallel_size,
    get_pipeline_model_parallel_group,
    get_pipeline_model_parallel_size,
    get_tensor_model_parallel_group,
    get_tensor_model_parallel_rank,
    get_tensor_model_parallel_size,
    model_parallel_is_initialized,
)


def _bucket_cap_bytes() -> int:
    return int(float(os.environ.get("ALLREDUCE_BUCKET_CAP_MB", "128")) * 1024 * 1024)


def param_is_not_shared(param) -> bool:
    return not getattr(param, "shared", False)


def _is_tp_dup(p) -> bool:
    return not getattr(p, "tensor_model_parallel", False)


def _grad_of(p):
    g = getattr(p, "main_grad", None)
    return g if g is not None else p.grad


def kv_replica_slices(p):
    """(first row, weight) of the replicated K/V rows of a fused GQA QKV weight/bias `p`: rows from
    `first row` on are kv heads held by `m` ranks each, weight 1/m.  None for other parameters."""
    qs = getattr(p, "qkv_split", None)
    if not qs or int(qs[2]) <= 1 or not model_parallel_is_initialized():
        return None
    q_rows, _, mult = qs
    return q_rows // get_tensor_model_parallel_size(), 1.0 / float(mult)


def get_grad_norm(parameters, norm_type: float = 2, zero1_optimizer: bool = False, zero1_optimizer_groups=None,
                  force_spmd: bool = True) -> torch.Tensor:
    """Global gradient norm (device tensor) over every model-parallel dimension."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if _grad_of(p) is not None and param_is_not_shared(p)]
    norm_type = float(norm_type)
    tp_rank = get_tensor_model_parallel_rank() if model_parallel_is_initialized() else 0
    dev = _grad_of(params[0]).device if params else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    ep_params = [p for p in params if getattr(p, "expert_model_parallel", False)]
    dense = [p for p in params if not getattr(p, "expert_model_parallel", False)]

    def local_stat(ps):
        grads = [_grad_of(p) for p in ps if (not _is_tp_dup(p)) or tp_rank == 0]
        if not grads:
            return torch.zeros(1, dtype=torch.float32, device=dev)
        if norm_type == float("inf"):
            return torch.stack([g.detach().abs().max().float() for g in grads]).max().reshape(1)
        norms = torch._foreach_norm([g.detach() for g in grads], norm_type)
        tot = torch.stack([n.float() for n in norms]).pow(norm_type).sum().reshape(1)
        for p in ps:   # replicated K/V rows count 1/m per replica
            kv = kv_replica_slices(p)
            if kv is not None:
                g = _grad_of(p).detach()[kv[0]:]
                tot = tot - (1.0 - kv[1]) * g.float().norm(norm_type).pow(norm_type)
        return tot

    op = dist.ReduceOp.MAX if norm_type == float("inf") else dist.ReduceOp.SUM
    total = local_stat(dense)
    if ep_params:
        ep_total = local_stat(ep_params)
        if model_parallel_is_initialized() and get_expert_model_parallel_size() > 1:
            dist.all_reduce(ep_total, op=op, group=get_expert_model_parallel_group())
        total = torch.maximum(total, ep_total) if op == dist.ReduceOp.MAX else total + ep_total
    if model_parallel_is_initialized():
        if get_tensor_model_parallel_size() > 1:
            dist.all_reduce(total, op=op, group=get_tensor_model_parallel_group())
        if get_pipeline_model_parallel_size() > 1:
            dist.all_reduce(total, op=op, group=get_pipeline_model_parallel_group())
        if zero1_optimizer and zero1_optimizer_groups is not None:
            dist.all_reduce(total, op=op, group=zero1_optimizer_groups)
    if norm_type == float("inf"):
        return total[0]
    return total[0].pow(1.0 / norm_type)


def clip_grads_with_norm(parameters, total_norm: torch.Tensor, max_norm: float) -> None:
    coef = torch.clamp(max_norm / (total_norm + 1e-6), max=1.0)
    grads = [_grad_of(p) for p in parameters if _grad_of(p) is not None]
    if grads:
        torch._foreach_mul_(grads, coef.to(grads[0].device))


def clip_grad_norm(parameters, max_norm: float, norm_type: float = 2, zero1_optimizer: bool = False,
                   zero1_optimizer_groups=None, force_spmd: bool = True) -> torch.Tensor:
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(parameters)
    total = get_grad_norm(parameters, norm_type, zero1_optimizer, zero1_optimizer_groups, force_spmd)
    clip_grads_with_norm(parameters, total, max_norm)
    return total


def _allreduce_bucketed(tensors: List[torch.Tensor], group, average_by: int = 1) -> None:
    """Coalesce into <= cap-byte flat buckets per dtype (reverse order), all-reduce, scatter back."""
    if not tensors or dist.get_world_size(group=group) == 1:
        return
    cap = _bucket_cap_bytes()
    by_dtype = {}
    for t in reversed(tensors):
        by_dtype.setdefault(t.dtype, []).append(t)
    for _, ts in by_dtype.items():
        buckets, cur, size = [], [], 0
        for t in ts:
            nb = t.numel() * t.element_size()
            if cur and size + nb > cap:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(t)
            size += nb
        if cur:
            buckets.append(cur)
        for bucket in buckets:
            flat = torch.cat([b.reshape(-1) for b in bucket])
            dist.all_reduce(flat, group=group)
            if average_by > 1:
                flat.div_(average_by)
            off = 0
            for b in bucket:
                n = b.numel()
                b.copy_(flat[off:off + n].view_as(b))
                off += n


def bucket_allreduce_gradients(grads_list: List[torch.Tensor], reduce_over_ep_group: bool = False) -> None:
    """All-reduce (sum) gradients over DP — or, for expert grads, over expert-DP (reference :243-310)."""
    if not model_parallel_is_initialized():
        return
    if reduce_over_ep_group:
        if get_expert_data_parallel_size() > 1:
            _allreduce_bucketed(grads_list, get_expert_data_parallel_group())
        return
    if get_data_parallel_size() > 1:
        _allreduce_bucketed(grads_list, get_data_parallel_group())


def allreduce_sequence_parallel_gradients(optimizer_or_params) -> None:
    """Sum over TP the grads of params replicated across TP whose inputs were sequence-sharded
    (norm weights, row biases) — one coalesced all-reduce (reference grads.py:313-329, X15)."""
    if not model_parallel_is_initialized() or get_tensor_model_parallel_size() == 1:
        return
    if hasattr(optimizer_or_params, "param_groups"):
        params = [p for g in optimizer_or_params.param_groups for p in g["params"]]
    else:
        params = list(optimizer_or_params)
    grads = [_grad_of(p) for p in params if getattr(p, "sequence_parallel_enabled", False) and _grad_of(p) is not None]
    if not grads:
        return
    _allreduce_bucketed(grads, get_tensor_model_parallel_group())
