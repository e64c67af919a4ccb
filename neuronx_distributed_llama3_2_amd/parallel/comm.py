"""Collective primitives used by every parallel component.

On GPUs these are single RCCL calls (torch.distributed NCCL backend = RCCL over xGMI) on flat,
contiguous buffers: `all_gather_into_tensor`, `reduce_scatter_tensor`, `all_reduce`,
`all_to_all_single`, `batch_isend_irecv`.  Async variants return the RCCL work handle so callers
overlap communication with compute (the collective runs on RCCL's internal stream and the
consumer waits on it before use).

The gloo backend (CPU test harness) lacks the "_base" flat-tensor collectives; the same calls are
emulated there with list all-gathers / all-reduce + slice, so the parallel code paths are the same
on CPU and GPU.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


def _is_gloo(group) -> bool:
    try:
        return dist.get_backend(group) == "gloo"
    except Exception:  # pragma: no cover
        return False


def all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """out[i*n:(i+1)*n] = inp of rank i (dim 0)."""
    if not _is_gloo(group):
        return dist.all_gather_into_tensor(out, inp.contiguous(), group=group, async_op=async_op)
    ws = dist.get_world_size(group=group)
    chunks = list(out.chunk(ws, dim=0))
    src = inp.detach().contiguous().cpu()   # gloo gathers host tensors (GPU tensors are staged)
    tmp = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(tmp, src, group=group)
    for c, t in zip(chunks, tmp):
        c.copy_(t)
    return _Done() if async_op else None


def reduce_scatter_tensor(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False,
                          op=dist.ReduceOp.SUM):
    """out = sum over ranks of inp[rank*n:(rank+1)*n] (dim 0)."""
    if not _is_gloo(group):
        return dist.reduce_scatter_tensor(out, inp.contiguous(), op=op, group=group, async_op=async_op)
    ws = dist.get_world_size(group=group)
    r = dist.get_rank(group=group)
    full = inp.contiguous().clone()
    dist.all_reduce(full, op=op, group=group)
    out.copy_(full.chunk(ws, dim=0)[r])
    return _Done() if async_op else None


def all_reduce(t: torch.Tensor, group=None, async_op: bool = False, op=dist.ReduceOp.SUM):
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    if not _is_gloo(group):
        return dist.all_to_all_single(out, inp.contiguous(), group=group, async_op=async_op)
    ws = dist.get_world_size(group=group)
    ins = list(inp.contiguous().chunk(ws, dim=0))
    outs = [torch.empty_like(c) for c in ins]
    _a2a_via_gather(outs, ins, group)
    for o, c in zip(out.chunk(ws, dim=0), outs):
        o.copy_(c)
    return _Done() if async_op else None


def _a2a_via_gather(outs: List[torch.Tensor], ins: List[torch.Tensor], group):
    """gloo has no all_to_all: every rank all-gathers the stacked chunks and keeps its column."""
    ws = dist.get_world_size(group=group)
    r = dist.get_rank(group=group)
    stacked = torch.stack(ins).cpu()
    gathered = [torch.empty_like(stacked) for _ in range(ws)]
    dist.all_gather(gathered, stacked, group=group)
    for src in range(ws):
        outs[src].copy_(gathered[src][r])


def send(t: torch.Tensor, dst: int, group=None):
    return dist.isend(t.contiguous(), dst, group=group)


def recv(t: torch.Tensor, src: int, group=None):
    return dist.irecv(t, src, group=group)


def batch_isend_irecv(ops: List[dist.P2POp]):
    if not ops:
        return []
    return dist.batch_isend_irecv(ops)
