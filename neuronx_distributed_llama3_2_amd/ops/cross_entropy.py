"""Vocab-parallel cross entropy on csrc/xent.hip.

Semantics match the reference `parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing)`
(src/neuronx_distributed/parallel_layers/loss_functions.py:11-135): logits are sharded along the
vocabulary over the tensor-parallel group, the loss is per token (no reduction).  Differences by
design: a single all-gather of per-row (max, sum-exp, target-logit, sum-logit) statistics replaces
the reference's three all-reduces, no fp64 copy of the logits is made, and the backward can
overwrite the logits buffer with the gradient (`inplace_backward`, saves a [N, V/tp] tensor).
Tokens equal to `ignore_index` get zero loss and zero gradient.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..parallel import comm

from ._ext import ext, use_native


def _combine(stats: torch.Tensor, group, world: int):
    """stats [N, 4] local -> (M, S, target_logit, sum_logits) global over the TP group.

    TP = 1 takes the columns as they are: reducing over a size-1 leading dim of the strided
    [1, N] view ran as torch's generic reduce_kernel at ~2.9 ms per call (8 calls, 23 ms of a
    3-s bench step: profiles/r4f_step_breakdown_tp1_halves_by_kernel.txt).  TP > 1 reduces over the
    rank axis laid out innermost ([N, 4, W] contiguous)."""
    if world == 1:
        return stats[:, 0], stats[:, 1], stats[:, 2], stats[:, 3]
    gathered = torch.empty((world,) + tuple(stats.shape), dtype=stats.dtype, device=stats.device)
    comm.all_gather_into_tensor(gathered, stats.contiguous(), group=group)
    g = gathered.permute(1, 2, 0).contiguous()            # [N, 4, W]
    m, s = g[:, 0], g[:, 1]
    M = m.amax(dim=-1)
    w = torch.where(m == float("-inf"), torch.zeros_like(m), torch.exp(m - M[:, None]))
    S = (s * w).sum(-1)
    T = g[:, 2].sum(-1)
    X = g[:, 3].sum(-1)
    return M, S, T, X


class ParallelCrossEntropyFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, label_smoothing, ignore_index, group, world, rank, inplace_backward):
        N_shape = target.shape
        V = logits.shape[-1]
        x = logits.reshape(-1, V)
        t = target.reshape(-1).contiguous().to(torch.int64)
        vocab_start = rank * V
        stats = torch.empty((x.shape[0], 4), dtype=torch.float32, device=x.device)
        ext().xent_stats(x, t, stats, vocab_start)
        M, S, T, X = _combine(stats, group, world)
        lse = torch.log(S) + M
        vtot = V * world
        nll = lse - T
        if label_smoothing > 0:
            loss = (1.0 - label_smoothing) * nll + label_smoothing * (lse - X / vtot)
        else:
            loss = nll
        valid = t != ignore_index
        loss = torch.where(valid, loss, torch.zeros_like(loss))
        ctx.save_for_backward(logits, t, M, S, valid)
        ctx.meta = (label_smoothing, world, rank, V, inplace_backward)
        return loss.view(N_shape)

    @staticmethod
    def backward(ctx, g):
        logits, t, M, S, valid = ctx.saved_tensors
        eps, world, rank, V, inplace = ctx.meta
        x = logits.reshape(-1, V)
        gv = torch.where(valid, g.reshape(-1).float(), torch.zeros_like(M))
        gstat = torch.stack([M, 1.0 / S, gv, torch.zeros_like(M)], dim=1).contiguous()
        if inplace and logits.dtype == torch.bfloat16:
            grad = x
        else:
            grad = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        ext().xent_bwd(x, t, gstat, grad, rank * V, float(eps), V * world)
        grad = grad.view(logits.shape)
        if grad.dtype != logits.dtype:
            grad = grad.to(logits.dtype)
        return grad, None, None, None, None, None, None, None


def parallel_cross_entropy_reference(logits, target, label_smoothing=0.0, ignore_index=-100):
    """Single-shard (full vocabulary) fp32 reference."""
    lf = logits.float().reshape(-1, logits.shape[-1])
    t = target.reshape(-1)
    loss = torch.nn.functional.cross_entropy(lf, t.clamp(min=0), reduction="none", label_smoothing=label_smoothing)
    loss = torch.where(t == ignore_index, torch.zeros_like(loss), loss)
    return loss.view(target.shape)


def vocab_parallel_cross_entropy(logits: torch.Tensor, target: torch.Tensor, label_smoothing: float = 0.0,
                                 ignore_index: int = -100, group=None, world: int = 1, rank: int = 0,
                                 inplace_backward: bool = False) -> torch.Tensor:
    if use_native(logits):
        return ParallelCrossEntropyFunc.apply(logits, target, label_smoothing, ignore_index, group, world, rank,
                                              inplace_backward)
    return _ParallelCrossEntropyRef.apply(logits, target, label_smoothing, ignore_index, group, world, rank)


class _ParallelCrossEntropyRef(torch.autograd.Function):
    """Torch reference of the sharded loss (works on gloo/CPU); same math as the kernel path."""

    @staticmethod
    def forward(ctx, logits, target, label_smoothing, ignore_index, group, world, rank):
        V = logits.shape[-1]
        x = logits.reshape(-1, V).float()
        t = target.reshape(-1).to(torch.int64)
        start = rank * V
        m = x.max(dim=-1).values
        s = torch.exp(x - m[:, None]).sum(-1)
        local = t - start
        inr = (local >= 0) & (local < V)
        tl = torch.where(inr, x.gather(1, local.clamp(0, V - 1)[:, None]).squeeze(1), torch.zeros_like(m))
        stats = torch.stack([m, s, tl, x.sum(-1)], dim=1)
        M, S, T, X = _combine(stats, group, world)
        lse = torch.log(S) + M
        nll = lse - T
        vtot = V * world
        loss = (1 - label_smoothing) * nll + label_smoothing * (lse - X / vtot) if label_smoothing > 0 else nll
        valid = t != ignore_index
        loss = torch.where(valid, loss, torch.zeros_like(loss))
        ctx.save_for_backward(x, local, inr, M, S, valid)
        ctx.meta = (label_smoothing, vtot, logits.dtype, logits.shape)
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, g):
        x, local, inr, M, S, valid = ctx.saved_tensors
        eps, vtot, dtype, shape = ctx.meta
        p = torch.exp(x - M[:, None]) / S[:, None]
        onehot = torch.zeros_like(p)
        onehot.scatter_(1, local.clamp(0, x.shape[1] - 1)[:, None], inr.float()[:, None])
        grad = p - (1 - eps) * onehot - eps / vtot
        gv = torch.where(valid, g.reshape(-1).float(), torch.zeros_like(M))
        grad = grad * gv[:, None]
        return grad.to(dtype).view(shape), None, None, None, None, None, None
