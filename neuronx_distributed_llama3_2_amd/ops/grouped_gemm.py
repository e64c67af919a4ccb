"""Grouped (ragged-M) expert GEMMs for dropless MoE (csrc/grouped_gemm.hip) and the device-side
token permutation around them.

Tokens are sorted by their chosen expert on the device; expert e owns rows offs[e]:offs[e+1] of
the sorted activations.  Nothing here reads a group size on the host, so a dropless MoE layer has
no device->host sync (reference: modules/moe/expert_mlps.py:169-265, utils/tensor_utils.py:4-62).

GPU tensors run the HIP kernels (forward, input gradient and the fp32 weight gradient, which is
accumulated straight into `main_grad` when the flat gradient buffer provides one); CPU tensors run
the plain-PyTorch reference (per-expert matmuls over the host-known offsets).
"""

from __future__ import annotations

from typing import Tuple

import torch

from ._ext import ext, use_native


def moe_permutation(expert_index: torch.Tensor, num_experts: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Stable sort of the T*k (token, choice) slots by expert, all on the device.

    Returns (order, inverse, offs): sorted slot s holds flat slot order[s] (token order[s] // k),
    flat slot i sits at sorted row inverse[i], and offs int32 [E + 1] are the group boundaries.
    """
    flat = expert_index.reshape(-1)
    order = torch.argsort(flat, stable=True)
    inverse = torch.empty_like(order)
    inverse.scatter_(0, order, torch.arange(order.numel(), device=order.device, dtype=order.dtype))
    counts = torch.zeros(num_experts, dtype=torch.int32, device=flat.device)
    counts.scatter_add_(0, flat.long(), torch.ones_like(flat, dtype=torch.int32))
    offs = torch.zeros(num_experts + 1, dtype=torch.int32, device=flat.device)
    offs[1:] = torch.cumsum(counts, 0, dtype=torch.int32)
    return order, inverse, offs


def grouped_linear_reference(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """y[offs[e]:offs[e+1]] = x[offs[e]:offs[e+1]] @ w[e] (fp32 accumulate), differentiable."""
    bounds = offs.tolist()
    outs = []
    for e in range(w.shape[0]):
        lo, hi = bounds[e], bounds[e + 1]
        if hi > lo:
            outs.append((x[lo:hi].float() @ w[e].float()).to(x.dtype))
    if not outs:
        return x.new_zeros(x.shape[0], w.shape[2]) + 0 * x.sum() * w.sum()
    y = torch.cat(outs, 0)
    if y.shape[0] < x.shape[0]:   # rows past offs[E] (none in a well-formed permutation)
        y = torch.cat([y, y.new_zeros(x.shape[0] - y.shape[0], y.shape[1])], 0)
    return y


class GroupedLinearFunc(torch.autograd.Function):
    """y = x @ W[e] per expert group; dx = dy @ W[e]^T; dW[e] = x_e^T dy_e (fp32)."""

    @staticmethod
    def forward(ctx, x, w, offs):
        x = x.contiguous()
        y = torch.empty(x.shape[0], w.shape[2], dtype=x.dtype, device=x.device)
        ext().grouped_gemm(0, x, w, offs, y, False)
        ctx.save_for_backward(x, w, offs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, offs = ctx.saved_tensors
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            ext().grouped_gemm(1, dy, w, offs, dx, False)
        dw = None
        if ctx.needs_input_grad[1]:
            mg = getattr(w, "main_grad", None)
            if mg is not None and mg.dtype == torch.float32 and mg.is_contiguous():
                ext().grouped_gemm(2, x, dy, offs, mg, True)
                cb = getattr(w, "_nxd_grad_ready", None)
                if cb is not None:
                    cb(w)
            else:
                g = torch.empty(w.shape, dtype=torch.float32, device=w.device)
                ext().grouped_gemm(2, x, dy, offs, g, False)
                if mg is not None:
                    mg.add_(g.to(mg.dtype))
                    cb = getattr(w, "_nxd_grad_ready", None)
                    if cb is not None:
                        cb(w)
                else:
                    dw = g.to(w.dtype)
        return dx, dw, None


def grouped_linear(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """Expert-grouped linear over expert-sorted rows: x [M, K], w [E, K, N], offs int32 [E + 1]."""
    if use_native(x, w, offs):
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
            raise TypeError("grouped_linear: the HIP kernel takes bf16 activations and weights")
        return GroupedLinearFunc.apply(x, w, offs)
    return grouped_linear_reference(x, w, offs)
