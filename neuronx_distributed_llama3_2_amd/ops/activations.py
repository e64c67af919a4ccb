"""SwiGLU on a fused gate_up projection (csrc/swiglu.hip)."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import ext, use_native


def swiglu_reference(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


class SwiGLUFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        h = torch.empty(gu.shape[:-1] + (gu.shape[-1] // 2,), dtype=gu.dtype, device=gu.device)
        ext().swiglu_fwd(gu, h)
        ctx.save_for_backward(gu)
        return h

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        dgu = torch.empty_like(gu)
        ext().swiglu_bwd(gu, dh.contiguous(), dgu)
        return dgu


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """h = silu(gate) * up for gu = [gate | up] along the last dim."""
    if use_native(gu):
        return SwiGLUFunc.apply(gu)
    return swiglu_reference(gu)
