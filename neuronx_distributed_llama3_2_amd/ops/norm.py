"""RMSNorm (optionally fused with the pre-norm residual add) on csrc/rmsnorm.hip.

Weight gradients follow the framework's gradient-buffer convention: if the weight carries a
`main_grad` fp32 buffer (a view into the flat gradient buffer, see parallel/grad_buffer.py) the
kernel's column reduction accumulates into it directly and autograd gets `None` for the weight;
otherwise a regular `.grad` is returned.  Sequence-parallel norm weights are tagged
`sequence_parallel_enabled` so their gradients are all-reduced over TP
(reference: src/neuronx_distributed/parallel_layers/grads.py:313-329).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._ext import ext, use_native


def rms_norm_reference(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def _notify_grad(param):
    cb = getattr(param, "_nxd_grad_ready", None)
    if cb is not None:
        cb(param)


def _weight_grad(w: torch.Tensor, dw32: torch.Tensor):
    """Return the autograd grad for `w` given an fp32 dW (or None if accumulated into main_grad)."""
    mg = getattr(w, "main_grad", None)
    if mg is not None:
        _notify_grad(w)
        return None
    return dw32.to(w.dtype)


class RMSNormFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, residual):
        H = x.shape[-1]
        xc = x.contiguous()
        y = torch.empty_like(xc)
        rstd = torch.empty(xc.numel() // H, dtype=torch.float32, device=x.device)
        if residual is not None:
            h = torch.empty_like(xc)
            ext().rmsnorm_fwd(xc, residual.contiguous(), w, y, h, rstd, float(eps))
        else:
            h = xc
            ext().rmsnorm_fwd(xc, None, w, y, None, rstd, float(eps))
        ctx.save_for_backward(h, w, rstd)
        ctx.has_res = residual is not None
        if residual is not None:
            return y, h
        return y, None

    @staticmethod
    def backward(ctx, dy, dh_extra):
        h, w, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(h)
        mg = getattr(w, "main_grad", None)
        if mg is not None:
            dw = mg
            accumulate = True
        else:
            dw = torch.empty(w.numel(), dtype=torch.float32, device=w.device)
            accumulate = False
        dres = dh_extra.contiguous() if (ctx.has_res and dh_extra is not None) else None
        if accumulate:
            from ..parallel_layers import stream_split   # (lazy: parallel_layers imports ops)

            stream_split.accumulate_begin(w)
        ext().rmsnorm_bwd(dy, h, w, rstd, dres, dx, dw.view(-1), accumulate)
        if accumulate:
            stream_split.accumulate_end(w)
        gw = _weight_grad(w, dw)
        if ctx.has_res:
            # h = x + residual: both inputs get the same gradient
            return dx, gw, None, dx
        return dx, gw, None, None


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5,
             residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns (y, h) where h = x + residual (or None without residual) and y = RMSNorm(h)."""
    if use_native(x, weight):
        y, h = RMSNormFunc.apply(x, weight, eps, residual)
        return y, h
    h = x + residual if residual is not None else None
    src = h if h is not None else x
    return rms_norm_reference(src, weight, eps), h
