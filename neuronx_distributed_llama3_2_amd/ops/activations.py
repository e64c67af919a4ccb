"""SwiGLU on a fused gate_up projection (csrc/swiglu.hip).

The backward also writes d(gate_up) transposed ([2I, T], token-contiguous) when the shape tiles by
64: the gate_up weight gradient runs as a TN GEMM on T-contiguous operands (ops/gemm.py), and the
transposed copy — attached to the returned gradient as `_nxd_t` — replaces the separate transpose
of the layer's largest activation gradient.  NXD_SWIGLU_DUAL=0 disables it.  Likewise the forward
(under autograd) writes h transposed, `h._nxd_t`, which the down projection saves in place of h for
its TN weight gradient (NXD_SWIGLU_DUAL_FWD=0 disables).
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._ext import ext, use_native


def swiglu_reference(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


_DUAL = os.environ.get("NXD_SWIGLU_DUAL", "1") == "1"
_DUAL_FWD = os.environ.get("NXD_SWIGLU_DUAL_FWD", "1") == "1"


class SwiGLUFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, want_t=False, want_grad_t=False):
        gu = gu.contiguous()
        ctx.want_grad_t = want_grad_t
        h = torch.empty(gu.shape[:-1] + (gu.shape[-1] // 2,), dtype=gu.dtype, device=gu.device)
        I = h.shape[-1]
        rows = h.numel() // I if I else 0
        if want_t and rows and rows % 64 == 0 and I % 64 == 0:
            # token-contiguous copy of h for the down projection's weight gradient (saved by the
            # next linear instead of h itself, see parallel_layers/layers.py)
            h_t = torch.empty((I, rows), dtype=gu.dtype, device=gu.device)
            ext().swiglu_fwd_dual(gu, h, h_t)
            h._nxd_t, h._nxd_t_ver = h_t, h._version
        else:
            ext().swiglu_fwd(gu, h)
        ctx.save_for_backward(gu)
        return h

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        dgu = torch.empty_like(gu)
        I2 = gu.shape[-1]
        rows = gu.numel() // I2 if I2 else 0
        if ctx.want_grad_t and _DUAL and rows and rows % 64 == 0 and (I2 // 2) % 64 == 0:
            dgu_t = torch.empty((I2, rows), dtype=gu.dtype, device=gu.device)
            ext().swiglu_bwd_dual(gu, dh.contiguous(), dgu, dgu_t)
            dgu._nxd_t, dgu._nxd_t_ver = dgu_t, dgu._version
            return dgu, None, None
        ext().swiglu_bwd(gu, dh.contiguous(), dgu)
        return dgu, None, None


def attached_token_major(x: torch.Tensor):
    """The producer-written transposed copy attached to `x` (`x._nxd_t`), or None when there is
    none or `x` was modified in place since it was written (in-place dropout, hooks, autograd
    accumulation): the copy is then stale and the consumer must transpose `x` itself."""
    t = getattr(x, "_nxd_t", None)
    if t is None or getattr(x, "_nxd_t_ver", None) != x._version:
        return None
    return t


def swiglu(gu: torch.Tensor, token_major: bool = False) -> torch.Tensor:
    """h = silu(gate) * up for gu = [gate | up] along the last dim.

    token_major=True: the caller feeds gu from, and h into, the framework's linear layers (dense
    MLP), which consume the token-major copies; other callers (MoE grouped GEMMs) would only pay
    for them."""
    if use_native(gu):
        train = token_major and torch.is_grad_enabled() and gu.requires_grad
        return SwiGLUFunc.apply(gu, _DUAL_FWD and train, train)
    return swiglu_reference(gu)
