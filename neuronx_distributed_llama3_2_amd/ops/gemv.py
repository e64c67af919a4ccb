"""Decode-path linear ops (csrc/gemv.hip): skinny GEMM for M <= 8 tokens with bf16 or int8 weights,
optional per-row / per-tensor scale, bias and fused SwiGLU epilogue; int8 -> bf16 dequantisation
for the prefill path.  CPU / large-M calls fall back to dequantise + GEMM."""

from __future__ import annotations

from typing import Optional

import torch

from ._ext import ext, use_native
from .gemm import linear as _linear


def dequantize_weight(w: torch.Tensor, scale: Optional[torch.Tensor], dtype=torch.bfloat16) -> torch.Tensor:
    """int8 [N, K] (* scale [N] / [N,1] / [1]) -> dtype [N, K]; bf16 weights pass through."""
    if w.dtype != torch.int8:
        return w
    if use_native(w) and dtype == torch.bfloat16 and w.shape[1] % 16 == 0:
        s = scale.reshape(-1).float().contiguous() if scale is not None else None
        out = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
        if s is not None and s.numel() == 1:
            ext().dequant_int8(w, s.expand(w.shape[0]).contiguous(), 1.0, out)
        else:
            ext().dequant_int8(w, s, 1.0, out)
        return out
    if scale is None:
        s = 1.0
    elif scale.numel() == 1:
        s = scale.float().reshape(())
    else:
        s = scale.float().reshape(-1, 1)
    return (w.float() * s).to(dtype)


def skinny_linear(x: torch.Tensor, w: torch.Tensor, scale: Optional[torch.Tensor] = None,
                  bias: Optional[torch.Tensor] = None, glu: bool = False) -> torch.Tensor:
    """x [..., K] @ W^T (+ bias) (W bf16 or int8 [Nw, K]); glu=True: W = [gate; up] rows and the
    result is silu(gate) * up of width Nw / 2."""
    K = x.shape[-1]
    lead = x.shape[:-1]
    M = x.numel() // K
    Nw = w.shape[0]
    N = Nw // 2 if glu else Nw
    if use_native(x, w) and M <= 8 and x.dtype == torch.bfloat16 and w.stride(-1) == 1:
        x2 = x.reshape(M, K)
        if x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        epl = 16 if w.dtype == torch.int8 else 8
        if K % epl == 0 and w.data_ptr() % 16 == 0 and w.stride(0) % epl == 0:
            y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
            s = None
            if scale is not None:
                s = scale.reshape(-1).float()
                s = (s.expand(Nw) if s.numel() == 1 else s).contiguous()
            ext().gemv(x2, w, s, 1.0, bias, y, glu)
            return y.view(lead + (N,))
    wd = dequantize_weight(w, scale, x.dtype) if w.dtype == torch.int8 else w
    y = _linear(x, wd, bias)
    if glu:
        from .activations import swiglu

        y = swiglu(y)
    return y


def expert_linear(x: torch.Tensor, w_t: torch.Tensor, eidx: torch.Tensor, xdiv: int = 1,
                  glu: bool = False) -> torch.Tensor:
    """MoE decode projection for P (token, expert-slot) pairs: y[p] = x[p // xdiv] @ W[eidx[p]]^T,
    W given output-major as w_t [E, Nw, K]; glu=True: rows [gate; up] -> silu(gate) * up.  Reads
    only the selected experts' weights (csrc/gemv.hip expert mode); static shapes, no host sync,
    so it is captured in the decode hipGraph."""
    P = eidx.numel()
    Nw, K = w_t.shape[1], w_t.shape[2]
    N = Nw // 2 if glu else Nw
    if use_native(x, w_t) and x.dtype == torch.bfloat16 and w_t.dtype == torch.bfloat16 and w_t.stride(2) == 1 \
            and K % 8 == 0 and w_t.stride(1) % 8 == 0 and w_t.stride(0) % 8 == 0 and w_t.data_ptr() % 16 == 0:
        x2 = x.reshape(-1, K)
        if x2.stride(1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        y = torch.empty((P, N), dtype=torch.bfloat16, device=x.device)
        ext().expert_gemv(x2, w_t, eidx.reshape(-1).to(torch.int32).contiguous(), int(xdiv), y, glu)
        return y
    rows = x.reshape(-1, K).index_select(0, torch.arange(P, device=x.device) // xdiv)
    y = torch.bmm(rows.unsqueeze(1), w_t.index_select(0, eidx.reshape(-1).long()).transpose(1, 2)).squeeze(1)
    if glu:
        from .activations import swiglu

        y = swiglu(y)
    return y
