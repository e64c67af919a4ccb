"""GEMM entry points of the linear layers (csrc/gemm.cpp: hipBLASLt with per-shape autotuning).

`linear(x, w)` = x @ w^T, `matmul(a, b)` = a @ b, `wgrad_accumulate_(mg, go, x)` does
mg += go^T @ x with bf16 operands accumulating into the fp32 `main_grad` in place (one GEMM with
beta = 1, no bf16 temporary).  On CPU, or with NXD_TUNED_GEMM=0, they fall back to torch.
"""

from __future__ import annotations

import os

import torch

from ._ext import ext, use_native

_ENABLED = os.environ.get("NXD_TUNED_GEMM", "1") == "1"


def _native(*t: torch.Tensor) -> bool:
    return _ENABLED and use_native(*t) and all(x.dtype in (torch.bfloat16, torch.float16) for x in t)


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, out: torch.Tensor = None) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T -> [..., N] (written into `out` if given: contiguous [..., N])."""
    shape = x.shape[:-1] + (w.shape[0],)
    if _native(x, w) and x.stride(-1) == 1:
        x2 = x.reshape(-1, x.shape[-1])
        y = out if out is not None else torch.empty(shape, dtype=x.dtype, device=x.device)
        ext().gemm(x2, w.t(), y.view(-1, w.shape[0]), None, 1.0, 0.0)
        return y + bias if bias is not None else y
    y = torch.nn.functional.linear(x, w, bias)
    if out is not None:
        out.copy_(y)
        return out
    return y


def matmul(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """a [..., K] @ b [K, N] -> [..., N] (written into `out` if given: contiguous [..., N])."""
    shape = a.shape[:-1] + (b.shape[1],)
    if _native(a, b) and a.stride(-1) == 1:
        a2 = a.reshape(-1, a.shape[-1])
        y = out if out is not None else torch.empty(shape, dtype=a.dtype, device=a.device)
        ext().gemm(a2, b, y.view(-1, b.shape[1]), None, 1.0, 0.0)
        return y
    y = torch.matmul(a, b)
    if out is not None:
        out.copy_(y)
        return out
    return y


_WGRAD_BF16 = os.environ.get("NXD_WGRAD_BF16", "0") == "1"
_scratch = {}


def _wgrad_scratch(n: int, dtype, device) -> torch.Tensor:
    key = (dtype, str(device))
    t = _scratch.get(key)
    if t is None or t.numel() < n:
        t = _scratch[key] = torch.empty(n, dtype=dtype, device=device)
    return t[:n]


def wgrad_accumulate_(mg: torch.Tensor, go2: torch.Tensor, x2: torch.Tensor) -> None:
    """mg [N, K] (fp32) += go2[T, N]^T @ x2[T, K].

    Default: one hipBLASLt GEMM with fp32 C/D and beta = 1.  NXD_WGRAD_BF16=1: bf16-output GEMM
    into a reused scratch, then an fp32 add (the per-micro-batch weight gradient is rounded to
    bf16 before the fp32 accumulation — the precision of the reference's XLA matmul + fp32
    grad accumulation; hipBLASLt's bf16-output solutions run faster than its fp32-output ones)."""
    if _native(go2, x2) and mg.is_contiguous():
        if _WGRAD_BF16:
            tmp = _wgrad_scratch(mg.numel(), go2.dtype, go2.device).view(mg.shape)
            ext().gemm(go2.t(), x2, tmp, None, 1.0, 0.0)
            mg.add_(tmp)
            return
        ext().gemm(go2.t(), x2, mg, None, 1.0, 1.0)
        return
    if go2.is_cuda:
        torch.addmm(mg, go2.t(), x2, out_dtype=torch.float32, out=mg)
    else:
        mg.add_(go2.t().float().matmul(x2.float()))
