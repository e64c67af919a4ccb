"""Flat-buffer optimizer primitives (csrc/optim.hip): multi-tensor grad norm, on-device clip
coefficient and a fused AdamW with fp32 master weights + bf16 copy-out.

All functions accept either GPU tensors (HIP kernels) or CPU tensors (torch reference), so the
optimizer logic above them is the same on both.
"""

from __future__ import annotations

from typing import Optional

import torch

from ._ext import ext, use_native


def flat_sumsq(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """out[0] (+)= sum(x^2) in fp32 for a contiguous flat buffer."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.numel() == 0:
        if not accumulate:
            out.zero_()
        return out
    if use_native(x):
        ext().flat_reduce(x.contiguous().view(-1), 0, out, accumulate)
        return out
    v = x.float().pow(2).sum()
    if accumulate:
        out += v
    else:
        out.fill_(float(v))
    return out


def flat_absmax(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.numel() == 0:
        if not accumulate:
            out.zero_()
        return out
    if use_native(x):
        ext().flat_reduce(x.contiguous().view(-1), 1, out, accumulate)
        return out
    v = x.float().abs().max()
    if accumulate:
        torch.maximum(out, v.reshape(1), out=out)
    else:
        out.fill_(float(v))
    return out


def clip_coefficient(stat: torch.Tensor, max_norm: float, is_sumsq: bool = True) -> torch.Tensor:
    """Device tensor [coef, norm] with coef = min(1, max_norm / (norm + 1e-6))."""
    coef = torch.empty(2, dtype=torch.float32, device=stat.device)
    if use_native(stat):
        ext().clip_coef(stat, coef, float(max_norm), bool(is_sumsq))
        return coef
    norm = stat[0].sqrt() if is_sumsq else stat[0]
    coef[0] = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    coef[1] = norm
    return coef


def _sr_hash(x: torch.Tensor) -> torch.Tensor:
    m = 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m
    return x ^ (x >> 16)


def stochastic_round_bf16(x: torch.Tensor, seed: int) -> torch.Tensor:
    """fp32 -> bf16 with stochastic rounding, bit-identical to the AdamW kernel's copy-out
    (csrc/optim.hip f2bf_sr): 16 hashed random bits of (seed, flat index) added below the bf16
    mantissa, then truncation; inf / nan round to nearest."""
    xf = x.detach().float().reshape(-1)
    u = xf.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    idx = torch.arange(xf.numel(), dtype=torch.int64, device=xf.device)
    h = _sr_hash((((idx * 0x9E3779B1) & 0xFFFFFFFF) ^ (idx >> 32) ^ (seed & 0xFFFFFFFF)) & 0xFFFFFFFF) & 0xFFFF
    t = ((u + h) & 0xFFFFFFFF) & 0xFFFF0000
    t = torch.where(t >= 2 ** 31, t - 2 ** 32, t).to(torch.int32)
    out = t.view(torch.float32).to(torch.bfloat16)
    special = (u & 0x7F800000) == 0x7F800000
    out = torch.where(special, xf.to(torch.bfloat16), out)
    return out.view(x.shape)


def sr_seed_for_step(step: int, base: int = 0x5EED) -> int:
    """Per-step seed (never 0: 0 means round-to-nearest in the kernel); identical on every rank so
    replicated parameters stay bit-identical."""
    x = (base * 0x9E3779B1 + step * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    x ^= x >> 16
    return x or 1


def adamw_flat_(p32: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
                p16: Optional[torch.Tensor], lr: float, beta1: float, beta2: float, eps: float, weight_decay: float,
                step: int, grad_scale: Optional[torch.Tensor] = None, grad_scale_host: float = 1.0,
                bias_correction: bool = True, sr_seed: int = 0, hyper: Optional[torch.Tensor] = None) -> None:
    """In-place AdamW (decoupled weight decay) over flat fp32 buffers; writes bf16 params to p16
    (stochastically rounded when sr_seed != 0).  hyper: optional device [lr, 1-beta1^t, 1-beta2^t]
    read by the kernel instead of lr / step (graph-captured optimizer steps)."""
    from .gemm import weights_updated

    weights_updated()   # the kernel writes weights behind autograd: K-major dgrad copies go stale
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    if use_native(p32, grad):
        ext().adamw_flat(p32, grad, exp_avg, exp_avg_sq, p16, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale,
                         grad_scale_host, int(sr_seed), hyper)
        return
    if hyper is not None:
        lr, bc1, bc2 = (float(x) for x in hyper[:3].tolist())
    g = grad.float() * grad_scale_host
    if grad_scale is not None:
        g = g * grad_scale[0]
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    denom = exp_avg_sq.sqrt() / (bc2 ** 0.5) + eps
    p32.mul_(1 - lr * weight_decay).addcdiv_(exp_avg, denom, value=-lr / bc1)
    if p16 is not None:
        if sr_seed and p16.dtype == torch.bfloat16:
            p16.copy_(stochastic_round_bf16(p32, sr_seed))
        else:
            p16.copy_(p32)


def scale_flat_(x: torch.Tensor, s: torch.Tensor) -> None:
    if use_native(x):
        ext().scale_flat(x, s)
    else:
        x.mul_(s[0])
