"""Attention with dropout on the attention probabilities (reference: the NKI flash-attention
kernels take `dropout_p` and a seed, src/neuronx_distributed/kernels/flash_attn.py:85-148,151-191).

On the GPU the hand-written CDNA4 flash kernels apply the dropout themselves (csrc/flash_attn_fwd.hip
/ flash_attn_bwd.hip `DROP` variants): the keep mask is a counter-based hash of (seed, batch,
global head, query, key) -- `dropout_keep_mask` below is its definition, shared bit-for-bit with
the kernels' drop_row_hash / drop_keep (csrc/common.h) -- so nothing is stored and the backward
regenerates exactly the forward's mask.  This module also holds the host path (CPU, or shapes the
kernels do not take): the same flash decomposition -- query chunks, fp32 row log-sum-exp,
nothing of size S x S kept for backward -- as batched GEMMs; the test oracle for the kernels.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

_M32 = 0xFFFFFFFF
Q_CHUNK = 256


def _hash32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_keep_mask(seed: int, B: int, H: int, q_idx: torch.Tensor, S_k: int, p: float,
                      head_offset: int = 0) -> torch.Tensor:
    """bool [B, H, len(q_idx), S_k]: True where the probability is kept (heads numbered from
    head_offset, so a tensor-parallel rank draws the same mask as the unsharded model)."""
    dev = q_idx.device
    b = torch.arange(B, device=dev, dtype=torch.int64).view(B, 1, 1, 1)
    h = torch.arange(head_offset, head_offset + H, device=dev, dtype=torch.int64).view(1, H, 1, 1)
    qi = q_idx.to(torch.int64).view(1, 1, -1, 1)
    ki = torch.arange(S_k, device=dev, dtype=torch.int64).view(1, 1, 1, -1)
    x = (seed & _M32) ^ ((b * 0x9E3779B1) & _M32) ^ ((h * 0x85EBCA6B) & _M32)
    x = _hash32(x & _M32)
    x = _hash32((x ^ ((qi * 0xC2B2AE35) & _M32)) & _M32)
    x = _hash32((x ^ ((ki * 0x27D4EB2F) & _M32)) & _M32)
    thresh = int(p * 4294967296.0)
    return x >= thresh


def _expand_kv(t: torch.Tensor, hq: int) -> torch.Tensor:
    hkv = t.shape[1]
    return t if hkv == hq else t.repeat_interleave(hq // hkv, dim=1)


def _scores(qc, k, scale, q_idx, causal, offset):
    s = torch.matmul(qc.float(), k.float().transpose(-1, -2)) * scale      # [B, H, c, Sk]
    if causal:
        kk = torch.arange(k.shape[2], device=k.device)
        s = s.masked_fill(kk.view(1, 1, 1, -1) > (q_idx + offset).view(1, 1, -1, 1), float("-inf"))
    return s


class DropoutAttentionFunc(torch.autograd.Function):
    """q [B, Hq, Sq, D], k/v [B, Hkv, Sk, D] -> o [B, Hq, Sq, D] (layout bhsd)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, p, seed, head_offset):
        B, Hq, Sq, D = q.shape
        ke, ve = _expand_kv(k, Hq), _expand_kv(v, Hq)
        Sk = ke.shape[2]
        offset = Sk - Sq
        o = torch.empty_like(q)
        lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
        for c0 in range(0, Sq, Q_CHUNK):
            qi = torch.arange(c0, min(Sq, c0 + Q_CHUNK), device=q.device)
            s = _scores(q[:, :, c0:c0 + len(qi)], ke, scale, qi, causal, offset)
            l = torch.logsumexp(s, -1)
            prob = torch.exp(s - l.unsqueeze(-1))
            keep = dropout_keep_mask(seed, B, Hq, qi, Sk, p, head_offset)
            pd = prob * keep / (1.0 - p)
            o[:, :, c0:c0 + len(qi)] = torch.matmul(pd, ve.float()).to(q.dtype)
            lse[:, :, c0:c0 + len(qi)] = l
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (causal, scale, p, seed, head_offset)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, scale, p, seed, head_offset = ctx.cfg
        B, Hq, Sq, D = q.shape
        Hkv = k.shape[1]
        ke, ve = _expand_kv(k, Hq).float(), _expand_kv(v, Hq).float()
        Sk = ke.shape[2]
        offset = Sk - Sq
        dq = torch.empty_like(q)
        dk = torch.zeros(B, Hq, Sk, D, dtype=torch.float32, device=q.device)
        dv = torch.zeros_like(dk)
        delta = (do.float() * o.float()).sum(-1)                               # [B, H, Sq]
        for c0 in range(0, Sq, Q_CHUNK):
            qi = torch.arange(c0, min(Sq, c0 + Q_CHUNK), device=q.device)
            sl = slice(c0, c0 + len(qi))
            s = _scores(q[:, :, sl], ke, scale, qi, causal, offset)
            prob = torch.exp(s - lse[:, :, sl].unsqueeze(-1))
            keep = dropout_keep_mask(seed, B, Hq, qi, Sk, p, head_offset) / (1.0 - p)
            doc = do[:, :, sl].float()
            dv += torch.matmul((prob * keep).transpose(-1, -2), doc)
            dp = torch.matmul(doc, ve.transpose(-1, -2)) * keep
            ds = prob * (dp - delta[:, :, sl].unsqueeze(-1)) * scale
            dq[:, :, sl] = torch.matmul(ds, ke).to(q.dtype)
            dk += torch.matmul(ds.transpose(-1, -2), q[:, :, sl].float())
        if Hkv != Hq:
            g = Hq // Hkv
            dk = dk.view(B, Hkv, g, Sk, D).sum(2)
            dv = dv.view(B, Hkv, g, Sk, D).sum(2)
        return dq, dk.to(k.dtype), dv.to(v.dtype), None, None, None, None, None


def attention_with_dropout(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, dropout_p: float, causal: bool = True,
                           softmax_scale: Optional[float] = None, seed: Optional[int] = None,
                           head_offset: int = 0) -> torch.Tensor:
    """bhsd attention with dropout on the probabilities (inverted scaling 1 / (1 - p))."""
    if not 0.0 <= dropout_p < 1.0:
        raise ValueError(f"dropout_p must be in [0, 1), got {dropout_p}")
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if seed is None:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=None).item())
    from ._ext import use_native

    if use_native(q, k, v) and q.shape[-1] in (64, 128) and q.dtype == torch.bfloat16:
        from .flash_attn import FlashAttnFunc

        qs, ks, vs = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)   # bhsd -> bshd views
        if qs.stride(-1) != 1 or any(st % 8 for st in qs.stride()[:3]):
            qs = qs.contiguous()
        if ks.stride(-1) != 1 or any(st % 8 for st in ks.stride()[:3]):
            ks = ks.contiguous()
        if vs.stride(-1) != 1 or any(st % 8 for st in vs.stride()[:3]):
            vs = vs.contiguous()
        o = FlashAttnFunc.apply(qs, ks, vs, causal, scale, ks.shape[1] - qs.shape[1],
                                (float(dropout_p), int(seed), int(head_offset)))
        return o.transpose(1, 2)
    return DropoutAttentionFunc.apply(q, k, v, causal, scale, float(dropout_p), int(seed), int(head_offset))
