"""Flash attention (fwd + bwd) on the CDNA4 kernels in csrc/flash_attn_{fwd,bwd}.hip.

API parity with the reference `nki_flash_attn_func` (src/neuronx_distributed/kernels/flash_attn.py:151-191)
but without its restrictions: any sequence length (the reference needs multiples of 2048), GQA
without `repeat_kv`, arbitrary strides (reads Q/K/V straight out of a fused QKV buffer), D = 64/128.

Also provides `rope_attention`, the training attention core used by the Llama model: RoPE applied
in place to the fused [S, B, (Hq+2Hkv)*D] QKV projection output, flash attention over strided
views of it, and a backward that writes dQ/dK/dV straight back into one fused dQKV buffer and
un-rotates it in place — no transposes, no repeat_kv, no separate q/k/v copies.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from ._ext import ext, use_native
from .rope import rope_inplace_


def attention_reference(q, k, v, causal: bool = True, softmax_scale: Optional[float] = None, causal_offset: Optional[int] = None):
    """Plain fp32 reference. q: [B, Sq, Hq, D], k/v: [B, Sk, Hkv, D] -> (o [B, Sq, Hq, D], lse [B, Hq, Sq])."""
    B, Sq, Hq, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    g = Hq // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        off = Sk - Sq if causal_offset is None else causal_offset
        qi = torch.arange(Sq, device=q.device)[:, None]
        ki = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(ki > qi + off, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return o, lse


_NO_DROPOUT = (0.0, 0, 0)


def _fwd(q, k, v, causal, scale, causal_offset, out=None, dropout=_NO_DROPOUT):
    B, Sq, Hq, D = q.shape
    o = out if out is not None else torch.empty(q.shape, dtype=q.dtype, device=q.device)
    lse = torch.empty((B, Hq, Sq), dtype=torch.float32, device=q.device)
    ext().flash_attn_fwd(q, k, v, o, lse, float(scale), bool(causal), int(causal_offset), *dropout)
    return o, lse


class FlashAttnFunc(torch.autograd.Function):
    """dropout = (p, seed, head_offset): dropout on the probabilities inside both kernels (keep mask
    hashed from (seed, batch, global head, query, key) -- ops/attention_dropout.dropout_keep_mask --
    so nothing is stored and the backward regenerates it)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, softmax_scale, causal_offset, dropout=_NO_DROPOUT):
        o, lse = _fwd(q, k, v, causal, softmax_scale, causal_offset, dropout=dropout)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale, ctx.off, ctx.dropout = causal, softmax_scale, causal_offset, dropout
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do if do.stride(-1) == 1 else do.contiguous()
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        ext().flash_attn_bwd(q, k, v, o, do, lse, dq, dk, dv, float(ctx.scale), bool(ctx.causal), int(ctx.off),
                             *ctx.dropout)
        return dq, dk, dv, None, None, None, None


def flash_attn_func(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    softmax_scale: Optional[float] = None, causal_offset: Optional[int] = None,
                    dropout_p: float = 0.0, seed: Optional[int] = None, head_offset: int = 0) -> torch.Tensor:
    """q: [B, Sq, Hq, D], k/v: [B, Sk, Hkv, D] (bf16, unit stride on D) -> o [B, Sq, Hq, D].
    dropout_p > 0: dropout on the attention probabilities (inverted scaling), mask from `seed`
    with local head h drawn as global head head_offset + h (tensor-parallel ranks)."""
    D = q.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    off = (k.shape[1] - q.shape[1]) if causal_offset is None else causal_offset
    if dropout_p:
        from .attention_dropout import attention_with_dropout

        if causal_offset is not None and causal_offset != k.shape[1] - q.shape[1]:
            raise ValueError("dropout attention supports the bottom-right causal alignment only")
        o = attention_with_dropout(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), dropout_p, causal=causal,
                                   softmax_scale=scale, seed=seed, head_offset=head_offset)
        return o.transpose(1, 2)
    if use_native(q, k, v):
        return FlashAttnFunc.apply(q, k, v, causal, scale, off)
    o, _ = attention_reference(q, k, v, causal, scale, off)
    return o.to(q.dtype)


def flash_attn_fwd_lse(q, k, v, causal=True, softmax_scale=None, causal_offset=None, out=None):
    """Forward only, returning (o, lse) — used by inference prefill and ring/segment merges."""
    D = q.shape[-1]
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    off = (k.shape[1] - q.shape[1]) if causal_offset is None else causal_offset
    if use_native(q, k, v):
        return _fwd(q, k, v, causal, scale, off, out=out)
    o, lse = attention_reference(q, k, v, causal, scale, off)
    o = o.to(q.dtype)
    if out is not None:
        out.copy_(o)
        o = out
    return o, lse


# --------------------------------------------------------------------------------------------
# fused RoPE + attention core over a [S, B, (Hq + 2Hkv) * D] QKV projection output
# --------------------------------------------------------------------------------------------


def _views(qkv: torch.Tensor, nq: int, nkv: int, D: int):
    """[S, B, W] -> q [B, S, nq, D], k/v [B, S, nkv, D] strided views (no copies)."""
    S, B, W = qkv.shape
    st = qkv.stride()
    q = qkv.as_strided((B, S, nq, D), (st[1], st[0], D, 1), qkv.storage_offset())
    k = qkv.as_strided((B, S, nkv, D), (st[1], st[0], D, 1), qkv.storage_offset() + nq * D)
    v = qkv.as_strided((B, S, nkv, D), (st[1], st[0], D, 1), qkv.storage_offset() + (nq + nkv) * D)
    return q, k, v


class RopeAttentionFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos_t, sin_t, nq, nkv, D, causal, scale, position_offset):
        S, B, W = qkv.shape
        flat = qkv.view(S * B, W)
        # rotate q and k heads (contiguous columns [0, (nq+nkv)*D)) in place; position = row // B
        rope_inplace_(flat, 0, nq + nkv, D, cos_t, sin_t, None, pos_div=B, pos_mod=cos_t.shape[0]) if position_offset == 0 else \
            rope_inplace_(flat, 0, nq + nkv, D, cos_t, sin_t,
                          (torch.arange(S * B, device=qkv.device) // B + position_offset))
        ctx.mark_dirty(qkv)
        # the rotated qkv output is never differentiated through: do not let autograd zero-fill
        # a [S, B, W] gradient for it every layer
        ctx.set_materialize_grads(False)
        q, k, v = _views(qkv, nq, nkv, D)
        o = torch.empty((S, B, nq * D), dtype=qkv.dtype, device=qkv.device)
        o_v = o.view(S, B, nq, D).permute(1, 0, 2, 3)
        _, lse = _fwd(q, k, v, causal, scale, 0, out=o_v)
        ctx.save_for_backward(qkv, o, lse, cos_t, sin_t)
        ctx.meta = (nq, nkv, D, causal, scale, position_offset)
        return qkv, o

    @staticmethod
    def backward(ctx, _dqkv_unused, do):
        qkv, o, lse, cos_t, sin_t = ctx.saved_tensors
        nq, nkv, D, causal, scale, position_offset = ctx.meta
        S, B, W = qkv.shape
        do = do.contiguous()
        q, k, v = _views(qkv, nq, nkv, D)
        o_v = o.view(S, B, nq, D).permute(1, 0, 2, 3)
        do_v = do.view(S, B, nq, D).permute(1, 0, 2, 3)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _views(dqkv, nq, nkv, D)
        ext().flash_attn_bwd(q, k, v, o_v, do_v, lse, dq, dk, dv, float(scale), bool(causal), 0)
        flat = dqkv.view(S * B, W)
        if position_offset == 0:
            rope_inplace_(flat, 0, nq + nkv, D, cos_t, sin_t, None, pos_div=B, pos_mod=cos_t.shape[0], sign=-1.0)
        else:
            rope_inplace_(flat, 0, nq + nkv, D, cos_t, sin_t,
                          (torch.arange(S * B, device=qkv.device) // B + position_offset), sign=-1.0)
        return dqkv, None, None, None, None, None, None, None, None


def rope_attention(qkv: torch.Tensor, cos_t: torch.Tensor, sin_t: torch.Tensor, nq: int, nkv: int, head_dim: int,
                   causal: bool = True, softmax_scale: Optional[float] = None, position_offset: int = 0) -> torch.Tensor:
    """Attention core of a Llama block.

    qkv: [S, B, (nq + 2 nkv) * D] output of the (column-parallel) QKV projection, q heads first,
    then k heads, then v heads.  Returns o: [S, B, nq * D].  `qkv` is rotated in place.
    """
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(head_dim)
    if use_native(qkv):
        assert qkv.is_contiguous(), "fused qkv must be contiguous"
        _, o = RopeAttentionFunc.apply(qkv, cos_t, sin_t, nq, nkv, head_dim, causal, scale, position_offset)
        return o
    # reference path (CPU): out-of-place, differentiable through plain torch ops
    S, B, W = qkv.shape
    x = qkv.view(S, B, nq + 2 * nkv, head_dim)
    pos = torch.arange(S, device=qkv.device) + position_offset
    c = cos_t.to(qkv.device)[pos][:, None, None, :].float()
    s = sin_t.to(qkv.device)[pos][:, None, None, :].float()

    def rot(t):
        tf = t.float()
        t1, t2 = tf[..., : head_dim // 2], tf[..., head_dim // 2:]
        return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1).to(t.dtype)

    q = rot(x[:, :, :nq]).permute(1, 0, 2, 3)
    k = rot(x[:, :, nq:nq + nkv]).permute(1, 0, 2, 3)
    v = x[:, :, nq + nkv:].permute(1, 0, 2, 3)
    g = nq // nkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(g, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(g, dim=1)
    sc = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=qkv.device).triu(1)
        sc = sc.masked_fill(mask, float("-inf"))
    p = torch.softmax(sc, dim=-1)
    o = torch.matmul(p, vf)  # [B, H, S, D]
    return o.permute(2, 0, 1, 3).reshape(S, B, nq * head_dim).to(qkv.dtype)
