"""Decode-path kernels (csrc/inference.hip): flash-decoding attention over a persistent KV cache,
in-place KV-cache writes, argmax and top-k multinomial sampling.

Cache layout: [batch, kv_heads, max_len, head_dim] (the reference's KV-cache parameter layout,
examples/inference/modules/model_base.py:114-125); valid length per sequence comes from a device
int32 tensor, so a decode step has static shapes and can be captured in a hipGraph.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from ._ext import ext, use_native

CHUNK = 128


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, seq_len: torch.Tensor,
                     cache_idx: Optional[torch.Tensor] = None, softmax_scale: Optional[float] = None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q: [B, T, Hq, D] new-token queries; keys [0, seq_len[b]) are valid for the LAST token, and
    token t sees keys < seq_len[b] - (T - 1 - t).  Returns [B, T, Hq, D]."""
    B, T, Hq, D = q.shape
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    if out is None:
        out = torch.empty((B, T, Hq, D), dtype=q.dtype, device=q.device)
    if use_native(q, k_cache):
        nsplit = max(1, (k_cache.shape[2] + CHUNK - 1) // CHUNK)
        ext().decode_attn(q, k_cache, v_cache, cache_idx.to(torch.int32) if cache_idx is not None else None,
                          seq_len.to(torch.int32), out, float(scale), nsplit)
        return out
    Hkv = k_cache.shape[1]
    g = Hq // Hkv
    for b in range(B):
        cb = int(cache_idx[b]) if cache_idx is not None else b
        L = int(seq_len[b])
        kk = k_cache[cb, :, :L].float().repeat_interleave(g, 0)  # [Hq, L, D]
        vv = v_cache[cb, :, :L].float().repeat_interleave(g, 0)
        qq = q[b].float().permute(1, 0, 2)  # [Hq, T, D]
        s = torch.matmul(qq, kk.transpose(-1, -2)) * scale
        ti = torch.arange(T, device=q.device)[:, None]
        ki = torch.arange(L, device=q.device)[None, :]
        s = s.masked_fill(ki >= (L - (T - 1 - ti)), float("-inf"))
        p = torch.softmax(s, -1)
        out[b] = torch.matmul(p, vv).permute(1, 0, 2).to(out.dtype)
    return out


def kv_cache_write(k_new: torch.Tensor, v_new: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                   positions: torch.Tensor, cache_idx: Optional[torch.Tensor] = None) -> None:
    """k_new/v_new: [B, T, Hkv, D]; writes cache[cache_idx[b], :, positions[b] + t] in place."""
    if use_native(k_new, k_cache):
        ext().kv_cache_write(k_new, v_new, k_cache, v_cache,
                             cache_idx.to(torch.int32) if cache_idx is not None else None, positions.to(torch.int32))
        return
    B, T = k_new.shape[:2]
    for b in range(B):
        cb = int(cache_idx[b]) if cache_idx is not None else b
        p0 = int(positions[b])
        n = max(0, min(T, k_cache.shape[2] - p0))
        k_cache[cb, :, p0:p0 + n] = k_new[b, :n].transpose(0, 1).to(k_cache.dtype)
        v_cache[cb, :, p0:p0 + n] = v_new[b, :n].transpose(0, 1).to(v_cache.dtype)


def argmax_rows(x: torch.Tensor) -> torch.Tensor:
    if use_native(x):
        out = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
        ext().argmax_rows(x if x.stride(-1) == 1 else x.contiguous(), out)
        return out
    return torch.argmax(x, dim=-1)


def greedy_advance_(logits: torch.Tensor, slot: torch.Tensor, out: torch.Tensor, step: torch.Tensor,
                    tokens: torch.Tensor, positions: torch.Tensor, cache_len: torch.Tensor) -> None:
    """Greedy decode tail in two launches (multi-workgroup argmax + state feed-back):
    t = argmax(logits, -1); out[:, step] = t; tokens = t; positions += 1; cache_len += 1; step += 1.
    `slot` is int64 [B] scratch that must be zero on entry (the kernel leaves it zeroed)."""
    if use_native(logits):
        ext().greedy_advance(logits if logits.stride(-1) == 1 else logits.contiguous(), slot, out, step,
                             tokens.view(-1), positions.view(-1), cache_len.view(-1))
        return
    t = torch.argmax(logits, dim=-1)
    B = logits.shape[0]
    out.scatter_(1, step.view(1, 1).expand(B, 1), t.view(B, 1))
    tokens.copy_(t.view(tokens.shape))
    positions.add_(1)
    cache_len.add_(1)
    step.add_(1)


def topk_sample(x: torch.Tensor, top_k: int, temperature: float = 1.0, uniform: Optional[torch.Tensor] = None,
                return_topk: bool = False):
    """Multinomial sampling among the top-k logits (reference Sampler.multinomial semantics:
    softmax over the sorted top-k, CDF, count entries below a uniform draw)."""
    B = x.shape[0]
    if uniform is None:
        uniform = torch.rand(B, device=x.device, dtype=torch.float32)
    if use_native(x):
        out = torch.empty(B, dtype=torch.int64, device=x.device)
        vals = torch.empty((B, top_k), dtype=torch.float32, device=x.device) if return_topk else None
        idx = torch.empty((B, top_k), dtype=torch.int64, device=x.device) if return_topk else None
        ext().topk_sample(x if x.stride(-1) == 1 else x.contiguous(), int(top_k), float(temperature), uniform.float(), out,
                          vals, idx)
        return (out, vals, idx) if return_topk else out
    v, i = torch.topk(x.float(), top_k, dim=-1)
    p = torch.softmax(v / (temperature if temperature > 0 else 1.0), dim=-1)
    cdf = torch.cumsum(p, -1)
    pick = (cdf < uniform[:, None]).sum(-1).clamp(max=top_k - 1)
    out = i.gather(1, pick[:, None]).squeeze(1)
    return (out, v, i) if return_topk else out
