"""Training flash-attention entry point with the reference's API
(src/neuronx_distributed/kernels/flash_attn.py:151-191 `nki_flash_attn_func`).

The reference takes q/k/v as [B, H, D, S] / [B, H, S, D] NKI layouts with S a multiple of 2048 and
runs the NKI kernel; here the CDNA4 HIP kernels (csrc/flash_attn_fwd.hip / flash_attn_bwd.hip) are
called with no sequence-length restriction and native GQA (fewer K/V heads than Q heads).  Layout
arguments are accepted in either form:
* `layout="bhsd"` (default, like torch SDPA): q [B, Hq, S, D], k/v [B, Hkv, S, D];
* `layout="bshd"`: q [B, S, Hq, D] (the framework's internal layout, zero-copy);
* `layout="nki"`: q [B, H, D, S], k [B, H, D, S], v [B, H, S, D] (reference NKI shapes).
"""

from __future__ import annotations

from typing import Optional

import torch

from ..ops.attention_dropout import attention_with_dropout
from ..ops.flash_attn import flash_attn_func as _fa


def _dropout_attn(q, k, v, causal, softmax_scale, layout, dropout_p, seed):
    """dropout_p > 0: dropout inside the CDNA4 flash kernels on the GPU (host path: the chunked flash
    decomposition, ops/attention_dropout.py) with a hashed keep mask; heads are numbered globally
    across tensor-parallel ranks so the mask matches the unsharded model."""
    from ..parallel_layers import parallel_state as ps

    if layout == "bshd":
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    elif layout == "nki":
        q, k, v = q.transpose(2, 3), k.transpose(2, 3), v
    elif layout != "bhsd":
        raise ValueError(f"unknown layout {layout}")
    off = ps.get_tensor_model_parallel_rank() * q.shape[1] if ps.model_parallel_is_initialized() else 0
    o = attention_with_dropout(q, k, v, dropout_p, causal=causal, softmax_scale=softmax_scale, seed=seed,
                               head_offset=off)
    return o.transpose(1, 2) if layout == "bshd" else o


def flash_attn_func(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    softmax_scale: Optional[float] = None, layout: str = "bhsd", dropout_p: float = 0.0,
                    seed: Optional[int] = None) -> torch.Tensor:
    if dropout_p:
        return _dropout_attn(q, k, v, causal, softmax_scale, layout, dropout_p, seed)
    if layout == "bshd":
        return _fa(q, k, v, causal=causal, softmax_scale=softmax_scale)
    if layout == "bhsd":
        o = _fa(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=causal, softmax_scale=softmax_scale)
        return o.transpose(1, 2)
    if layout == "nki":
        o = _fa(q.permute(0, 3, 1, 2), k.permute(0, 3, 1, 2), v.transpose(1, 2), causal=causal,
                softmax_scale=softmax_scale)
        return o.transpose(1, 2)  # [B, H, S, D]
    raise ValueError(f"unknown layout {layout}")


def nki_flash_attn_func(query, key, value, droupout_p: float = 0.0, softmax_scale: Optional[float] = None,
                        causal: bool = True, seed: Optional[int] = None):
    """Reference-named alias: query/key [B, H, D, S], value [B, H, S, D] -> [B, H, S, D]."""
    return flash_attn_func(query, key, value, causal=causal, softmax_scale=softmax_scale, layout="nki",
                           dropout_p=droupout_p, seed=seed)
