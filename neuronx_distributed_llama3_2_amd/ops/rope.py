"""Rotary position embedding: host-side fp32 cos/sin tables + in-place HIP rotation.

Tables follow HF Llama / Llama-3 (`rope_type="llama3"`) frequency scaling, computed once in fp32 on
the host (reference: examples/inference/llama3/neuron_modeling_llama.py:234-298,
examples/training/llama/training_utils.py:224-232).  The device kernel (csrc/rope.hip) reads
them and rotates q/k heads in place inside a fused QKV buffer.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from ._ext import ext, use_native


def llama3_inv_freq(dim: int, base: float = 500000.0, factor: Optional[float] = None, low_freq_factor: float = 1.0,
                    high_freq_factor: float = 4.0, original_max_position_embeddings: int = 8192) -> torch.Tensor:
    inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.int64).double() / dim))
    if factor is None:
        return inv_freq.float()
    low_wl = original_max_position_embeddings / low_freq_factor
    high_wl = original_max_position_embeddings / high_freq_factor
    wavelen = 2 * math.pi / inv_freq
    smooth = (original_max_position_embeddings / wavelen - low_freq_factor) / (high_freq_factor - low_freq_factor)
    scaled = torch.where(wavelen > low_wl, inv_freq / factor, inv_freq)
    mid = (wavelen <= low_wl) & (wavelen >= high_wl)
    scaled = torch.where(mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
    return scaled.float()


def inv_freq_from_config(config, head_dim: int) -> torch.Tensor:
    # transformers >= 5 keeps theta and scaling in `rope_parameters`; older configs use
    # `rope_theta` + `rope_scaling`
    rp = getattr(config, "rope_parameters", None) or {}
    rs = rp if isinstance(rp, dict) and rp else (getattr(config, "rope_scaling", None) or {})
    base = rs.get("rope_theta") if isinstance(rs, dict) else None
    if base is None:
        base = getattr(config, "rope_theta", None)
    base = float(base if base is not None else 10000.0)
    rtype = rs.get("rope_type", rs.get("type")) if isinstance(rs, dict) else None
    if rtype == "llama3":
        return llama3_inv_freq(head_dim, base, float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)),
                               float(rs.get("high_freq_factor", 4.0)),
                               int(rs.get("original_max_position_embeddings", 8192)))
    if rtype == "linear":
        return llama3_inv_freq(head_dim, base) / float(rs["factor"])
    return llama3_inv_freq(head_dim, base)


def rope_tables(inv_freq: torch.Tensor, max_pos: int, device=None):
    """cos/sin tables [max_pos, D/2] fp32 (the rotate-half convention repeats them on both halves)."""
    pos = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(pos, inv_freq.double())
    return freqs.cos().float().to(device), freqs.sin().float().to(device)


def _rope_ref_(buf2d: torch.Tensor, col0: int, nheads: int, D: int, cos_t, sin_t, pos: torch.Tensor, sign: float):
    T = buf2d.shape[0]
    x = buf2d[:, col0:col0 + nheads * D].reshape(T, nheads, D).float()
    c = cos_t[pos].unsqueeze(1).float()
    s = sin_t[pos].unsqueeze(1).float() * sign
    x1, x2 = x[..., : D // 2], x[..., D // 2:]
    o = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    buf2d[:, col0:col0 + nheads * D] = o.reshape(T, nheads * D).to(buf2d.dtype)


def rope_inplace_(buf2d: torch.Tensor, col0: int, nheads: int, head_dim: int, cos_t: torch.Tensor, sin_t: torch.Tensor,
                  positions: Optional[torch.Tensor] = None, pos_div: int = 1, pos_mod: Optional[int] = None,
                  sign: float = 1.0) -> torch.Tensor:
    """Rotate `nheads` heads starting at column `col0` of each row of `buf2d` ([T, W] view, unit
    column stride) in place.  Position of row t: positions[t] or (t // pos_div) % pos_mod."""
    T, W = buf2d.shape[0], buf2d.stride(0)
    if pos_mod is None:
        pos_mod = cos_t.shape[0]
    if use_native(buf2d):
        assert buf2d.stride(1) == 1
        ext().rope_inplace(buf2d, T, W, col0, nheads, head_dim, cos_t, sin_t,
                           positions.to(torch.int64).contiguous() if positions is not None else None,
                           pos_div, pos_mod, float(sign))
        return buf2d
    if positions is None:
        positions = (torch.arange(T, device=buf2d.device) // pos_div) % pos_mod
    _rope_ref_(buf2d, col0, nheads, head_dim, cos_t.to(buf2d.device), sin_t.to(buf2d.device), positions.long(), sign)
    return buf2d


def apply_rotary_reference(x: torch.Tensor, cos_t: torch.Tensor, sin_t: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
    """Out-of-place fp32 reference for [..., S, H, D] tensors with positions [S] (HF rotate_half)."""
    D = x.shape[-1]
    c = cos_t[positions].unsqueeze(-2).float()
    s = sin_t[positions].unsqueeze(-2).float()
    xf = x.float()
    x1, x2 = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
