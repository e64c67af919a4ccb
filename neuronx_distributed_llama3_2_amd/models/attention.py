"""Attention core shared by the non-Llama example models (GPT-NeoX, BERT).

Dispatch (explicit, not a silent fallback): the CDNA4 flash-attention kernels cover head_dim 64 /
128 with no key-padding mask on the GPU; other head sizes (GPT-NeoX-20B has 96) or padded BERT
batches use PyTorch SDPA; on the CPU the fp32 reference path of ops.flash_attn_func runs.
"""

from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool,
              key_padding_mask: Optional[torch.Tensor] = None, dropout_p: float = 0.0) -> torch.Tensor:
    """q/k/v [B, S, H, D] -> o [B, S, H, D]; key_padding_mask [B, S] (1 = keep); dropout_p on the
    attention probabilities (the flash kernels' in-kernel dropout; heads numbered globally over
    the tensor-parallel ranks, seed from the host RNG, which every rank seeds alike, so TP ranks draw one mask)."""
    D = q.shape[-1]
    has_pad = key_padding_mask is not None and not bool(key_padding_mask.all())
    if not has_pad and (not q.is_cuda or D in (64, 128)):
        if dropout_p:
            from ..parallel_layers import parallel_state as ps

            off = ps.get_tensor_model_parallel_rank() * q.shape[2] if ps.model_parallel_is_initialized() else 0
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
            return ops.flash_attn_func(q, k, v, causal=causal, dropout_p=dropout_p, seed=seed, head_offset=off)
        return ops.flash_attn_func(q, k, v, causal=causal)
    mask = None
    if has_pad:
        mask = key_padding_mask[:, None, None, :].bool()
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), attn_mask=mask,
                                       is_causal=causal and mask is None, scale=1.0 / math.sqrt(D),
                                       dropout_p=dropout_p)
    return o.transpose(1, 2)
