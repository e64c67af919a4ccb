"""Vocab-parallel embedding lookup on csrc/embedding.hip (mask fused into the gather; backward
scatter-adds with f32 atomics straight into the weight's fp32 main_grad).

Reference: ParallelEmbedding._forward_shard_across_vocab (src/neuronx_distributed/parallel_layers/layers.py:215-238),
which masks with three extra elementwise passes and relies on F.embedding's dense backward.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import ext, use_native


class EmbeddingFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, vocab_start):
        idc = ids.contiguous().to(torch.int64)
        out = torch.empty(tuple(ids.shape) + (weight.shape[1],), dtype=weight.dtype, device=weight.device)
        ext().embedding_fwd(idc, weight, out, int(vocab_start))
        ctx.save_for_backward(idc)
        ctx.weight = weight
        ctx.vocab_start = vocab_start
        return out

    @staticmethod
    def backward(ctx, dout):
        (idc,) = ctx.saved_tensors
        w = ctx.weight
        mg = getattr(w, "main_grad", None)
        dw = mg if mg is not None else torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        if mg is not None:   # atomics, but a tied lm_head's GEMM read-modify-writes the same buffer
            from ..parallel_layers import stream_split

            stream_split.accumulate_begin(w)
        ext().embedding_bwd(idc, dout.contiguous(), dw.view(w.shape), int(ctx.vocab_start))
        if mg is not None:
            stream_split.accumulate_end(w)
        if mg is not None:
            cb = getattr(w, "_nxd_grad_ready", None)
            if cb is not None:
                cb(w)
            return None, None, None
        return None, dw.to(w.dtype), None


def vocab_parallel_embedding(ids: torch.Tensor, weight: torch.Tensor, vocab_start: int = 0) -> torch.Tensor:
    """Rows of `weight` (the [vocab_end - vocab_start, H] shard) for ids inside the shard, 0 elsewhere."""
    if use_native(ids, weight):
        return EmbeddingFunc.apply(ids, weight, vocab_start)
    V = weight.shape[0]
    local = ids - vocab_start
    mask = (local >= 0) & (local < V)
    out = F.embedding(local.clamp(0, V - 1), weight)
    return out * mask.unsqueeze(-1).to(out.dtype)
