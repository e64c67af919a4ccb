"""Sequence-parallel layout and communication/GEMM overlap for TP+SP linear layers.

Chunk-interleaved SP layout
---------------------------
Megatron SP gives TP rank r the contiguous rows [r*S/tp, (r+1)*S/tp) of the sequence.  Here the
sequence is first cut into `c` chunks (NXD_SP_CHUNKS; default per TP degree, see _DEFAULT_CHUNKS) and EACH chunk is split over the
TP ranks: the local shard of rank r is [chunk 0 part r | chunk 1 part r | ...].  Everything outside
the TP regions (residual stream, RMSNorm, dropout) is row-wise, so the row order of a local shard is
irrelevant to the math — but with this layout the all-gather of chunk j returns the CONTIGUOUS
rows [j*S/c, (j+1)*S/c) of the full sequence, and the reduce-scatter of those full rows is exactly
each rank's part j.  That makes the collectives chunkable without any re-ordering copies:

* column-parallel forward (and row-parallel backward): the c all-gathers are issued up front on
  RCCL's stream and the GEMM of chunk j waits only for gather j (the GEMM of chunk j overlaps the
  gathers of chunks j+1..);
* row-parallel forward (and column-parallel backward): the GEMM of chunk j is followed by its
  asynchronous reduce-scatter, which overlaps the GEMM of chunk j+1 (and, in backward, the
  weight-gradient GEMM).

Over xGMI (7 point-to-point links per MI355X) a TP=8 ring moves ~64 MiB per SP collective per
layer at S=8192 — as much time as the GEMMs themselves, so hiding it is what makes TP=8 scale.
c = 1 reproduces the reference layout (parallel_layers/mappings.py:237-308 of the reference).
"""

from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import gemm as _gemm
from ..parallel import comm
from .parallel_state import get_tensor_model_parallel_group

_SP_CHUNKS = int(os.environ["NXD_SP_CHUNKS"]) if "NXD_SP_CHUNKS" in os.environ else None

# Default chunk count per TP degree, for the micro-batch bench.py runs each degree at (MBS_BY_TP:
# 2 sequences at TP2, 4 at TP4 / TP8).  Chunking trades exposed communication (the first gather /
# last reduce-scatter of each op, ~T/c) for smaller GEMMs.  GEMM side per layer (fwd + dgrad,
# Llama-3-8B, S=8192, tools/bench_sp_chunks.py, profiles/r3_sp_chunks_gemm_mbs.jsonl), c = 1/2/4/8:
# TP8 mbs 4: 2.67 / 2.68 / 2.80 / 3.20 ms; TP4 mbs 4: 4.90 / 4.97 / 5.09 / 5.32; TP2 mbs 2: 4.81 /
# 4.84 / 4.97 / 5.83.  Going from c=2 to c=4 costs 0.12-0.13 ms per layer and saves ~T/4 on each
# of the ~3 exposed collective ends per layer, T = one 32k-token (256 MiB) SP all-gather or
# reduce-scatter: a win for any T above ~0.17 ms, i.e. below ~1.3 TB/s of ring bandwidth -- every
# plausible xGMI figure.  c=8 costs 0.5 ms per layer at TP8 and is not worth it.  (At micro-batch 1
# the GEMMs are 4x smaller and chunking costs relatively more: profiles/r1_sp_chunks_gemm.jsonl.)
# Round 4, with the two staggered SP halves on the emulated ranks (profiles/r4_emulate_sp_chunks_halves.jsonl):
# TP8 at 400 GB/s c = 1 / 2 / 4 / 8: 552 / 511 / 517 / 573 ms per step; TP4 at 200 GB/s c = 2 / 4 / 8: 939 / 898 /
# 923; TP2 at 70 GB/s: 1,843 / 1,753 / 1,830.
_DEFAULT_CHUNKS = {2: 4, 4: 4, 8: 2}


def set_sequence_parallel_chunks(c: Optional[int]) -> None:
    """Override the chunk count for every TP degree (None restores the per-degree defaults)."""
    global _SP_CHUNKS
    _SP_CHUNKS = None if c is None else max(1, int(c))


def get_sequence_parallel_chunks(tp: int = 8) -> int:
    return _SP_CHUNKS if _SP_CHUNKS is not None else _DEFAULT_CHUNKS.get(tp, 2)


def _chunks(local_rows: int, tp: int = 8) -> int:
    c = get_sequence_parallel_chunks(tp)
    while c > 1 and local_rows % c:
        c -= 1
    return c


def _ws(group) -> int:
    return dist.get_world_size(group=group)


# ------------------------------------------------------------------------------- plain collectives
def gather_start(x: torch.Tensor, group=None) -> Tuple[torch.Tensor, List, int]:
    """Launch the chunked all-gather of a local SP shard [S/tp, ...] -> full [S, ...]; returns
    (full buffer, per-chunk handles, c)."""
    group = group if group is not None else get_tensor_model_parallel_group()
    tp = _ws(group)
    x = x.contiguous()
    Sl = x.shape[0]
    c = _chunks(Sl, tp)
    full = torch.empty((tp * Sl,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    fv = full.view((c, tp * (Sl // c)) + tuple(x.shape[1:]))
    xv = x.view((c, Sl // c) + tuple(x.shape[1:]))
    hs = [comm.all_gather_into_tensor(fv[j], xv[j], group=group, async_op=True) for j in range(c)]
    return full, hs, c


def sp_gather(x: torch.Tensor, group=None) -> torch.Tensor:
    group = group if group is not None else get_tensor_model_parallel_group()
    if _ws(group) == 1:
        return x
    full, hs, _ = gather_start(x, group)
    for h in hs:
        h.wait()
    return full


def sp_reduce_scatter(x: torch.Tensor, group=None) -> torch.Tensor:
    """Full [S, ...] (partial sums) -> this rank's SP shard [S/tp, ...] in the chunked layout."""
    group = group if group is not None else get_tensor_model_parallel_group()
    tp = _ws(group)
    if tp == 1:
        return x
    x = x.contiguous()
    S = x.shape[0]
    assert S % tp == 0, f"sequence {S} not divisible by TP {tp}"
    Sl = S // tp
    c = _chunks(Sl, tp)
    out = torch.empty((Sl,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    ov = out.view((c, Sl // c) + tuple(x.shape[1:]))
    xv = x.view((c, S // c) + tuple(x.shape[1:]))
    hs = [comm.reduce_scatter_tensor(ov[j], xv[j], group=group, async_op=True) for j in range(c)]
    for h in hs:
        h.wait()
    return out


def sp_split(x: torch.Tensor, group=None) -> torch.Tensor:
    """Full [S, ...] (replicated) -> this rank's SP shard in the chunked layout."""
    group = group if group is not None else get_tensor_model_parallel_group()
    tp = _ws(group)
    if tp == 1:
        return x
    r = dist.get_rank(group=group)
    S = x.shape[0]
    Sl = S // tp
    c = _chunks(Sl, tp)
    return x.reshape((c, tp, Sl // c) + tuple(x.shape[1:]))[:, r].reshape((Sl,) + tuple(x.shape[1:])).contiguous()


# ------------------------------------------------------------------------------- fused GEMM + comm
def gather_linear(x_local: torch.Tensor, weight: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Column-parallel SP forward: (all-gather(x_local) @ weight^T, gathered x), chunk-pipelined."""
    group = group if group is not None else get_tensor_model_parallel_group()
    if _ws(group) == 1:
        return _gemm.linear(x_local, weight), x_local
    full, hs, c = gather_start(x_local, group)
    out = torch.empty(tuple(full.shape[:-1]) + (weight.shape[0],), dtype=full.dtype, device=full.device)
    fv = full.view((c, full.shape[0] // c) + tuple(full.shape[1:]))
    ov = out.view((c, out.shape[0] // c) + tuple(out.shape[1:]))
    for j in range(c):
        hs[j].wait()
        _gemm.linear(fv[j], weight, out=ov[j])
    return out, full


def gather_matmul(g_local: torch.Tensor, weight: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-parallel SP backward: (all-gather(g_local) @ weight, gathered g), chunk-pipelined."""
    group = group if group is not None else get_tensor_model_parallel_group()
    if _ws(group) == 1:
        return _gemm.dgrad(g_local, weight), g_local
    full, hs, c = gather_start(g_local, group)
    out = torch.empty(tuple(full.shape[:-1]) + (weight.shape[1],), dtype=full.dtype, device=full.device)
    fv = full.view((c, full.shape[0] // c) + tuple(full.shape[1:]))
    ov = out.view((c, out.shape[0] // c) + tuple(out.shape[1:]))
    for j in range(c):
        hs[j].wait()
        _gemm.dgrad(fv[j], weight, out=ov[j])
    return out, full


def _gemm_reduce_scatter(fn, x_full: torch.Tensor, n_out: int, group) -> Tuple[torch.Tensor, List]:
    tp = _ws(group)
    S = x_full.shape[0]
    Sl = S // tp
    c = _chunks(Sl, tp)
    out_full = torch.empty(tuple(x_full.shape[:-1]) + (n_out,), dtype=x_full.dtype, device=x_full.device)
    local = torch.empty((Sl,) + tuple(out_full.shape[1:]), dtype=x_full.dtype, device=x_full.device)
    xv = x_full.view((c, S // c) + tuple(x_full.shape[1:]))
    fv = out_full.view((c, S // c) + tuple(out_full.shape[1:]))
    lv = local.view((c, Sl // c) + tuple(out_full.shape[1:]))
    hs = []
    for j in range(c):
        fn(xv[j], fv[j])
        hs.append(comm.reduce_scatter_tensor(lv[j], fv[j], group=group, async_op=True))
    return local, hs


def linear_reduce_scatter_start(x_full: torch.Tensor, weight: torch.Tensor, group=None):
    """Row-parallel SP forward: reduce_scatter(x_full @ weight^T) with each chunk's reduce-scatter
    overlapping the next chunk's GEMM; returns (local shard, handles) — wait before use."""
    group = group if group is not None else get_tensor_model_parallel_group()
    x_full = x_full.contiguous()
    return _gemm_reduce_scatter(lambda a, o: _gemm.linear(a, weight, out=o), x_full, weight.shape[0], group)


def matmul_reduce_scatter_start(g_full: torch.Tensor, weight: torch.Tensor, group=None):
    """Column-parallel SP backward: reduce_scatter(g_full @ weight), chunk-pipelined."""
    group = group if group is not None else get_tensor_model_parallel_group()
    g_full = g_full.contiguous()
    return _gemm_reduce_scatter(lambda a, o: _gemm.dgrad(a, weight, out=o), g_full, weight.shape[1], group)
