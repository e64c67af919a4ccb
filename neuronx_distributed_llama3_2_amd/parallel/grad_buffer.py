"""Flat parameter / gradient buffers with bucketed, backward-overlapped data-parallel reduction.

The MI355X-native replacement of the reference's end-of-step gradient handling
(bucket_allreduce_gradients: src/neuronx_distributed/parallel_layers/grads.py:243-310, and the
torch_xla ZeroRedundancyOptimizer internals: src/neuronx_distributed/optimizer/zero_redundancy_optimizer.py):

* Parameters of one kind are re-homed into ONE contiguous bf16 buffer and get an fp32 `main_grad`
  view into ONE contiguous fp32 gradient buffer.  Linear / norm / embedding kernels accumulate
  weight gradients straight into `main_grad` (no `.grad` tensors, no per-step zeroing of
  thousands of tensors: one memset per buffer).
* The gradient buffer is cut into buckets (default 128 MiB of fp32 = `NXD_DP_BUCKET_MB`) in
  reverse registration order, i.e. the order backward produces them.  When every parameter of a
  bucket has reported its gradient (the `_nxd_grad_ready` hook fired by the autograd functions),
  the bucket's reduce-scatter (ZeRO-1) or all-reduce is launched asynchronously on RCCL's stream,
  so DP communication overlaps the rest of backward.  Buckets are padded to a multiple of
  `dp * 16` elements so each rank's slice stays 64-byte aligned for the vectorised kernels.
* Parameters used more than once per step (tied embeddings) delay their bucket to the final
  synchronisation so a partial gradient is never sent.
* Buffers are keyed by (param group, kind): kind separates TP-sharded parameters from
  TP-replicated ones (counted once in the grad norm) and, among the latter, sequence-parallel
  ones (norm weights / row biases whose grads are summed over TP in ONE coalesced all-reduce).
"""

from __future__ import annotations

import os
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import comm

KIND_SHARDED = "tp_sharded"
KIND_DUP_SP = "tp_dup_sp"
KIND_DUP = "tp_dup"


def param_kind(p: torch.nn.Parameter, sp_reduce: bool = True) -> str:
    if getattr(p, "tensor_model_parallel", False) or getattr(p, "expert_model_parallel", False):
        return KIND_SHARDED
    if sp_reduce and getattr(p, "sequence_parallel_enabled", False):
        return KIND_DUP_SP
    return KIND_DUP


def _bucket_elems() -> int:
    return int(float(os.environ.get("NXD_DP_BUCKET_MB", "128")) * 1024 * 1024 // 4)


def plan_flat_layout(numels: Sequence[int], dp: int, cap: int, align: int = 16):
    """Offsets of tensors (in the given order) in a flat buffer cut into buckets of ~`cap`
    elements, each padded to a multiple of `align * dp` so every DP rank's slice stays aligned.
    Returns (offsets, [(bucket_start, bucket_end, first_idx, end_idx)], total_numel).  Pure
    function: the ZeRO checkpoint converter re-plans layouts for other DP sizes with it."""
    unit = align * dp
    offsets, spans = [], []
    pos, bstart, first = 0, 0, 0
    for i, n in enumerate(numels):
        offsets.append(pos)
        pos += (n + align - 1) // align * align
        if pos - bstart >= cap:
            end = (pos + unit - 1) // unit * unit
            spans.append((bstart, end, first, i + 1))
            pos, bstart, first = end, end, i + 1
    if first < len(numels):
        end = (pos + unit - 1) // unit * unit
        spans.append((bstart, end, first, len(numels)))
        pos = end
    return offsets, spans, pos


class _Bucket:
    __slots__ = ("start", "end", "params", "pending", "handle", "delayed", "out")

    def __init__(self, start, end, params, delayed):
        self.start, self.end = start, end
        self.params = list(params)
        self.pending = set(id(p) for p in params)
        self.handle = None
        self.delayed = delayed
        self.out = None


class FlatBuffer:
    """One flat bf16 parameter buffer + fp32 grad buffer + DP buckets for a list of parameters."""

    ALIGN = 16  # elements

    def __init__(self, params: Sequence[torch.nn.Parameter], dp_group=None, zero1: bool = False,
                 grad_dtype: torch.dtype = torch.float32, shared_ids: Optional[set] = None, name: str = "",
                 avg_world: Optional[int] = None):
        self.params = list(params)
        self.name = name
        self.dp_group = dp_group
        self.dp = dist.get_world_size(group=dp_group) if (dp_group is not None and dist.is_initialized()) else 1
        self.dp_rank = dist.get_rank(group=dp_group) if (dp_group is not None and dist.is_initialized()) else 0
        self.zero1 = zero1 and self.dp > 1
        # gradients are averaged over `avg_world` data-parallel replicas (default: the reduction
        # group).  Expert-parallel buffers reduce over the expert-data-parallel group but average over
        # the whole DP world: every EP rank's tokens reached the expert through the all-to-all
        # (reference NeuronEPZero1Optimizer scales EP grads by 1 / EP after the EDP reduction).
        self.avg_world = avg_world if avg_world is not None else self.dp
        shared_ids = shared_ids or set()
        assert self.params, "empty parameter list"
        dev = self.params[0].device
        pdt = self.params[0].dtype
        assert all(p.dtype == pdt and p.device == dev for p in self.params), "mixed dtype/device in one buffer"
        # ---- layout: reverse registration order (backward order), buckets of ~cap elements
        order = list(reversed(self.params))
        offs, spans, total = plan_flat_layout([p.numel() for p in order], self.dp, _bucket_elems(), self.ALIGN)
        offsets: Dict[int, Tuple[int, int]] = {id(p): (o, p.numel()) for p, o in zip(order, offs)}
        buckets_spec = [(bs, be, order[i0:i1]) for (bs, be, i0, i1) in spans]
        pos = total
        self.numel = pos
        self.param_data = torch.zeros(self.numel, dtype=pdt, device=dev)
        self.grad_data = torch.zeros(self.numel, dtype=grad_dtype, device=dev)
        for p in self.params:
            off, n = offsets[id(p)]
            view = self.param_data[off:off + n].view_as(p)
            view.copy_(p.data)
            p.data = view
            p.main_grad = self.grad_data[off:off + n].view(p.shape)
            p.grad = None
            p._nxd_grad_ready = self._on_grad_ready
            p._nxd_buffer = self
        self.offsets = offsets
        # pipeline-shared parameters (tied across stages) are summed across stages at the end of the
        # step, so their bucket must wait for the final synchronisation too
        self.buckets = [_Bucket(s, e, ps, any(id(q) in shared_ids or getattr(q, "_nxd_pp_shared", False)
                                                  or getattr(q, "_nxd_tied", False) for q in ps))
                        for (s, e, ps) in buckets_spec]
        self._bucket_of = {id(p): b for b in self.buckets for p in b.params}
        # Overlap is ARMED per step: the training loop (or the pipeline runtime) calls set_sync(True)
        # right before the backward of the LAST micro-batch; finish_grad_sync() disarms it.  Unarmed,
        # every bucket is reduced at the optimizer step (always correct under grad accumulation).
        self.sync_enabled = False
        _LIVE_BUFFERS.append(self)
        self.overlap = os.environ.get("NXD_DP_OVERLAP", "1") == "1"
        self._hooks = []
        for p in self.params:  # generic modules that still produce .grad
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._post_accumulate))
        # ZeRO-1 shard of this rank: slice [r*len/dp, (r+1)*len/dp) of every bucket
        self.shard_numel = sum((b.end - b.start) // self.dp for b in self.buckets) if self.zero1 else self.numel

    # ---------------------------------------------------------------- grad readiness / comm
    def _post_accumulate(self, p):
        if p.grad is not None:
            from ..parallel_layers import stream_split   # (lazy: parallel_layers imports this module)

            stream_split.accumulate_begin(p)
            p.main_grad.add_(p.grad.float() if p.main_grad.dtype == torch.float32 else p.grad)
            stream_split.accumulate_end(p)
            p.grad = None
        self._on_grad_ready(p)

    def _on_grad_ready(self, p):
        if not (self.sync_enabled and self.overlap) or self.dp == 1:
            return
        b = self._bucket_of.get(id(p))
        if b is None or b.delayed:
            return
        b.pending.discard(id(p))
        if not b.pending and b.handle is None:
            self._launch(b)

    def _launch(self, b: _Bucket):
        g = self.grad_data[b.start:b.end]
        if self.zero1:
            n = (b.end - b.start) // self.dp
            b.out = self.grad_data[b.start + self.dp_rank * n: b.start + (self.dp_rank + 1) * n]
            b.handle = comm.reduce_scatter_tensor(b.out, g, group=self.dp_group, async_op=True)
        else:
            b.handle = comm.all_reduce(g, group=self.dp_group, async_op=True)

    def finish_grad_sync(self, average: bool = True) -> None:
        """Launch any bucket not yet launched, wait for all, average over DP."""
        self.sync_enabled = False
        if self.dp == 1:
            if average and self.avg_world > 1:
                self.grad_data.div_(self.avg_world)
            return
        for b in self.buckets:
            if b.handle is None:
                self._launch(b)
        for b in self.buckets:
            b.handle.wait()
            b.handle = None
            b.pending = set(id(p) for p in b.params)
            if average:
                if self.zero1:
                    b.out.div_(self.avg_world)
                else:
                    self.grad_data[b.start:b.end].div_(self.avg_world)
        comm.assert_no_pending_collectives("finish_grad_sync")

    # ---------------------------------------------------------------- ZeRO-1 views
    def shard_ranges(self) -> List[Tuple[int, int]]:
        """(start, end) of this rank's slice in every bucket (whole buffer when not ZeRO-1)."""
        if not self.zero1:
            return [(0, self.numel)]
        out = []
        for b in self.buckets:
            n = (b.end - b.start) // self.dp
            out.append((b.start + self.dp_rank * n, b.start + (self.dp_rank + 1) * n))
        return out

    def gather_params(self) -> None:
        """ZeRO-1: all-gather every bucket's updated bf16 slices (in place).

        Every writer of `param_data` (optimizer steps, state-dict loads, DCP loads) calls this
        afterwards, so this is where the GEMM layer's K-major weight copies are invalidated -- also
        without ZeRO-1: writes through `param_data[s:e]` do not bump the params' own version
        counters (they are views of the flat buffer), so nothing else would notice."""
        from ..ops.gemm import weights_updated

        weights_updated()
        if not self.zero1:
            return
        handles = []
        for b in self.buckets:
            n = (b.end - b.start) // self.dp
            full = self.param_data[b.start:b.end]
            mine = full[self.dp_rank * n:(self.dp_rank + 1) * n]
            handles.append(comm.all_gather_into_tensor(full, mine, group=self.dp_group, async_op=True))
        for h in handles:
            h.wait()
        comm.assert_no_pending_collectives("gather_params")

    def zero_grad(self) -> None:
        self.grad_data.zero_()

    def set_sync(self, enabled: bool) -> None:
        self.sync_enabled = enabled


class _LiveSet:
    def __init__(self):
        import weakref

        self._s = weakref.WeakSet()

    def append(self, b):
        self._s.add(b)

    def __iter__(self):
        return iter(list(self._s))


_LIVE_BUFFERS = _LiveSet()


def arm_grad_sync(enabled: bool = True) -> None:
    """Arm (or disarm) backward-overlapped DP reduction on every live flat buffer."""
    for b in list(_LIVE_BUFFERS):
        b.set_sync(enabled)


def find_shared_params(model: torch.nn.Module) -> set:
    """ids of parameters registered in more than one module (e.g. tied embeddings)."""
    count = defaultdict(int)
    for _, m in model.named_modules(remove_duplicate=False):
        for _, p in m.named_parameters(recurse=False):
            count[id(p)] += 1
    return {k for k, v in count.items() if v > 1}


def tag_shared_params(model: torch.nn.Module) -> set:
    """Mark parameters registered in more than one module (tied embeddings) with `_nxd_tied` so
    every FlatBuffer built over them later -- whatever optimizer front-end builds it and whether or
    not it is handed the model -- defers their bucket's reduction to `finish_grad_sync` (the second
    use's gradient lands after the first use's hook fired)."""
    ids = find_shared_params(model)
    for p in model.parameters():
        if id(p) in ids:
            p._nxd_tied = True
    return ids
