"""Collective primitives used by every parallel component.

On GPUs these are single RCCL calls (torch.distributed NCCL backend = RCCL over xGMI) on flat,
contiguous buffers: `all_gather_into_tensor`, `reduce_scatter_tensor`, `all_reduce`,
`all_to_all_single`, `batch_isend_irecv`.  Async variants return the RCCL work handle so callers
overlap communication with compute (the collective runs on RCCL's internal stream and the
consumer waits on it before use).

Stream-ordering debug mode (`NXD_COMM_DEBUG=1` or `set_comm_debug(True)`): every
async handle is registered with its op, shape and call site until `.wait()`; `assert_no_pending_
collectives(where)` (called by the gradient buffer once backward's reductions are drained) fails
with the list of collectives that were launched but never waited on — the use-before-wait /
leaked-handle class of bugs that otherwise shows up as silent corruption or a hang at exit.

The gloo backend (CPU test harness) lacks the "_base" flat-tensor collectives; the same calls are
emulated there with list all-gathers / all-reduce + slice, so the parallel code paths are the same
on CPU and GPU.

Direct-peer layer (parallel/peer_allreduce.py over csrc/peer_allreduce.hip): the tensor-parallel
decode all-reduces run on it by default, the sequence-parallel all-gather / reduce-scatter with
`NXD_SP_PEER=1`.  Everything else is torch's ProcessGroupNCCL (RCCL over xGMI).
"""

from __future__ import annotations

import collections
import itertools
import os
import traceback
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

_debug = os.environ.get("NXD_COMM_DEBUG", "0") == "1"
_pending: Dict[int, str] = {}
_ids = itertools.count()


def set_comm_debug(enabled: bool) -> None:
    global _debug
    _debug = bool(enabled)
    _pending.clear()


def comm_debug_enabled() -> bool:
    return _debug


class _Tracked:
    """Async work handle registered in the pending table until waited on."""

    def __init__(self, work, key):
        self._work, self._key = work, key

    def wait(self, *a, **k):
        r = self._work.wait(*a, **k) if self._work is not None else True
        _pending.pop(self._key, None)
        return r

    def is_completed(self):
        return self._work.is_completed() if self._work is not None else True

    def __getattr__(self, name):
        return getattr(self._work, name)


def _track(work, op: str, t: torch.Tensor):
    if not _debug:
        return work
    key = next(_ids)
    site = traceback.extract_stack(limit=4)[0]
    _pending[key] = f"{op}{tuple(t.shape)} {t.dtype} from {os.path.basename(site.filename)}:{site.lineno}"
    return _Tracked(work, key)


def pending_collectives() -> List[str]:
    return list(_pending.values())


# Flight recorder: the last collectives this process issued (sequence number, op, shape, dtype,
# group size), always on -- one deque append per call.  A hung job's watchdog prints it on every
# rank (bench.py); ranks whose last sequence numbers differ are the ones that diverged.
_FLIGHT = collections.deque(maxlen=int(os.environ.get("NXD_COMM_FLIGHT", "64")))
_seq = itertools.count()


def _fr(op: str, t: torch.Tensor, group) -> None:
    try:
        ws = dist.get_world_size(group=group)
    except Exception:  # pragma: no cover
        ws = -1
    _FLIGHT.append((next(_seq), op, tuple(t.shape), str(t.dtype).replace("torch.", ""), ws))


def flight_record(last: Optional[int] = None) -> List[str]:
    recs = list(_FLIGHT)[-last:] if last else list(_FLIGHT)
    return [f"#{n} {op}{shape} {dt} ws={ws}" for n, op, shape, dt, ws in recs]


def assert_no_pending_collectives(where: str) -> None:
    if _debug and _pending:
        raise AssertionError(f"{where}: {len(_pending)} async collective(s) never waited on: "
                             + "; ".join(_pending.values()))


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


# NXD_SP_PEER=1: all-gather / reduce-scatter of GPU tensors (the sequence-parallel activations) over
# IPC-mapped peer buffers, one kernel per call reading every peer directly
# (parallel/peer_allreduce.py PeerCollectives; any group backend, so ranks sharing one GPU over gloo
# run it too).  Off by default: not yet measured across GPUs.
_peer = os.environ.get("NXD_SP_PEER", "0") == "1"
_peer_colls: Dict[object, object] = {}


def _peer_for(group, t: torch.Tensor, op=None):
    if not _peer or not t.is_cuda or (op is not None and op != dist.ReduceOp.SUM):
        return None
    if t.element_size() not in (2, 4) or (t.numel() * t.element_size()) % 16:
        return None
    key = group if group is not None else "world"
    c = _peer_colls.get(key)
    if c is None:
        from .peer_allreduce import PeerCollectives

        c = _peer_colls[key] = PeerCollectives(group)
    return c


def check_peer_collectives(sync: bool = True) -> None:
    """Raise if a peer collective lost a peer (csrc/peer_allreduce.hip marks the call and writes NaN):
    the optimizer step calls this whenever the peer path carried the step's collectives, after a
    stream sync so the step's own calls are covered (the error word is pinned host memory)."""
    if not _peer_colls:
        return
    if sync and torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()
    for c in _peer_colls.values():
        c.check()


def _is_gloo(group) -> bool:
    try:
        return dist.get_backend(group) == "gloo"
    except Exception:  # pragma: no cover
        return False


def all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """out[i*n:(i+1)*n] = inp of rank i (dim 0)."""
    _fr("all_gather", out, group)
    pc = _peer_for(group, inp)
    if pc is not None and (inp.numel() % 8 == 0):
        w = pc.all_gather(out, inp, async_op=async_op)
        return _track(w, "all_gather", out) if async_op else None
    if not _is_gloo(group):
        w = dist.all_gather_into_tensor(out, inp.contiguous(), group=group, async_op=async_op)
        return _track(w, "all_gather", out) if async_op else w
    ws = dist.get_world_size(group=group)
    chunks = list(out.chunk(ws, dim=0))
    src = inp.detach().contiguous().cpu()   # gloo gathers host tensors (GPU tensors are staged)
    tmp = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(tmp, src, group=group)
    for c, t in zip(chunks, tmp):
        c.copy_(t)
    return _track(_Done(), "all_gather", out) if async_op else None


def reduce_scatter_tensor(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False,
                          op=dist.ReduceOp.SUM):
    """out = sum over ranks of inp[rank*n:(rank+1)*n] (dim 0)."""
    _fr("reduce_scatter", inp, group)
    pc = _peer_for(group, inp, op)
    if pc is not None and out.numel() % 8 == 0 and inp.dtype in (torch.bfloat16, torch.float32):
        w = pc.reduce_scatter(out, inp, async_op=async_op)
        return _track(w, "reduce_scatter", inp) if async_op else None
    if not _is_gloo(group):
        w = dist.reduce_scatter_tensor(out, inp.contiguous(), op=op, group=group, async_op=async_op)
        return _track(w, "reduce_scatter", inp) if async_op else w
    ws = dist.get_world_size(group=group)
    r = dist.get_rank(group=group)
    full = inp.contiguous().clone()
    dist.all_reduce(full, op=op, group=group)
    out.copy_(full.chunk(ws, dim=0)[r])
    return _track(_Done(), "reduce_scatter", inp) if async_op else None


def all_reduce(t: torch.Tensor, group=None, async_op: bool = False, op=dist.ReduceOp.SUM):
    _fr("all_reduce", t, group)
    w = dist.all_reduce(t, op=op, group=group, async_op=async_op)
    return _track(w, "all_reduce", t) if async_op else w


def all_reduce_coalesced(tensors: List[torch.Tensor], group=None) -> None:
    """In-place sum of every tensor over `group`: one all-reduce of their concatenation (copied back)."""
    tensors = [t for t in tensors if t.numel()]
    if not tensors or dist.get_world_size(group=group) == 1:
        return
    _fr(f"all_reduce_coalesced[{len(tensors)}]", tensors[0], group)
    if len(tensors) == 1:
        dist.all_reduce(tensors[0], group=group)
        return
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, group=group)
    off = 0
    for t in tensors:
        t.copy_(flat[off:off + t.numel()].view_as(t))
        off += t.numel()


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    _fr("all_to_all", inp, group)
    if not _is_gloo(group):
        w = dist.all_to_all_single(out, inp.contiguous(), group=group, async_op=async_op)
        return _track(w, "all_to_all", inp) if async_op else w
    ws = dist.get_world_size(group=group)
    ins = list(inp.contiguous().chunk(ws, dim=0))
    outs = [torch.empty_like(c) for c in ins]
    _a2a_via_gather(outs, ins, group)
    for o, c in zip(out.chunk(ws, dim=0), outs):
        o.copy_(c)
    return _track(_Done(), "all_to_all", inp) if async_op else None


def _a2a_via_gather(outs: List[torch.Tensor], ins: List[torch.Tensor], group):
    """gloo has no all_to_all: every rank all-gathers the stacked chunks and keeps its column."""
    ws = dist.get_world_size(group=group)
    r = dist.get_rank(group=group)
    stacked = torch.stack(ins).cpu()
    gathered = [torch.empty_like(stacked) for _ in range(ws)]
    dist.all_gather(gathered, stacked, group=group)
    for src in range(ws):
        outs[src].copy_(gathered[src][r])


def send(t: torch.Tensor, dst: int, group=None):
    _fr(f"send->{dst}", t, group)
    return dist.isend(t.contiguous(), dst, group=group)


def recv(t: torch.Tensor, src: int, group=None):
    _fr(f"recv<-{src}", t, group)
    return dist.irecv(t, src, group=group)


def batch_isend_irecv(ops: List[dist.P2POp]):
    if not ops:
        return []
    _fr(f"batch_p2p[{len(ops)}]", ops[0].tensor, ops[0].group)
    return dist.batch_isend_irecv(ops)
