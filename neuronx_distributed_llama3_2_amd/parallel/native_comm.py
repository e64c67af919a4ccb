"""Native RCCL collective layer (csrc/comm.cpp) for the framework's own buckets.

torch.distributed (backend "nccl" = RCCL) stays the default communication path; this module adds,
per process group, an RCCL communicator created directly from C++ plus:

* coalesced launches -- a list of tensors in ONE RCCL group call (all-reduce, reduce-scatter,
  all-gather, batched send/recv), instead of one ProcessGroup work object per tensor;
* bucketed all-reduce -- many small tensors packed into a persistent 16-B-aligned staging buffer
  by one HIP kernel (csrc/comm_pack.hip), one all-reduce, one unpack;
* explicit streams and events -- collectives run on the communicator's own (high-priority) HIP
  stream, ordered after the producer's stream by an event; `wait()` orders the consumer; tensors
  are recorded on the comm stream so the caching allocator never recycles them early.

The RCCL environment (channels, protocol, xGMI settings: parallel/rccl_env.py) applies at
communicator creation exactly as for torch's communicators.
"""

from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..ops._ext import ext


def _rccl_path() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class Work:
    """Handle of an asynchronous native collective."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.event)

    def is_completed(self) -> bool:
        return self.event.query()


class NativeCommunicator:
    def __init__(self, group=None, high_priority: bool = True, staging_bytes: int = 64 << 20):
        if not torch.cuda.is_available():
            raise RuntimeError("NativeCommunicator needs a GPU (RCCL)")
        if not dist.is_initialized():
            raise RuntimeError("initialise torch.distributed first (the RCCL unique id travels over it)")
        C = ext()
        C.comm_load(_rccl_path())
        self.group = group
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
        self.rank = dist.get_rank(group) if group is not None else dist.get_rank()
        self.size = len(ranks)
        uid = [C.comm_unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(uid, src=ranks[0], group=group)
        self.device = torch.cuda.current_device()
        self.handle = C.comm_init(uid[0], self.size, self.rank, self.device)
        self.stream = torch.cuda.Stream(priority=-1 if high_priority else 0)
        self._staging = None
        self._staging_bytes = staging_bytes

    # ---------------------------------------------------------------- plumbing
    def _enter(self, tensors: Sequence[torch.Tensor]):
        self.stream.wait_stream(torch.cuda.current_stream())
        for t in tensors:
            t.record_stream(self.stream)

    def _leave(self, async_op: bool) -> Optional[Work]:
        ev = torch.cuda.Event()
        ev.record(self.stream)
        w = Work(ev)
        if not async_op:
            w.wait()
            return None
        return w

    def staging(self, nbytes: int) -> torch.Tensor:
        if self._staging is None or self._staging.numel() < nbytes:
            self._staging = torch.empty(max(nbytes, self._staging_bytes), dtype=torch.uint8, device=self.device)
        return self._staging

    # ---------------------------------------------------------------- collectives
    def all_reduce(self, tensors: List[torch.Tensor], op: str = "sum", async_op: bool = False):
        self._enter(tensors)
        ext().comm_all_reduce(self.handle, list(tensors), op, self.stream.cuda_stream)
        return self._leave(async_op)

    def reduce_scatter(self, outs: List[torch.Tensor], ins: List[torch.Tensor], op: str = "sum", async_op: bool = False):
        self._enter(list(outs) + list(ins))
        ext().comm_reduce_scatter(self.handle, list(outs), list(ins), op, self.stream.cuda_stream)
        return self._leave(async_op)

    def all_gather(self, outs: List[torch.Tensor], ins: List[torch.Tensor], async_op: bool = False):
        self._enter(list(outs) + list(ins))
        ext().comm_all_gather(self.handle, list(outs), list(ins), self.stream.cuda_stream)
        return self._leave(async_op)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        self._enter([out, inp])
        ext().comm_all_to_all(self.handle, out, inp, self.stream.cuda_stream)
        return self._leave(async_op)

    def batch_p2p(self, sends=(), send_peers=(), recvs=(), recv_peers=(), async_op: bool = False):
        self._enter(list(sends) + list(recvs))
        ext().comm_batch_p2p(self.handle, list(sends), [int(p) for p in send_peers], list(recvs),
                             [int(p) for p in recv_peers], self.stream.cuda_stream)
        return self._leave(async_op)

    def bucketed_all_reduce(self, tensors: List[torch.Tensor], op: str = "sum", async_op: bool = False):
        """All-reduce many small same-dtype tensors as one collective through the staging buffer."""
        if not tensors:
            return None
        need = sum((t.numel() * t.element_size() + 15) // 16 * 16 for t in tensors)
        st = self.staging(need)
        self._enter(list(tensors) + [st])
        ext().comm_bucketed_all_reduce(self.handle, list(tensors), st, op, self.stream.cuda_stream)
        return self._leave(async_op)

    def close(self) -> None:
        if getattr(self, "handle", None) is not None:
            torch.cuda.synchronize()
            ext().comm_destroy(self.handle)
            self.handle = None
