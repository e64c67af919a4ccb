"""Pipeline point-to-point communication (reference: src/neuronx_distributed/pipeline/comm.py:38-197).

Tensors move with REAL RCCL send/recv between neighbouring stages (the reference emulates p2p with
2-rank all-gathers because its XLA backend has none); all the sends/receives a stage issues between
two compute tasks are submitted as ONE `batch_isend_irecv` group, which is what makes bidirectional
exchanges between neighbours deadlock-free.  Python metadata (tensor shapes/dtypes, discovered
once per input shape) travels over the gloo pipeline group.
"""

from __future__ import annotations

from typing import Any, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state as ps


class P2PGroup:
    """Asynchronous p2p runtime of one pipeline step.

    `send`/`recv` collect ops; `issue()` submits everything collected since the previous issue as
    ONE `batch_isend_irecv` exchange (neighbours' exchanges pair up in issue order, which is what
    keeps bidirectional traffic deadlock-free) and returns immediately: on RCCL the transfer runs
    on the communicator's own HIP stream while the compute stream keeps going.  Only a consumer
    waits -- `wait_for(tensors)` waits the exchange(s) that fill those receive buffers (on RCCL a
    stream-level wait: the host never blocks) -- and sent buffers stay referenced until their
    exchange is retired, so a send never blocks the next compute task.  `flush()` retires all.
    """

    def __init__(self):
        self.ops: List[dist.P2POp] = []
        self.keep: List[torch.Tensor] = []
        # gloo (CPU tests, the one-GPU multi-rank rehearsal) moves raw pointers from its own host
        # threads with no HIP stream ordering: GPU tensors are staged through host copies, a send
        # after the producing stream finished, a receive copied in when its exchange is retired
        self._stage = dist.is_initialized() and dist.get_backend() == "gloo"
        self._copy_in: List[Tuple[torch.Tensor, torch.Tensor]] = []   # (host buffer, device tensor)
        self._inflight: List[Tuple[list, List[torch.Tensor]]] = []   # (works, tensors) per exchange
        self._exchange_of: dict = {}                                  # id(recv buffer) -> exchange
        self.max_inflight = 64   # bound on outstanding exchanges (oldest retired first)

    def send(self, t: torch.Tensor, dst: int):
        t = t.contiguous()
        if self._stage and t.is_cuda:
            t = t.detach().cpu()   # waits for the producing stream
        self.keep.append(t)
        self.ops.append(dist.P2POp(dist.isend, t, dst))

    def recv(self, t: torch.Tensor, src: int):
        self.keep.append(t)
        buf = t
        if self._stage and t.is_cuda:
            buf = torch.empty(t.shape, dtype=t.dtype, device="cpu")
            self.keep.append(buf)
            self._copy_in.append((buf, t))
        self.ops.append(dist.P2POp(dist.irecv, buf, src))

    def issue(self) -> None:
        if not self.ops:
            return
        works = dist.batch_isend_irecv(self.ops)
        ex = (list(works), self.keep, self._copy_in)
        self._inflight.append(ex)
        for op in self.ops:
            if op.op is dist.irecv:
                self._exchange_of[id(op.tensor)] = ex
        for _, dev in self._copy_in:
            self._exchange_of[id(dev)] = ex
        self.ops, self.keep, self._copy_in = [], [], []
        while len(self._inflight) > self.max_inflight:
            self._retire(self._inflight[0])

    def _retire(self, ex) -> None:
        works, tensors, copy_in = ex
        for w in works:
            w.wait()
        works.clear()
        for host, dev in copy_in:
            dev.copy_(host)
            self._exchange_of.pop(id(dev), None)
        copy_in.clear()
        for t in tensors:
            self._exchange_of.pop(id(t), None)
        # by identity: tuple == would compare the (possibly emptied) lists element-wise, i.e. tensors
        self._inflight = [e for e in self._inflight if e is not ex]

    def wait_for(self, tensors) -> None:
        """Make the receive buffers in `tensors` safe to read (issues pending ops first)."""
        self.issue()
        for t in tensors:
            ex = self._exchange_of.get(id(t))
            if ex is not None:
                self._retire(ex)

    def pending(self) -> int:
        return len(self._inflight) + (1 if self.ops else 0)

    def flush(self):
        self.issue()
        while self._inflight:
            self._retire(self._inflight[0])


def send(tensor: torch.Tensor, dst: int) -> None:
    g = P2PGroup()
    g.send(tensor, dst)
    g.flush()


def recv_from(tensor: torch.Tensor, src: int) -> torch.Tensor:
    g = P2PGroup()
    g.recv(tensor, src)
    g.flush()
    return tensor


def send_python_object(obj: Any, dst: int) -> None:
    dist.send_object_list([obj], dst=dst, group=ps.get_pp_gloo_group())


def recv_python_object(src: int) -> Any:
    box = [None]
    dist.recv_object_list(box, src=src, group=ps.get_pp_gloo_group())
    return box[0]
