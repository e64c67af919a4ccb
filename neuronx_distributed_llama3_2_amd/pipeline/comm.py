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
    """Collects p2p ops, then issues them as one group and waits."""

    def __init__(self):
        self.ops: List[dist.P2POp] = []
        self.keep: List[torch.Tensor] = []

    def send(self, t: torch.Tensor, dst: int):
        t = t.contiguous()
        self.keep.append(t)
        self.ops.append(dist.P2POp(dist.isend, t, dst))

    def recv(self, t: torch.Tensor, src: int):
        self.ops.append(dist.P2POp(dist.irecv, t, src))

    def flush(self):
        if not self.ops:
            return
        reqs = dist.batch_isend_irecv(self.ops)
        for r in reqs:
            r.wait()
        self.ops = []
        self.keep = []


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
