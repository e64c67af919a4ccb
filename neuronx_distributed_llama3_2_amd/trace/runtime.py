"""Single-controller front end for SPMD inference: one worker process per GPU (rank), driven
from the user's process (reference: trace/trace.py:57-112 TensorParallelNeuronModel runs TP ranks
from one process; trace/model_builder.py:130-261 spawns rank processes).

Each worker initialises torch.distributed (RCCL over xGMI when there is a GPU per rank, gloo on
the CPU otherwise), builds and captures its shard through a picklable `build_fn(rank, world,
*args)`, then serves commands from its queue.  A forward makes every rank replay its graphs
(their collectives meet over RCCL); rank 0 returns the outputs.

Tensor I/O goes through PERSISTENT shared-memory buffers, not through the command queues: the
controller copies each input into its bound shared input buffer (re-bound only when a larger
shape arrives), every rank views the same pages and copies them to its GPU; rank 0 writes the
outputs into shared output buffers it handed to the controller once.  A call's queue traffic is
a few small tuples (shapes / dtypes), so the per-call cost is two memcpys plus the H2D / D2H
copies, independent of how the tensors were produced.
"""

from __future__ import annotations

import math
import os
import socket
import traceback
from typing import Any, Callable, List, Sequence

import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _to_host(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_host(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_host(v) for k, v in x.items()}
    return x


class _SharedSlots:
    """Growable set of shared-memory CPU buffers, one per tensor position of a call."""

    def __init__(self):
        self.bufs: List[torch.Tensor] = []

    def fit(self, tensors: List[torch.Tensor]) -> bool:
        """Make every slot large enough and of the right dtype; True when (re)allocation happened
        (the new buffers must then be handed to the other side)."""
        changed = len(self.bufs) != len(tensors)
        new = []
        for i, t in enumerate(tensors):
            b = self.bufs[i] if i < len(self.bufs) else None
            if b is None or b.dtype != t.dtype or b.numel() < t.numel():
                b = torch.empty(max(t.numel(), 1), dtype=t.dtype).share_memory_()
                changed = True
            new.append(b)
        self.bufs = new
        return changed

    def write(self, tensors: List[torch.Tensor]):
        meta = []
        for b, t in zip(self.bufs, tensors):
            b[:t.numel()].copy_(t.detach().reshape(-1), non_blocking=False)
            meta.append(tuple(t.shape))
        return meta

    def views(self, meta):
        return [b[:math.prod(shape)].view(shape) for b, shape in zip(self.bufs, meta)]


def _tensor_bytes(x) -> int:
    if isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, (list, tuple)):
        return sum(_tensor_bytes(v) for v in x)
    if isinstance(x, dict):
        return sum(_tensor_bytes(v) for v in x.values())
    return 0


def _flatten_out(out):
    """(tensors, structure) of a forward's output: a tensor or a (nested) list / tuple of them."""
    if isinstance(out, torch.Tensor):
        return [out], "T"
    if isinstance(out, (list, tuple)) and all(isinstance(o, torch.Tensor) for o in out):
        return list(out), ("L" if isinstance(out, list) else "U", len(out))
    return None, None


def _unflatten_out(tensors, structure):
    if structure == "T":
        return tensors[0]
    kind, _ = structure
    return list(tensors) if kind == "L" else tuple(tensors)


def _to_dev(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    if isinstance(x, (list, tuple)):
        return type(x)(_to_dev(v, dev) for v in x)
    return x


def worker_device(rank: int, world: int) -> torch.device:
    if os.environ.get("NXD_SPMD_DEVICE", "") == "cpu" or not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", rank % torch.cuda.device_count())


def _worker_main(rank, world, port, build_fn, build_args, cmd_q, res_q):
    import torch.distributed as dist

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    try:
        dev = worker_device(rank, world)
        gpus = torch.cuda.device_count() if dev.type == "cuda" else 0
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        backend = "nccl" if dev.type == "cuda" and gpus >= world else "gloo"
        dist.init_process_group(backend, rank=rank, world_size=world)
        from ..parallel_layers import parallel_state as ps

        ps.initialize_model_parallel(tensor_model_parallel_size=world)
        obj = build_fn(rank, world, *build_args)
        res_q.put(("ready", rank, None))
    except Exception:
        res_q.put(("err", rank, traceback.format_exc()))
        return
    in_slots = _SharedSlots()
    out_slots = _SharedSlots()
    while True:
        cmd, payload = cmd_q.get()
        if cmd == "stop":
            break
        try:
            if cmd == "bind":         # new shared input buffers (shape growth / first call)
                in_slots.bufs = list(payload)
                res_q.put(("ok", rank, None))
            elif cmd == "forward_shm":
                inputs = [v.to(dev, non_blocking=False) for v in in_slots.views(payload)]
                out = obj(*inputs)
                reply = None
                if rank == 0:
                    tensors, structure = _flatten_out(out)
                    if tensors is None:                       # not tensor-shaped: plain (pickled) reply
                        reply = ("obj", _to_host(out))
                    else:
                        host = [t.detach().cpu() for t in tensors]
                        rebound = out_slots.fit(host)
                        meta = out_slots.write(host)
                        reply = ("shm", structure, meta, out_slots.bufs if rebound else None)
                res_q.put(("ok", rank, reply))
            elif cmd == "forward":
                out = obj(*_to_dev(payload, dev))
                res_q.put(("ok", rank, _to_host(out) if rank == 0 else None))
            elif cmd == "call":      # (method name, args[, kwargs]): e.g. save, generate
                name, args = payload[0], payload[1]
                kwargs = payload[2] if len(payload) > 2 else {}
                r = getattr(obj, name)(*_to_dev(args, dev), **kwargs)
                res_q.put(("ok", rank, _to_host(r) if rank == 0 else None))
        except Exception:
            res_q.put(("err", rank, traceback.format_exc()))
    try:
        dist.destroy_process_group()
    except Exception:
        pass


class SpmdWorkerPool:
    last_host_bytes = 0

    def __init__(self, world: int, build_fn: Callable, build_args: Sequence[Any] = (), timeout: float = 1800.0):
        ctx = mp.get_context("spawn")
        self.world, self.timeout = world, timeout
        port = _free_port()
        self.cmd_q = [ctx.Queue() for _ in range(world)]
        self.res_q = ctx.Queue()
        self.procs = [ctx.Process(target=_worker_main, args=(r, world, port, build_fn, tuple(build_args),
                                                              self.cmd_q[r], self.res_q), daemon=True)
                      for r in range(world)]
        for p in self.procs:
            p.start()
        self._in_slots = _SharedSlots()
        self._out_slots = _SharedSlots()
        self._collect()

    def _collect(self):
        results = [None] * self.world
        errs = []
        for _ in range(self.world):
            kind, rank, val = self.res_q.get(timeout=self.timeout)
            if kind == "err":
                errs.append(f"rank {rank}:\n{val}")
            results[rank] = val
        if errs:
            self.close()
            raise RuntimeError("SPMD worker failed:\n" + "\n".join(errs))
        return results[0]

    def forward(self, *inputs: torch.Tensor):
        if not all(isinstance(t, torch.Tensor) for t in inputs):
            host = _to_host(list(inputs))
            for q in self.cmd_q:
                q.put(("forward", host))
            return self._collect()
        slots = self._in_slots
        if slots.fit(list(inputs)):
            for q in self.cmd_q:
                q.put(("bind", slots.bufs))
            self._collect()
        meta = slots.write(list(inputs))
        for q in self.cmd_q:
            q.put(("forward_shm", meta))
        reply = self._collect()
        if reply[0] == "obj":
            return reply[1]
        _, structure, out_meta, new_bufs = reply
        if new_bufs is not None:
            self._out_slots.bufs = list(new_bufs)
        # copy out of the shared buffers: the next call overwrites them
        outs = [v.clone() for v in self._out_slots.views(out_meta)]
        return _unflatten_out(outs, structure)

    __call__ = forward

    def call(self, name: str, *args, **kwargs):
        """Run `obj.<name>(*args, **kwargs)` on every rank (tensors moved to each rank's device);
        rank 0's result comes back.  `last_host_bytes` counts the tensor bytes this call moved
        between the controller and the workers."""
        for q in self.cmd_q:
            q.put(("call", (name, args, kwargs)))
        r = self._collect()
        self.last_host_bytes = self.world * _tensor_bytes(args) + _tensor_bytes(kwargs) * self.world + _tensor_bytes(r)
        return r

    def close(self) -> None:
        for q in self.cmd_q:
            try:
                q.put(("stop", None))
            except Exception:
                pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.procs = []

    def __del__(self):
        if getattr(self, "procs", None):
            self.close()
