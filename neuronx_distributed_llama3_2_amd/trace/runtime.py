"""Single-controller front end for SPMD inference: one worker process per GPU (rank), driven
from the user's process (reference: trace/trace.py:57-112 TensorParallelNeuronModel runs TP ranks
from one process; trace/model_builder.py:130-261 spawns rank processes).

Each worker initialises torch.distributed (RCCL over xGMI when there is a GPU per rank, gloo on
the CPU otherwise), builds and captures its shard through a picklable `build_fn(rank, world,
*args)`, then serves commands from its queue.  A forward sends the (host) inputs to every rank;
every rank replays its graphs (their collectives meet over RCCL); rank 0 returns the outputs.
"""

from __future__ import annotations

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
    while True:
        cmd, payload = cmd_q.get()
        if cmd == "stop":
            break
        try:
            if cmd == "forward":
                out = obj(*_to_dev(payload, dev))
                res_q.put(("ok", rank, _to_host(out) if rank == 0 else None))
            elif cmd == "call":      # (method name, args): e.g. save
                name, args = payload
                r = getattr(obj, name)(*args)
                res_q.put(("ok", rank, _to_host(r) if rank == 0 else None))
        except Exception:
            res_q.put(("err", rank, traceback.format_exc()))
    try:
        dist.destroy_process_group()
    except Exception:
        pass


class SpmdWorkerPool:
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
        host = _to_host(list(inputs))
        for q in self.cmd_q:
            q.put(("forward", host))
        return self._collect()

    __call__ = forward

    def call(self, name: str, *args):
        for q in self.cmd_q:
            q.put(("call", (name, args)))
        return self._collect()

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
