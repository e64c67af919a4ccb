"""Process launcher for the Lightning integration (reference: lightning/launcher.py:12-91
`_NeuronXLALauncher`, which spawns workers with torch_xla's xmp.spawn or, under torchrun, runs the
function in the already-created rank process).

MI355X mapping: one process per GPU.  Under torchrun (or any launcher that sets LOCAL_RANK /
WORLD_SIZE) the function runs in place on this rank.  Otherwise the launcher starts `num_processes`
fresh rank processes itself (spawn start method, before any HIP call in them), with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, joins them, re-raises the first failure
and returns rank 0's result.  `NeuronLauncher` has no Lightning dependency (it is what the
tests drive on gloo); `_NeuronXLALauncher` adapts it to Lightning's launcher interface.
"""

from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable, Optional

import torch.multiprocessing as mp

from ._compat import HAVE_LIGHTNING


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank: int, world: int, addr: str, port: int, function: Callable, args, kwargs, queue) -> None:
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=str(port))
    try:
        out = function(*args, **kwargs)
        queue.put((rank, True, out if rank == 0 else None))
    except BaseException:  # reported to the parent, which re-raises
        queue.put((rank, False, traceback.format_exc()))
        raise


class NeuronLauncher:
    """Runs `function` on every rank of a single-node job and returns rank 0's result."""

    def __init__(self, num_processes: int, start_method: str = "spawn", master_addr: str = "127.0.0.1"):
        self.num_processes = int(num_processes)
        self.start_method = start_method
        self.master_addr = master_addr
        self.procs = []

    @property
    def creates_processes_externally(self) -> bool:
        return "LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ

    @property
    def is_interactive_compatible(self) -> bool:
        return False

    def launch(self, function: Callable, *args: Any, **kwargs: Any) -> Any:
        if self.creates_processes_externally or self.num_processes <= 1:
            return function(*args, **kwargs)
        ctx = mp.get_context(self.start_method)
        queue = ctx.SimpleQueue()
        port = int(os.environ.get("MASTER_PORT") or _free_port())
        self.procs = [ctx.Process(target=_rank_main, args=(r, self.num_processes, self.master_addr, port, function,
                                                           args, kwargs, queue))
                      for r in range(self.num_processes)]
        for p in self.procs:
            p.start()
        results = {}
        failure: Optional[str] = None
        while len(results) < self.num_processes:
            rank, ok, payload = queue.get()
            results[rank] = payload
            if not ok and failure is None:
                failure = f"rank {rank} failed:\n{payload}"
                for p in self.procs:
                    if p.is_alive():
                        p.terminate()
                break
        for p in self.procs:
            p.join()
        if failure is None:
            bad = [p.exitcode for p in self.procs if p.exitcode != 0]
            if bad:
                failure = f"rank processes exited with codes {bad}"
        if failure is not None:
            raise RuntimeError(failure)
        return results.get(0)


if HAVE_LIGHTNING:  # pragma: no cover - Lightning is not installed in this build environment
    try:
        from lightning.pytorch.strategies.launchers.launcher import _Launcher  # type: ignore
    except ImportError:
        from pytorch_lightning.strategies.launchers.launcher import _Launcher  # type: ignore

    class _NeuronXLALauncher(_Launcher):
        """Lightning launcher over NeuronLauncher (reference name kept)."""

        def __init__(self, strategy) -> None:
            self._strategy = strategy
            self._core = NeuronLauncher(getattr(strategy, "num_processes", 1))

        @property
        def is_interactive_compatible(self) -> bool:
            return False

        def launch(self, function: Callable, *args: Any, trainer=None, **kwargs: Any) -> Any:
            if self._core.creates_processes_externally:
                self._strategy._local_rank = int(os.environ["LOCAL_RANK"])
            return self._core.launch(function, *args, **kwargs)
