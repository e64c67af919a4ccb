"""Failure detection, fault injection and restart supervision.

The reference has no elastic training, heartbeats or fault injection; its robustness is limited to
checkpoint `done` markers + cleanup of interrupted tags (src/neuronx_distributed/trainer/
checkpoint.py:62-89, 232-242), resume-from-latest (examples/training/llama/
tp_zero1_llama_hf_pretrain.py:371-391) and storage retries (trainer/checkpoint_storage.py:280-302).
This module keeps those semantics (see trainer/checkpoint.py) and adds:

* `fault_point(name)` — named injection sites compiled into the checkpoint writer and the training
  loop.  `NXD_FAULT_INJECT="site[@rank][:action][,...]"` arms them; action `exit` (default:
  `os._exit(FAULT_EXIT_CODE)`, i.e. a rank dying without cleanup), `raise` (`InjectedFault`) or
  `hang` (sleeps forever; for watchdog tests).  Disarmed sites cost one dict lookup.
* `StepWatchdog` — a host heartbeat: if the training loop does not `kick()` within `timeout_s`
  (a hung RCCL collective, a stuck kernel) it dumps every thread's Python stack and, by default,
  terminates the process so the supervisor can restart it.  RCCL's own watchdog
  (`TORCH_NCCL_ASYNC_ERROR_HANDLING`) is configured by `configure_collective_watchdog()`.
* `run_with_restarts(cmd)` — minimal elastic supervisor: runs the training command as a child
  process and restarts it (up to `max_restarts`) when it fails; the script resumes from the latest
  checkpoint that has its `done` marker (`loading_step="latest_if_exists"` semantics).
"""

from __future__ import annotations

import faulthandler
import os
import subprocess
import sys
import threading
import time
from datetime import timedelta
from typing import Callable, Dict, List, Optional, Sequence, Tuple

FAULT_EXIT_CODE = 43
_ENV = "NXD_FAULT_INJECT"


class InjectedFault(RuntimeError):
    pass


_parsed: Optional[Tuple[str, Dict[str, Tuple[Optional[int], int, str]]]] = None
_hits: Dict[str, int] = {}


def _sites() -> Dict[str, Tuple[Optional[int], int, str]]:
    global _parsed
    spec = os.environ.get(_ENV, "")
    if _parsed is None or _parsed[0] != spec:
        sites = {}
        for item in filter(None, (s.strip() for s in spec.split(","))):
            action = "exit"
            if ":" in item:
                item, action = item.split(":", 1)
            hit = 1
            if "#" in item:
                item, h = item.split("#", 1)
                hit = int(h)
            rank = None
            if "@" in item:
                item, r = item.split("@", 1)
                rank = int(r)
            if action not in ("exit", "raise", "hang"):
                raise ValueError(f"{_ENV}: unknown action {action!r}")
            sites[item] = (rank, hit, action)
        _parsed = (spec, sites)
        _hits.clear()
    return _parsed[1]


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0"))


def fault_point(name: str) -> None:
    """Injection site `name`; a no-op unless armed through NXD_FAULT_INJECT."""
    sites = _sites()
    if name not in sites:
        return
    rank, hit, action = sites[name]
    if rank is not None and rank != _rank():
        return
    _hits[name] = _hits.get(name, 0) + 1
    if _hits[name] != hit:
        return
    if action == "raise":
        raise InjectedFault(f"injected fault at {name}")
    if action == "hang":
        while True:
            time.sleep(3600)
    sys.stderr.write(f"[nxd] injected fault at {name}: exiting rank {_rank()}\n")
    sys.stderr.flush()
    os._exit(FAULT_EXIT_CODE)


class StepWatchdog:
    """Host-side heartbeat for the training loop.

        wd = StepWatchdog(timeout_s=600)
        for step in ...:
            train_step(); wd.kick()
        wd.stop()

    On expiry: dump all thread stacks to stderr, call `on_timeout` (if given), then exit the process
    with `exit_code` unless `on_timeout` is given and `exit_on_timeout` is False.
    """

    def __init__(self, timeout_s: float, on_timeout: Optional[Callable[[], None]] = None,
                 exit_on_timeout: Optional[bool] = None, exit_code: int = 124, poll_s: Optional[float] = None):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout
        self.exit_on_timeout = (on_timeout is None) if exit_on_timeout is None else exit_on_timeout
        self.exit_code = exit_code
        self.fired = False
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._poll = poll_s if poll_s is not None else min(1.0, self.timeout_s / 4)
        self._t = threading.Thread(target=self._loop, name="nxd-step-watchdog", daemon=True)
        self._t.start()

    def kick(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        self._t.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
        return False

    def _loop(self):
        while not self._stop.wait(self._poll):
            if time.monotonic() - self._last > self.timeout_s:
                self.fired = True
                sys.stderr.write(f"[nxd] step watchdog: no progress for {self.timeout_s:.0f}s on rank {_rank()}\n")
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                if self.on_timeout is not None:
                    self.on_timeout()
                if self.exit_on_timeout:
                    os._exit(self.exit_code)
                return


def configure_collective_watchdog(timeout_s: float = 1800.0) -> timedelta:
    """Enable RCCL async error handling (a failed / timed-out collective tears the process down
    instead of hanging every rank) and return the timeout to pass to init_process_group."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
    os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "1")
    return timedelta(seconds=timeout_s)


def run_with_restarts(cmd: Sequence[str], max_restarts: int = 3, env: Optional[Dict[str, str]] = None,
                      backoff_s: float = 1.0, on_restart: Optional[Callable[[int, int], Dict[str, str]]] = None) -> int:
    """Run `cmd` as a child process; on a non-zero exit restart it up to `max_restarts` times.

    `on_restart(attempt, returncode)` may return env overrides for the next attempt (e.g. to disarm
    an injected fault).  Returns the final exit code.  The child resumes from its own checkpoints.
    """
    attempt, cur_env = 0, dict(os.environ if env is None else env)
    while True:
        rc = subprocess.call(list(cmd), env=cur_env)
        if rc == 0 or attempt >= max_restarts:
            return rc
        attempt += 1
        sys.stderr.write(f"[nxd] worker exited with {rc}; restart {attempt}/{max_restarts}\n")
        if on_restart is not None:
            cur_env.update(on_restart(attempt, rc) or {})
        time.sleep(backoff_s)


def main(argv: Optional[List[str]] = None) -> int:
    """`python -m neuronx_distributed_llama3_2_amd.utils.resilience --max-restarts N -- <cmd ...>`"""
    import argparse

    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        raise SystemExit("usage: resilience [--max-restarts N] -- <command ...>")
    i = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--backoff", type=float, default=5.0)
    a = ap.parse_args(argv[:i])
    return run_with_restarts(argv[i + 1:], max_restarts=a.max_restarts, backoff_s=a.backoff)


if __name__ == "__main__":
    sys.exit(main())
