"""Rank-aware logging (reference: src/neuronx_distributed/utils/logger.py:16-112).

`NXD_LOG_LEVEL` sets the level (default INFO), `NXD_LOG_HIDE_TIME=1` drops timestamps,
`NXD_LOG_STREAM=stderr` sends records to stderr instead of stdout (bench.py: stdout carries only its
JSON result line); by default only global rank 0 emits records.
"""

from __future__ import annotations

import logging
import os
import sys

_LOGGERS = {}


def get_log_level() -> int:
    lvl = os.environ.get("NXD_LOG_LEVEL", "INFO").upper()
    return {"TRACE": logging.DEBUG, "DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING,
            "WARNING": logging.WARNING, "ERROR": logging.ERROR, "FATAL": logging.CRITICAL,
            "OFF": logging.CRITICAL + 10}.get(lvl, logging.INFO)


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0"))


class _RankFilter(logging.Filter):
    def __init__(self, rank0_only: bool):
        super().__init__()
        self.rank0_only = rank0_only

    def filter(self, record):
        return (not self.rank0_only) or _rank() == 0


def get_logger(name: str = "neuronx_distributed", rank0_only: bool = True) -> logging.Logger:
    key = (name, rank0_only)
    if key in _LOGGERS:
        return _LOGGERS[key]
    lg = logging.getLogger(f"{name}{'' if rank0_only else '.all'}")
    lg.setLevel(get_log_level())
    lg.propagate = False
    if not lg.handlers:
        h = logging.StreamHandler(sys.stderr if os.environ.get("NXD_LOG_STREAM") == "stderr" else sys.stdout)
        fmt = "%(levelname)s %(name)s: %(message)s" if os.environ.get("NXD_LOG_HIDE_TIME") == "1" else \
            "%(asctime)s.%(msecs)03d %(levelname)s %(name)s: %(message)s"
        h.setFormatter(logging.Formatter(fmt, datefmt="%Y-%m-%d %H:%M:%S"))
        h.addFilter(_RankFilter(rank0_only))
        lg.addHandler(h)
    _LOGGERS[key] = lg
    return lg
