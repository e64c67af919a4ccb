"""RCCL (torch.distributed "nccl" backend on ROCm) environment for a single MI355X node.

Eight MI355X in a node are fully connected by xGMI: 7 point-to-point links per GPU, no switch.
A ring collective therefore runs at the rate of ONE link per direction per channel, and the
knob that matters is how many channels (= RCCL workgroups, i.e. CUs taken from compute) each
collective uses.  The chunked SP overlap (parallel_layers/sp.py) wants collectives that leave
most CUs to the concurrent GEMM; a pure comm benchmark wants many channels.  Both are settable:

    NXD_RCCL_CHANNELS=<n>   -> NCCL_MAX_NCHANNELS = n (default 16; 0 / "auto": RCCL picks)
    NXD_COMM_HIGH_PRIORITY  -> TP / EP groups get high-priority RCCL streams (default 1;
                               parallel_layers/parallel_state.py)

Default channel cap, from profiles/r3_cu_interference.jsonl (one MI355X: TP=8-shape GEMMs and the
FA forward on the compute stream while a copy kernel of K workgroups -- RCCL runs one per channel --
streams on a side stream): any concurrent side kernel costs 12-30 % at K = 4-16 (flat), rising to
1.4-2.4x at K = 64-128.  A ring channel moves about one xGMI link's worth, so 16 channels (> 2 per
link of the 7) keep the links busy while staying on the flat part of that curve for the SP
all-gathers / reduce-scatters that overlap GEMMs.  Only the cap is set (RCCL may use fewer).

`apply_rccl_env()` sets library defaults BEFORE `init_process_group` without overriding anything
the user exported; `log_comm_config()` logs the effective RCCL-related environment once per
process, so every run records the configuration its numbers were taken with.
"""

from __future__ import annotations

import os
from typing import Dict, Optional

from ..utils.logger import get_logger

logger = get_logger()

# defaults that are safe for any workload on one node
RCCL_DEFAULTS: Dict[str, str] = {
    # the dmabuf IPC path is the only one the ROCm driver on these nodes supports
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    # stash collective inputs in the work object instead of recordStream-ing them into the
    # caching allocator (no cross-stream free-list fragmentation under async SP collectives)
    "TORCH_NCCL_AVOID_RECORD_STREAMS": "1",
}

DEFAULT_CHANNELS = 16

_PREFIXES = ("NCCL_", "RCCL_", "TORCH_NCCL_", "NXD_RCCL", "NXD_COMM", "NXD_SP_CHUNKS", "HSA_ENABLE_IPC",
             "TENSILE_STREAMK")
_logged = False


def apply_rccl_env(extra: Optional[Dict[str, str]] = None, world_size: int = 1) -> Dict[str, str]:
    """Set the library's RCCL defaults (and `extra`) where the environment does not already
    define them.  Returns what was set.  Call before `torch.distributed.init_process_group`.

    NXD_COMM_RESERVE_CUS=n (multi-rank runs only): cap hipBLASLt's persistent stream-K GEMMs at
    (CUs - n) workgroups (TENSILE_STREAMK_MAX_CUS), so n CUs stay free for the RCCL channel
    kernels: a stream-K GEMM holds one workgroup on every CU for its whole duration, and a
    collective launched behind it cannot start until one retires (the emulated TP=8 rank's link
    kernels started late behind them: profiles/r4_stream_timeline_8layers.jsonl)."""
    want = dict(RCCL_DEFAULTS)
    ch = os.environ.get("NXD_RCCL_CHANNELS", str(DEFAULT_CHANNELS))
    if ch and ch not in ("0", "auto"):
        want["NCCL_MAX_NCHANNELS"] = ch
    reserve = int(os.environ.get("NXD_COMM_RESERVE_CUS", "0") or 0)
    if reserve > 0 and world_size > 1:
        want["TENSILE_STREAMK_MAX_CUS"] = str(max(1, _num_cus() - reserve))
    if extra:
        want.update(extra)
    applied = {}
    for k, v in want.items():
        if k not in os.environ:
            os.environ[k] = str(v)
            applied[k] = str(v)
    return applied


def _num_cus() -> int:
    try:
        import torch

        if torch.cuda.is_available():
            return int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    except Exception:  # pragma: no cover
        pass
    return 256


def comm_config() -> Dict[str, str]:
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(_PREFIXES)}


def log_comm_config(force: bool = False) -> Dict[str, str]:
    global _logged
    cfg = comm_config()
    if force or not _logged:
        _logged = True
        logger.info("> communication environment: %s", " ".join(f"{k}={v}" for k, v in cfg.items()) or "(defaults)")
    return cfg
