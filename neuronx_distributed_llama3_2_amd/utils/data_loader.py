"""Input pipeline: native token loader (csrc/dataloader.cpp: mmap'd corpus, C++ worker threads,
pinned batch ring) + device prefetch on a side HIP stream (the MI355X replacement of torch_xla's
MpDeviceLoader, reference src/neuronx_distributed/pipeline/model.py:1590-1591).

    loader = TokenDataLoader("corpus.bin", seq_len=8192, batch=1, dp_rank=r, dp_size=d, token_bytes=4)
    for batch in DevicePrefetcher(loader, device):   # {"input_ids", "labels"} on the GPU
        ...

`write_token_file` converts token id arrays / HF datasets to the flat corpus format.
"""

from __future__ import annotations

from typing import Dict, Iterable, Optional

import numpy as np
import torch

from ..ops._ext import ext


def write_token_file(path: str, token_arrays: Iterable, token_bytes: int = 4) -> int:
    """Concatenate token id sequences into a flat uint16/uint32 file; returns #tokens."""
    dt = np.uint16 if token_bytes == 2 else np.uint32
    n = 0
    with open(path, "wb") as f:
        for arr in token_arrays:
            a = np.asarray(arr, dtype=np.int64)
            if token_bytes == 2 and a.size and a.max() >= 1 << 16:
                raise ValueError("token id does not fit uint16")
            a.astype(dt).tofile(f)
            n += a.size
    return n


class TokenDataLoader:
    """Iterator over [batch, seq_len + 1] int64 host batches from the native loader."""

    def __init__(self, path: str, seq_len: int, batch: int, dp_rank: int = 0, dp_size: int = 1, seed: int = 0,
                 token_bytes: int = 4, threads: int = 4, prefetch: int = 4, pin: bool = True):
        self._l = ext().TokenLoader(path, token_bytes, seq_len, batch, dp_rank, dp_size, seed, threads, prefetch,
                                    pin and torch.cuda.is_available())
        self.seq_len, self.batch = seq_len, batch

    def __iter__(self):
        return self

    def __next__(self) -> torch.Tensor:
        return self._l.next()

    def state_dict(self) -> Dict[str, int]:
        e, s = self._l.state()
        return {"epoch": int(e), "step": int(s)}

    def load_state_dict(self, st: Dict[str, int]) -> None:
        self._l.set_state(int(st["epoch"]), int(st["step"]))

    @property
    def steps_per_epoch(self) -> int:
        return int(self._l.steps_per_epoch())


class DevicePrefetcher:
    """Copies the next host batch to the device on a side stream while the current step runs;
    yields {"input_ids", "labels"} ([batch, seq_len] each, labels = inputs shifted by one)."""

    def __init__(self, loader, device: Optional[torch.device] = None):
        self.loader = loader
        self.device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                                 else torch.device("cpu"))
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._next = None

    def _stage(self):
        host = next(self.loader)
        if self.stream is None:
            t = host.clone()
        else:
            with torch.cuda.stream(self.stream):
                t = host.to(self.device, non_blocking=True)
            # the host slot is recycled by the loader's next call: finish this small copy first
            self.stream.synchronize()
        self._next = t

    def __iter__(self):
        return self

    def __next__(self) -> Dict[str, torch.Tensor]:
        if self._next is None:
            self._stage()
        t = self._next
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            t.record_stream(torch.cuda.current_stream(self.device))
        self._stage()   # prefetch the following batch
        return {"input_ids": t[:, :-1], "labels": t[:, :-1]}
