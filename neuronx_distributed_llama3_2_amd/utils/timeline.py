"""Chrome-trace timeline of named events (reference: src/neuronx_distributed/utils/timeline.py:14-135).

Events are recorded as complete ("ph": "X") Chrome-trace records, one process row per rank.  On a
GPU the start/end of every event can also be stamped with HIP events on the current stream
(`gpu=True`), which measures when the GPU actually ran the work instead of when Python enqueued
it; those are resolved once per step (a single synchronise at `mark_step_end`).
Load the file in chrome://tracing or Perfetto.
"""

from __future__ import annotations

import json
import time
from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import Dict, List, Optional

import torch


class Event:
    __slots__ = ("label", "rank", "start", "end", "gpu_start", "gpu_end")

    def __init__(self, label: str, rank: int, start: float = -1, end: float = -1):
        self.label, self.rank, self.start, self.end = label, rank, start, end
        self.gpu_start = self.gpu_end = None


class Timeline(ABC):
    """mark_event_start(label) / mark_event_end(label) / mark_step_end() — the step end gathers all
    ranks' events and rank 0 appends them to `trace_file_path`."""

    def __init__(self, trace_file_path: Optional[str], rank: int, gpu: bool = False):
        self.enabled = trace_file_path is not None
        self.trace_file_path = trace_file_path
        self.rank = rank
        self.step = 0
        self.gpu = gpu and torch.cuda.is_available()
        self._t0_gpu = None
        self._t0_host = None
        self._clean_states()
        if self.enabled and self.should_record and self.rank == 0:
            with open(self.trace_file_path, "a") as f:
                f.write("[\n")

    @property
    @abstractmethod
    def should_record(self) -> bool:
        ...

    @abstractmethod
    def _collect_events_for_all_ranks(self) -> None:
        ...

    def _clean_states(self):
        self.current_rank_events: Dict[str, Event] = OrderedDict()
        self.all_rank_events: Optional[List[Dict[str, dict]]] = None

    @staticmethod
    def _now_us() -> float:
        return time.time() * 1e6

    def _gpu_event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        if self._t0_gpu is None:
            self._t0_gpu, self._t0_host = e, self._now_us()
        return e

    def mark_event_start(self, label: str) -> None:
        if not (self.enabled and self.should_record):
            return
        assert label not in self.current_rank_events, f"event {label} already started"
        ev = Event(label, self.rank, start=self._now_us())
        if self.gpu:
            ev.gpu_start = self._gpu_event()
        self.current_rank_events[label] = ev

    def mark_event_end(self, label: str) -> None:
        if not (self.enabled and self.should_record):
            return
        ev = self.current_rank_events[label]
        ev.end = self._now_us()
        if self.gpu:
            ev.gpu_end = self._gpu_event()

    def _resolved(self) -> Dict[str, dict]:
        if self.gpu and self._t0_gpu is not None:
            torch.cuda.synchronize()
        out = OrderedDict()
        for label, ev in self.current_rank_events.items():
            assert ev.end >= 0, f"event {label} never ended"
            rec = {"name": label, "pid": ev.rank, "tid": 0, "ts": ev.start, "dur": ev.end - ev.start}
            out[label] = rec
            if ev.gpu_start is not None and ev.gpu_end is not None:
                t0 = self._t0_host + self._t0_gpu.elapsed_time(ev.gpu_start) * 1e3
                out[label + "@gpu"] = {"name": label, "pid": ev.rank, "tid": 1, "ts": t0,
                                       "dur": ev.gpu_start.elapsed_time(ev.gpu_end) * 1e3}
        return out

    def mark_step_end(self) -> None:
        if not (self.enabled and self.should_record):
            return
        self.current_rank_events_resolved = self._resolved()
        self._collect_events_for_all_ranks()
        if self.rank == 0:
            self._dump_events()
        self._clean_states()
        self._t0_gpu = None
        self.step += 1

    def _dump_events(self) -> None:
        with open(self.trace_file_path, "a") as f:
            for events in self.all_rank_events or []:
                for rec in events.values():
                    f.write(json.dumps({"cat": "comp", "ph": "X", "args": {"step": self.step}, **rec}) + ",\n")

    def _create_instant_event(self, label: str, timestamp: float) -> str:
        return json.dumps({"cat": "comp", "ph": "i", "name": label, "ts": timestamp, "tid": self.step,
                           "pid": self.rank, "s": "p"}) + ",\n"


class LocalTimeline(Timeline):
    """Single-process timeline (no gathering)."""

    @property
    def should_record(self) -> bool:
        return self.enabled

    def _collect_events_for_all_ranks(self) -> None:
        self.all_rank_events = [self.current_rank_events_resolved]
