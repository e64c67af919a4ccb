"""Pipeline timeline: one Chrome-trace row per pipeline stage
(reference: src/neuronx_distributed/pipeline/timeline.py:10-24)."""

from __future__ import annotations

from ..parallel_layers.parallel_state import (
    gather_python_object,
    get_data_parallel_rank,
    get_pp_gloo_group,
    get_tensor_model_parallel_rank,
)
from ..utils.timeline import Timeline


class PPTimeline(Timeline):
    def __init__(self, trace_file_path, pp_rank, gpu: bool = False):
        super().__init__(trace_file_path, pp_rank, gpu=gpu)
        self.group = get_pp_gloo_group() if self.enabled else None

    @property
    def should_record(self) -> bool:
        # one row per stage: only the DP=0, TP=0 member of each pipeline records
        return self.enabled and get_data_parallel_rank() == 0 and get_tensor_model_parallel_rank() == 0

    def _collect_events_for_all_ranks(self) -> None:
        self.all_rank_events = gather_python_object(self.current_rank_events_resolved, group=self.group)
