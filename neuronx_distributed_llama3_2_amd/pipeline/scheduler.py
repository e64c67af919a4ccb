"""Pipeline schedules as pure generators of per-step task lists.

Public task / schedule names follow the reference (src/neuronx_distributed/pipeline/scheduler.py:4-541)
and the generated sequences are the same (1F1B: warmup forwards, steady one-forward-one-backward,
cooldown backwards, then ReduceGradsTask; interleaved: Megatron virtual-pipeline order with the
last stage sending before receiving), so a schedule can be inspected and unit-tested without any
process group.  The MI355X runtime (pipeline/model.py) executes the compute tasks in this order and
groups each step's sends/receives into one RCCL `batch_isend_irecv` so adjacent stages never
deadlock on point-to-point ordering.
"""

from __future__ import annotations

from typing import Iterator, List


class PipelineTask:
    def __init__(self, mb: int, model_chunk: int = 0, graph_break: bool = True):
        self.mb = mb
        self.model_chunk = model_chunk
        self.graph_break = graph_break

    def __eq__(self, other) -> bool:
        return (type(self) is type(other) and self.mb == other.mb and self.model_chunk == other.model_chunk
                and self.graph_break == other.graph_break)

    def __hash__(self):
        return hash((type(self).__name__, self.mb, self.model_chunk))

    def __repr__(self):
        return (f"{type(self).__name__}_microbatch_{self.mb}_modelchunk_{self.model_chunk}"
                f"_graphbreak_{self.graph_break}")


class ForwardStepTask(PipelineTask):
    pass


class ForwardPreprocessTask(PipelineTask):
    """receive this micro-batch's activations from the previous stage"""


class ForwardPostprocessTask(PipelineTask):
    """send this micro-batch's activations to the next stage"""


class BackwardStepTask(PipelineTask):
    pass


class BackwardPreprocessTask(PipelineTask):
    """receive this micro-batch's output gradients from the next stage"""


class BackwardPostprocessTask(PipelineTask):
    """send this micro-batch's input gradients to the previous stage"""


class PostProcessTask:
    def __init__(self, graph_break: bool = True):
        self.mb = -1
        self.model_chunk = -1
        self.graph_break = graph_break


class ReduceGradsTask(PostProcessTask):
    def __repr__(self):
        return "ReduceGradsTask"

    def __eq__(self, other) -> bool:
        return type(self) is type(other)

    def __hash__(self):
        return hash("ReduceGradsTask")


class PipeSchedule:
    def __init__(self, num_microbatches: int, stages: int, stage_id: int):
        self.num_microbatches = num_microbatches
        self.stages = stages
        self.stage_id = stage_id
        self.prev_stage = stage_id - 1
        self.next_stage = stage_id + 1

    def steps(self) -> Iterator[List[PipelineTask]]:
        raise NotImplementedError

    def _valid_micro_batch(self, mb: int) -> bool:
        return 0 <= mb < self.num_microbatches

    def _valid_stage(self, s: int) -> bool:
        return 0 <= s < self.stages

    @property
    def stage(self):
        return self.stage_id

    @property
    def num_stages(self):
        return self.stages

    @property
    def is_first_stage(self):
        return self.stage_id == 0

    @property
    def is_last_stage(self):
        return self.stage_id == self.stages - 1

    def __iter__(self):
        return iter(self.steps())


class InferenceSchedule(PipeSchedule):
    """Fill-drain forward only."""

    def steps(self):
        for mb in range(self.num_microbatches):
            yield [ForwardPreprocessTask(mb), ForwardStepTask(mb), ForwardPostprocessTask(mb)]


class Train1F1BSchedule(PipeSchedule):
    """Non-interleaved 1F1B:  warmup = stages - stage - 1 forwards, then alternating F/B, then the
    remaining backwards, then a ReduceGradsTask.  In the steady state the backward receive of a
    step is ordered before the forward send of the previous micro-batch (deadlock-free)."""

    def __init__(self, num_microbatches: int, stages: int, stage_id: int):
        super().__init__(num_microbatches, stages, stage_id)
        self.num_warmup_steps = min(stages - stage_id - 1, num_microbatches)
        self.num_steady_state_microbatches = num_microbatches - self.num_warmup_steps
        self.num_remaining_microbatches = self.num_warmup_steps

    def _step_to_micro_batch(self, step: int):
        w = self.num_warmup_steps
        s = self.num_steady_state_microbatches
        if step < w:
            return step, True
        if step < w + 2 * s:
            k = step - w
            return (k // 2 + w, True) if k % 2 == 0 else (k // 2, False)
        return s + (step - w - 2 * s), False

    def steps(self):
        total = 2 * self.num_microbatches
        prev_mb = -1
        has_next = self._valid_stage(self.next_stage)
        has_prev = self._valid_stage(self.prev_stage)
        for step in range(total):
            mb, fwd = self._step_to_micro_batch(step)
            cmds: List[PipelineTask] = []
            if fwd:
                cmds.append(ForwardPreprocessTask(mb))
                cmds.append(ForwardStepTask(mb))
                if mb < self.num_warmup_steps and has_next:
                    cmds.append(ForwardPostprocessTask(mb))
            else:
                if has_next:
                    cmds.append(BackwardPreprocessTask(mb))
                    if mb < self.num_steady_state_microbatches:
                        cmds.append(ForwardPostprocessTask(prev_mb))
                cmds.append(BackwardStepTask(mb))
                if has_prev:
                    cmds.append(BackwardPostprocessTask(mb))
            prev_mb = mb
            yield cmds
        yield [ReduceGradsTask()]


class TrainInterleavedSchedule(PipeSchedule):
    """Virtual-pipeline (interleaved) schedule: each stage holds `num_model_chunks` chunks; chunk c of
    stage s is virtual stage c * stages + s.  Micro-batches advance in groups of `stages`."""

    def __init__(self, num_microbatches: int, num_model_chunks: int, stages: int, stage_id: int,
                 fused_send_recv: bool = False, fused_fwd_bwd: bool = False, use_odd_even_scheduler: bool = False):
        super().__init__(num_microbatches, stages, stage_id)
        if num_microbatches % stages != 0:
            raise ValueError(
                f"Interleaved pipeline requires num_microbatches % pipeline_parallel_size == 0, current "
                f"num_microbatches {num_microbatches} and pipeline_parallel_size {stages}")
        if num_microbatches <= stages:
            fused_send_recv = fused_fwd_bwd = False
        self.num_model_chunks = num_model_chunks
        self.fused_send_recv = fused_send_recv
        self.fused_fwd_bwd = fused_fwd_bwd
        self.use_odd_even_scheduler = use_odd_even_scheduler
        self.num_microbatches_steps = num_microbatches * num_model_chunks
        if num_microbatches == stages:
            self.num_warmup_steps = self.num_microbatches_steps
        else:
            w = 2 * (stages - stage_id - 1) + (num_model_chunks - 1) * stages
            self.num_warmup_steps = min(w, self.num_microbatches_steps)
        self.num_steady_state_steps = self.num_microbatches_steps - self.num_warmup_steps
        self.num_remaining_steps = self.num_warmup_steps

    def get_model_chunk_id(self, step: int, is_forward: bool = True) -> int:
        if not is_forward:
            step -= self.num_warmup_steps
        group = self.stages * self.num_model_chunks
        chunk = (step % group) // self.stages
        return chunk if is_forward else self.num_model_chunks - 1 - chunk

    def get_microbatch_id(self, step: int, is_forward: bool = True) -> int:
        if not is_forward:
            step -= self.num_warmup_steps
        group = self.stages * self.num_model_chunks
        return self.stages * (step // group) + (step % group) % self.stages

    def _recv_fwd_send_bwd(self, step, is_forward=True):
        if is_forward:
            step += 1
        return not (self.stage_id == 0 and self.get_model_chunk_id(step, is_forward) == 0)

    def _recv_bwd_send_fwd(self, step, is_forward=True):
        if not is_forward:
            step += 1
        return not (self.stage_id == self.stages - 1 and
                    self.get_model_chunk_id(step, is_forward) == self.num_model_chunks - 1)

    def _task(self, cls, step, is_forward, gb=True):
        return cls(self.get_microbatch_id(step, is_forward), model_chunk=self.get_model_chunk_id(step, is_forward),
                   graph_break=gb)

    def _comm(self, step, cmds, fwd_pre, fwd_post, bwd_pre, bwd_post):
        fp = lambda: self._task(ForwardPreprocessTask, step + 1, True, not self.fused_send_recv or not bwd_post)  # noqa
        fo = lambda: self._task(ForwardPostprocessTask, step, True, not self.fused_send_recv or not bwd_pre)  # noqa
        bp = lambda: self._task(BackwardPreprocessTask, step + 1, False)  # noqa
        bo = lambda: self._task(BackwardPostprocessTask, step, False)  # noqa
        if self.use_odd_even_scheduler:
            order = [(fwd_pre, fp), (fwd_post, fo), (bwd_post, bo), (bwd_pre, bp)] if self.stage_id % 2 == 0 else \
                [(fwd_post, fo), (fwd_pre, fp), (bwd_pre, bp), (bwd_post, bo)]
        elif self.stage_id != self.stages - 1:
            order = [(fwd_pre, fp), (bwd_post, bo), (fwd_post, fo), (bwd_pre, bp)]
        else:  # last stage sends before it receives
            order = [(fwd_post, fo), (bwd_pre, bp), (fwd_pre, fp), (bwd_post, bo)]
        cmds.extend(make() for cond, make in order if cond)

    def steps(self):
        w, s = self.num_warmup_steps, self.num_steady_state_steps
        total = w + s + self.num_remaining_steps + 1
        for step in range(total):
            cmds: List[PipelineTask] = []
            if step == total - 1:
                yield [ReduceGradsTask()]
                return
            if step < w:
                if step == 0:
                    cmds.append(self._task(ForwardPreprocessTask, 0, True))
                cmds.append(self._task(ForwardStepTask, step, True))
                self._comm(step, cmds, fwd_pre=step != self.num_microbatches_steps - 1,
                           fwd_post=self._recv_bwd_send_fwd(step, True),
                           bwd_pre=step == w - 1 and self._recv_bwd_send_fwd(step, False), bwd_post=False)
            elif step < w + s:
                cmds.append(self._task(ForwardStepTask, step, True, not self.fused_fwd_bwd))
                cmds.append(self._task(BackwardStepTask, step, False))
                self._comm(step, cmds, fwd_pre=step != w + s - 1, fwd_post=self._recv_bwd_send_fwd(step, True),
                           bwd_pre=self._recv_bwd_send_fwd(step, False), bwd_post=self._recv_fwd_send_bwd(step, False))
            else:
                cmds.append(self._task(BackwardStepTask, step, False))
                self._comm(step, cmds, fwd_pre=False, fwd_post=False,
                           bwd_pre=step != total - 2 and self._recv_bwd_send_fwd(step, False),
                           bwd_post=self._recv_fwd_send_bwd(step, False))
            yield cmds


TrainSchedule = Train1F1BSchedule
