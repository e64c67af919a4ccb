"""Training step captured in ONE hipGraph (the reference gets whole-step graphs from the
XLA compiler: one NEFF per training step, trainer/trainer.py + torch_xla mark_step).

`GraphedTrainStep(model, optimizer, loss_fn, example_batch)` runs a few warm-up steps on a side
stream (hipBLASLt autotuning, K-major weight copies, workspace allocations -- everything that must
not happen during capture), restores the model and optimizer to their pre-warm-up state, then
captures: forward + backward of `accum` micro-batches + the optimizer step (flat AdamW with device
step counter / bias corrections / clip coefficient, see FlatMixedPrecisionAdamW.make_capturable).
Each call copies the batch into the static input buffers and replays the graph: one host launch
per step, no host synchronisation.  Worth it when a step is launch-bound (small models, small
per-GPU shards); the Llama-3-8B bench step is GEMM-bound and runs eagerly.

Constraints (checked): every input keeps its shape and dtype; single process or a DP group whose
collectives are RCCL (graph-capturable); the optimizer is a FlatMixedPrecisionAdamW.
"""

from __future__ import annotations

from typing import Callable, List, Sequence

import torch
from .graph_capture import graph_capture


class GraphedTrainStep:
    def __init__(self, model: torch.nn.Module, optimizer, loss_fn: Callable[..., torch.Tensor],
                 example_batches: Sequence[Sequence[torch.Tensor]], warmup: int = 2):
        """loss_fn(model, *micro_batch) -> scalar loss (already divided by the number of micro-batches
        if the caller wants a mean); example_batches: one tuple of tensors per micro-batch."""
        inner = getattr(optimizer, "optimizer", optimizer)
        if not hasattr(inner, "make_capturable"):
            raise TypeError("GraphedTrainStep needs a FlatMixedPrecisionAdamW-based optimizer")
        self.model, self.optimizer, self.inner, self.loss_fn = model, optimizer, inner, loss_fn
        self.static: List[List[torch.Tensor]] = [[t.detach().clone() for t in mb] for mb in example_batches]
        if not all(t.is_cuda for mb in self.static for t in mb):
            raise ValueError("graph capture needs GPU inputs")
        # snapshot: warm-up steps must not change the training state
        snap_params = [b.buf.param_data.clone() for b in inner.buffers]
        snap_state = [(b.master.clone(), b.exp_avg.clone(), b.exp_avg_sq.clone()) for b in inner.buffers]
        snap_step = inner.step_count
        inner.make_capturable()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._restore(snap_params, snap_state, snap_step)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph):
            self.static_loss = self._step()
        torch.cuda.synchronize()
        # capture records without executing, but its host-side bookkeeping (step counter) advanced
        self._restore(snap_params, snap_state, snap_step)
        self.replays = 0

    def _restore(self, params, state, step):
        inner = self.inner
        with torch.no_grad():
            for b, p, (m, ea, eas) in zip(inner.buffers, params, state):
                b.buf.param_data.copy_(p)
                b.master.copy_(m)
                b.exp_avg.copy_(ea)
                b.exp_avg_sq.copy_(eas)
                b.buf.grad_data.zero_()
        inner.step_count = step
        inner._dev_step.fill_(float(step))
        from ..ops.gemm import weights_updated

        weights_updated()

    def _step(self) -> torch.Tensor:
        total = None
        n = len(self.static)
        for i, mb in enumerate(self.static):
            if hasattr(self.optimizer, "set_grad_sync"):
                self.optimizer.set_grad_sync(i == n - 1)
            loss = self.loss_fn(self.model, *mb)
            loss.backward()
            total = loss.detach() if total is None else total + loss.detach()
        self.optimizer.step()
        self.optimizer.zero_grad()
        return total

    def __call__(self, *micro_batches: Sequence[torch.Tensor]) -> torch.Tensor:
        """Copy the micro-batches into the static inputs and replay; returns the summed loss
        (a device tensor overwritten by the next replay)."""
        if len(micro_batches) != len(self.static):
            raise ValueError(f"expected {len(self.static)} micro-batches")
        for dst, src in zip(self.static, micro_batches):
            for d, s_ in zip(dst, src):
                if d.shape != s_.shape or d.dtype != s_.dtype:
                    raise ValueError(f"graphed step input changed: {tuple(s_.shape)} {s_.dtype} vs {tuple(d.shape)} {d.dtype}")
                d.copy_(s_, non_blocking=True)
        self.inner.sync_lr()
        self.graph.replay()
        self.inner.step_count += 1
        self.replays += 1
        return self.static_loss
