"""Training-side profiling and observability.

The reference traces with a Chrome-trace `Timeline` (utils/timeline.py:14-137, disabled for PP at
pipeline/model.py:302-305), a torch.profiler CPU trace around inference generation
(examples/inference/runner.py:107-120) and reports seq/s throughput.  On MI355X:

* `annotate(name)` — roctx range (torch.cuda.nvtx is backed by roctx on ROCm) + torch.profiler
  `record_function`, so phases show up in both `rocprofv3 --marker-trace` and Kineto traces;
* `profile_steps(step_fn, ...)` — Kineto (CPU + HIP activity) trace of a few steps, exported as a
  Chrome trace plus a per-kernel table;
* `PhaseTimer` — HIP-event timing of named phases (fwd / bwd / optimizer) without a host sync per
  phase; results are read once per report;
* `model_flops_per_token` / `mfu` — dense-transformer training FLOPs (6·N plus causal attention)
  against the bf16 dense MFMA peak, reported by bench.py next to tokens/s.
"""

from __future__ import annotations

import contextlib
import os
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import torch

# dense (no 2:1 sparsity) bf16 MFMA peak of one MI355X, FLOP/s
MI355X_BF16_DENSE_PEAK = 2.5e15


@contextlib.contextmanager
def annotate(name: str):
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:  # pragma: no cover - roctx unavailable in this build
            pass
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


def profile_steps(step_fn: Callable[[], None], steps: int = 3, warmup: int = 1, out_dir: str = "profiles",
                  tag: str = "train", row_limit: int = 40) -> str:
    """Run `warmup + steps` calls of step_fn under torch.profiler; write `<out_dir>/<tag>_trace.json`
    (Chrome trace) and `<out_dir>/<tag>_kernels.txt` (top ops by device time).  Returns the table."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    os.makedirs(out_dir, exist_ok=True)
    sched = torch.profiler.schedule(wait=0, warmup=warmup, active=steps, repeat=1)
    with torch.profiler.profile(activities=acts, schedule=sched, record_shapes=False) as prof:
        for _ in range(warmup + steps):
            step_fn()
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            prof.step()
    prof.export_chrome_trace(os.path.join(out_dir, f"{tag}_trace.json"))
    key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
    table = prof.key_averages().table(sort_by=key, row_limit=row_limit)
    with open(os.path.join(out_dir, f"{tag}_kernels.txt"), "w") as f:
        f.write(table)
    return table


class PhaseTimer:
    """Accumulates wall time of named phases using HIP events (host timer on CPU).

        t = PhaseTimer()
        with t.phase("fwd"): ...
        with t.phase("bwd"): ...
        t.summary()   # {"fwd": ms, "bwd": ms}  (synchronises once)
    """

    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self._gpu = torch.cuda.is_available()
        self._events: Dict[str, List] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self._gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            with annotate(name):
                yield
            e.record()
            self._events[name].append((s, e))
        else:
            import time

            t0 = time.perf_counter()
            yield
            self._events[name].append((t0, time.perf_counter()))

    def summary(self, reset: bool = True) -> Dict[str, float]:
        if self._gpu:
            torch.cuda.synchronize()
            out = {k: sum(s.elapsed_time(e) for s, e in v) for k, v in self._events.items()}
        else:
            out = {k: 1000.0 * sum(e - s for s, e in v) for k, v in self._events.items()}
        if reset:
            self._events.clear()
        return out


def model_flops_per_token(num_params: float, num_layers: int, hidden: int, seq_len: int, causal: bool = True) -> float:
    """Training FLOPs per token: 6·N for the weight GEMMs (fwd + 2x bwd) plus attention scores and
    PV, 12·L·H·S for full attention (fwd 4·L·H·S, bwd 8·L·H·S), halved for causal masking."""
    attn = 12.0 * num_layers * hidden * seq_len * (0.5 if causal else 1.0)
    return 6.0 * num_params + attn


def mfu(tokens_per_s: float, flops_per_token: float, n_gpus: int, peak: float = MI355X_BF16_DENSE_PEAK) -> float:
    return tokens_per_s * flops_per_token / (n_gpus * peak)


def llama_num_params(cfg) -> int:
    """Parameter count of a Llama-architecture config (untied embeddings unless tie_word_embeddings)."""
    h, L, v = cfg.hidden_size, cfg.num_hidden_layers, cfg.vocab_size
    nh = cfg.num_attention_heads
    kvh = getattr(cfg, "num_key_value_heads", nh) or nh
    hd = getattr(cfg, "head_dim", None) or h // nh
    inter = cfg.intermediate_size
    attn = h * nh * hd + 2 * h * kvh * hd + nh * hd * h
    mlp = 3 * h * inter
    per_layer = attn + mlp + 2 * h
    emb = v * h * (1 if getattr(cfg, "tie_word_embeddings", False) else 2)
    return L * per_layer + emb + h
