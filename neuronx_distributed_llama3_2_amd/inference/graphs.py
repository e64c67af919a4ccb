"""Device-resident decode loop captured in hipGraphs (MI355X replacement of the reference's
per-bucket compiled token-generation NEFFs + SPMD runtime: trace/model_builder.py:380-451,
trace/spmd.py:32-187).

One graph holds `steps` consecutive decode steps for a fixed batch: forward (all layers, TP
all-reduces included — RCCL kernels capture into the graph), sampling from a pre-drawn uniform
buffer, write of the sampled token into the output ring, and the feed-back of token / position /
cache length for the next step — every update is a device op, so a replay runs `steps` tokens
with ONE host launch and no synchronisation.  The host only checks for EOS between replays.
"""

from __future__ import annotations

import os
from typing import Optional

import torch

from .. import ops
from ..utils.sampling import Sampler
from ..utils.graph_capture import graph_capture

# greedy decoding ends each step with the fused argmax + feed-back launch pair (ops.greedy_advance_)
GREEDY_FUSED = os.environ.get("NXD_GREEDY_FUSED", "1") == "1"


class DecodeState:
    """Static device buffers shared by the captured graphs of one batch size."""

    def __init__(self, batch: int, max_steps: int, device):
        self.tokens = torch.zeros((batch, 1), dtype=torch.int64, device=device)
        self.positions = torch.zeros((batch, 1), dtype=torch.int64, device=device)
        self.cache_len = torch.ones(batch, dtype=torch.int32, device=device)
        # int32: the cache-row index the decode kernels take (no per-step conversion launch)
        self.seq_ids = torch.arange(batch, dtype=torch.int32, device=device)
        self.out = torch.zeros((batch, max_steps), dtype=torch.int64, device=device)
        self.step = torch.zeros(1, dtype=torch.int64, device=device)
        self.uniform = torch.rand((max_steps, batch), dtype=torch.float32, device=device)
        self.argmax_slot = torch.zeros(batch, dtype=torch.int64, device=device)
        self.batch, self.max_steps = batch, max_steps

    def load(self, first_tokens: torch.Tensor, start_positions: torch.Tensor, seq_ids: Optional[torch.Tensor] = None,
             uniform: Optional[torch.Tensor] = None) -> None:
        B = self.batch
        self.tokens.copy_(first_tokens.view(B, 1))
        self.positions.copy_(start_positions.view(B, 1))
        self.cache_len.copy_(start_positions.view(B).to(torch.int32) + 1)
        if seq_ids is not None:
            self.seq_ids.copy_(seq_ids.view(B))
        self.step.zero_()
        if uniform is not None:
            self.uniform.copy_(uniform)
        else:
            self.uniform.uniform_()


def decode_step(model, sampler: Sampler, st: DecodeState) -> None:
    """One token for every sequence; all state lives in `st` (graph-capturable)."""
    B = st.batch
    logits = model.forward_tokens(st.tokens, st.positions, st.seq_ids, st.cache_len)[:, -1]
    if GREEDY_FUSED and sampler.top_k == 1 and not getattr(sampler, "is_medusa", False):
        ops.greedy_advance_(logits, st.argmax_slot, st.out, st.step, st.tokens, st.positions, st.cache_len)
        return
    u = st.uniform.index_select(0, st.step).view(B)
    nxt = sampler.sample(logits, u)
    st.out.scatter_(1, st.step.view(1, 1).expand(B, 1), nxt.view(B, 1))
    st.tokens.copy_(nxt.view(B, 1))
    st.positions.add_(1)
    st.cache_len.add_(1)
    st.step.add_(1)


class DecodeGraph:
    def __init__(self, model, sampler: Sampler, state: DecodeState, steps: int, use_graph: bool = True):
        self.model, self.sampler, self.state, self.steps = model, sampler, state, steps
        self.graph = None
        if use_graph and state.tokens.is_cuda:
            self._capture()

    def _run_eager(self):
        for _ in range(self.steps):
            decode_step(self.model, self.sampler, self.state)

    def _capture(self):
        st = self.state
        saved = [t.clone() for t in (st.tokens, st.positions, st.cache_len, st.step)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._run_eager()  # warm-up: allocator pools, GEMM heuristics, kernel loading
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip((st.tokens, st.positions, st.cache_len, st.step), saved):
            t.copy_(v)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph):
            self._run_eager()
        for t, v in zip((st.tokens, st.positions, st.cache_len, st.step), saved):
            t.copy_(v)

    def replay(self) -> None:
        if self.graph is not None:
            self.graph.replay()
        else:
            self._run_eager()
