"""Greedy speculative (assisted) decoding with a draft model, device-resident and hipGraph-captured
(reference: src/neuronx_distributed/utils/speculative_decoding.py:40-187 `_standard_assisted_decoding`;
the reference runs the draft/verify/accept loop on the host with a sync per round).

One ROUND = K draft decode steps + one target forward over K+1 tokens + acceptance, all on the
device with static shapes, so `rounds_per_graph` rounds replay from ONE hipGraph launch:

    draft:   [prev, tok] @ [p-1, p]  -> c1      (re-feeding p-1 keeps the draft cache exact
             c1 @ p+1 -> c2 ... c_{K-1} @ p+K-1 -> cK        whether or not all of the previous
                                                             round's candidates were accepted)
    target:  [tok, c1 .. cK] @ [p .. p+K]  -> t0 .. tK       (decode attention over the cache;
                                                             token i sees keys <= p+i)
    accept:  n = #leading i with c_{i+1} == t_i;  emit c1..cn, t_n;  tok <- t_n, p <- p+n+1

Per-sequence n (batched speculation): positions / cache lengths are per-row device tensors, the
kernels take them as inputs.  KV entries written for rejected candidates lie at positions >= the
new p and are overwritten before they become valid.  Output equals the target's own greedy
decode (up to bf16 GEMM nondeterminism).
"""

from __future__ import annotations

from typing import Optional

import torch

from ..ops.decode import argmax_rows
from ..utils.graph_capture import graph_capture

__all__ = ["SpeculativeDecoder", "SpecState", "spec_round"]


class SpecState:
    def __init__(self, batch: int, K: int, cap: int, device):
        self.tok = torch.zeros((batch, 1), dtype=torch.int64, device=device)
        self.prev = torch.zeros((batch, 1), dtype=torch.int64, device=device)
        self.pos = torch.zeros(batch, dtype=torch.int64, device=device)
        self.seq_ids = torch.arange(batch, dtype=torch.int64, device=device)
        self.out = torch.zeros((batch, cap + K + 1), dtype=torch.int64, device=device)
        self.wptr = torch.zeros(batch, dtype=torch.int64, device=device)
        self.accepted = torch.zeros(batch, dtype=torch.int64, device=device)  # total accepted drafts
        self.rounds = torch.zeros(1, dtype=torch.int64, device=device)
        self.batch, self.K, self.cap = batch, K, cap


def _greedy(logits: torch.Tensor) -> torch.Tensor:
    return argmax_rows(logits.reshape(-1, logits.shape[-1])).view(logits.shape[:-1])


def spec_round(target, draft, st: SpecState) -> None:
    """One speculation round for every sequence (graph-capturable: device ops only)."""
    B, K = st.batch, st.K
    dev = st.tok.device
    ar = torch.arange(K + 1, device=dev)
    # ---- draft: K candidates
    d_in = torch.cat([st.prev, st.tok], 1)
    d_pos = torch.stack([st.pos - 1, st.pos], 1)
    lg = draft.forward_tokens(d_in, d_pos, st.seq_ids, (st.pos + 1).to(torch.int32))[:, -1]
    c = [_greedy(lg)]
    for j in range(1, K):
        lg = draft.forward_tokens(c[-1].view(B, 1), (st.pos + j).view(B, 1), st.seq_ids,
                                  (st.pos + j + 1).to(torch.int32))[:, -1]
        c.append(_greedy(lg))
    cand = torch.stack(c, 1)                                   # [B, K]
    # ---- target verifies K+1 positions in one pass
    v_in = torch.cat([st.tok, cand], 1)                        # [B, K+1]
    v_pos = st.pos.view(B, 1) + ar
    t = _greedy(target.forward_tokens(v_in, v_pos, st.seq_ids, (st.pos + K + 1).to(torch.int32)))  # [B, K+1]
    # ---- accept the longest agreeing prefix + the target's next token
    n = torch.cumprod((cand == t[:, :K]).to(torch.int64), 1).sum(1)          # [B]
    emit = torch.cat([cand, torch.zeros_like(cand[:, :1])], 1)
    emit.scatter_(1, n.view(B, 1), t.gather(1, n.view(B, 1)))
    idx = st.wptr.view(B, 1) + ar
    keep = ar.view(1, -1) <= n.view(B, 1)
    st.out.scatter_(1, idx, torch.where(keep, emit, st.out.gather(1, idx)))
    st.prev.copy_(v_in.gather(1, n.view(B, 1)))
    st.tok.copy_(t.gather(1, n.view(B, 1)))
    st.pos.add_(n + 1)
    st.wptr.add_(n + 1)
    st.accepted.add_(n)
    st.rounds.add_(1)


class SpeculativeDecoder:
    """Target + draft `LlamaForCausalLMInference` pair (same vocabulary).  Both KV caches must
    hold max_length + K + 2 positions (the inference app sizes them from speculation_length)."""

    def __init__(self, target, draft, speculation_length: int = 4, rounds_per_graph: int = 4,
                 use_graph: Optional[bool] = None):
        assert speculation_length >= 1
        self.target, self.draft = target, draft
        self.K = int(speculation_length)
        self.rounds_per_graph = max(1, int(rounds_per_graph))
        self.use_graph = target.config.use_hip_graphs if use_graph is None else use_graph
        self._graphs = {}
        self._states = {}
        self.last_stats = {}
        need = target.config.max_length + (self.K + 1) * self.rounds_per_graph + 2
        for m in (target, draft):   # KV caches need room for a whole replay past max_length
            if m.cache_len < need:
                m.cache_len = need
                m.model.setup_kv_cache(m.max_batch, need, m.device)

    def _state(self, B: int) -> SpecState:
        st = self._states.get(B)
        if st is None:
            cap = self.target.config.max_length + (self.K + 1) * self.rounds_per_graph
            st = self._states[B] = SpecState(B, self.K, cap, self.target.device)
        return st

    def _run(self, st: SpecState) -> None:
        for _ in range(self.rounds_per_graph):
            spec_round(self.target.model, self.draft.model, st)

    def _replay(self, st: SpecState) -> None:
        if not (self.use_graph and st.tok.is_cuda):
            self._run(st)
            return
        g = self._graphs.get(st.batch)
        if g is None:
            bufs = (st.tok, st.prev, st.pos, st.out, st.wptr, st.accepted, st.rounds)
            saved = [t.clone() for t in bufs]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._run(st)   # warm-up (GEMM tuning, allocator pools) — writes only discarded slots
            torch.cuda.current_stream().wait_stream(s)
            for t, v in zip(bufs, saved):
                t.copy_(v)
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self._run(st)
            for t, v in zip(bufs, saved):
                t.copy_(v)
            self._graphs[st.batch] = g
        g.replay()

    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                 max_new_tokens: Optional[int] = None, eos_token_id=None, pad_token_id: Optional[int] = None,
                 **unused) -> torch.Tensor:
        tgt, drf = self.target, self.draft
        dev = tgt.device
        B, T = input_ids.shape
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        lengths = attention_mask.to(dev).sum(1)
        limit = tgt.config.max_length - int(lengths.max())
        max_new_tokens = int(min(max_new_tokens if max_new_tokens is not None else limit, limit))
        if eos_token_id is None:
            eos_token_id = getattr(tgt.model_config, "eos_token_id", None)
        eos = torch.tensor(eos_token_id if isinstance(eos_token_id, (list, tuple)) else
                           ([eos_token_id] if eos_token_id is not None else []), device=dev, dtype=torch.int64)
        pad_id = pad_token_id if pad_token_id is not None else (int(eos[0]) if eos.numel() else 0)
        # prefill both models; the target's first token starts the speculation
        logits = tgt._context_encode(input_ids, attention_mask)
        drf._context_encode(input_ids, attention_mask)
        first = argmax_rows(logits)
        st = self._state(B)
        ids = input_ids.to(dev)
        st.tok.copy_(first.view(B, 1))
        st.prev.copy_(ids.gather(1, (lengths - 1).view(B, 1)))
        st.pos.copy_(lengths)
        st.seq_ids.copy_(torch.arange(B, device=dev))
        st.out.zero_()
        st.out[:, 0] = first
        st.wptr.fill_(1)
        st.accepted.zero_()
        st.rounds.zero_()
        # each round emits >= 1 token; stop once every row has max_new_tokens (or hit EOS)
        max_rounds = max(0, max_new_tokens - 1)
        while True:
            w = st.wptr.min()
            if int(w) >= max_new_tokens or int(st.rounds) >= max_rounds:
                break
            if int(st.pos.max()) + (self.K + 1) * self.rounds_per_graph >= tgt.cache_len:
                break
            self._replay(st)
            if eos.numel():
                seen = torch.isin(st.out[:, :int(st.wptr.max())], eos).any(1)
                if bool(seen.all()):
                    break
        out = st.out[:, :max_new_tokens].clone()
        n_out = torch.minimum(st.wptr, torch.full_like(st.wptr, max_new_tokens))
        valid = torch.arange(max_new_tokens, device=dev).view(1, -1) < n_out.view(B, 1)
        out = out.masked_fill(~valid, pad_id)
        if eos.numel():
            hit = torch.isin(out, eos).int()
            out = out.masked_fill((hit.cumsum(1) - hit) > 0, pad_id)
        rounds = max(1, int(st.rounds))
        self.last_stats = {"rounds": rounds, "accepted_per_round": float(st.accepted.float().mean()) / rounds,
                           "tokens_per_round": float((st.wptr - 1).float().mean()) / rounds}
        tgt.kv_cache_populated = drf.kv_cache_populated = False
        return torch.cat([ids, out], 1)
