"""Medusa tree speculative decoding (reference: src/neuronx_distributed/utils/medusa_utils.py:6-212,
utils/speculative_decoding.py:189-272 `_medusa_assisted_decoding`,
examples/inference/llama3/neuron_modeling_llama.py:345-430 Medusa heads).

Medusa heads: head i predicts the token i+2 steps ahead from the target's final hidden state
(`medusa_head_{i}` = ResBlock(hidden) -> Linear(hidden, vocab); ResBlock(x) = x + SiLU(W x + b)).
A tree of candidate continuations (`medusa_choices`: paths of top-k ranks per head) is verified
in ONE target pass with a tree attention mask (LlamaInferenceModel.forward_tree); the longest
path whose tokens match the target's greedy predictions is accepted, and only that path's K/V is
committed to the KV cache.  Greedy; batch size 1 (as the reference).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.decode import argmax_rows

TOPK = 10  # candidates kept per Medusa head (tree rank indices must be < TOPK)

# a small default tree (paths of per-head top-k ranks); any list of paths works
DEFAULT_MEDUSA_CHOICES: List[List[int]] = [
    [0], [1], [2], [0, 0], [0, 1], [1, 0], [0, 0, 0], [0, 0, 1], [0, 1, 0], [0, 0, 0, 0]]


class ResBlock(nn.Module):
    def __init__(self, hidden_size: int, dtype=None, device=None):
        super().__init__()
        self.linear = nn.Linear(hidden_size, hidden_size, dtype=dtype, device=device)
        nn.init.zeros_(self.linear.weight)   # identity at init (standard Medusa)

    def forward(self, x):
        return x + F.silu(self.linear(x))


class MedusaHeads(nn.Module):
    """`num_heads` Medusa heads; parameter names `medusa_head_{i}.0.linear.*` / `medusa_head_{i}.1.weight`
    as in the reference model."""

    def __init__(self, hidden_size: int, vocab_size: int, num_heads: int, dtype=None, device=None):
        super().__init__()
        self.num_heads = num_heads
        for i in range(num_heads):
            setattr(self, f"medusa_head_{i}", nn.Sequential(
                ResBlock(hidden_size, dtype=dtype, device=device),
                nn.Linear(hidden_size, vocab_size, bias=False, dtype=dtype, device=device)))

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        """h [..., H] -> logits [num_heads, ..., V]."""
        return torch.stack([getattr(self, f"medusa_head_{i}")(h) for i in range(self.num_heads)], 0)


def medusa_tree_buffers(choices: Sequence[Sequence[int]], topk: int = TOPK) -> Dict[str, torch.Tensor]:
    """Static tree description.  Node 0 is the root (the token the target already predicted);
    node j >= 1 is choices sorted by (depth, ranks).  Returns
      attn_mask [N, N] (1 where node j is node i or an ancestor of i),
      tree_indices [N] (index of each node's token in [root, head0 top-k, head1 top-k, ...]),
      position_ids [N] (depth of each node),
      retrieve_indices [R, depth_max + 1] (node indices of every root-to-leaf path, -1 padded)."""
    paths = sorted((tuple(c) for c in choices), key=lambda c: (len(c), c))
    assert all(0 <= r < topk for c in paths for r in c), "tree ranks must be < topk"
    node_of = {(): 0}
    for j, c in enumerate(paths):
        node_of[c] = j + 1
    for c in paths:
        assert c[:-1] in node_of, f"tree path {list(c)} has no parent"
    N = len(paths) + 1
    mask = torch.eye(N)
    mask[:, 0] = 1
    tree_idx = torch.zeros(N, dtype=torch.long)
    depth = torch.zeros(N, dtype=torch.long)
    for c in paths:
        j = node_of[c]
        for a in range(1, len(c)):
            mask[j, node_of[c[:a]]] = 1
        tree_idx[j] = 1 + (len(c) - 1) * topk + c[-1]
        depth[j] = len(c)
    leaves = [c for c in paths if not any(len(o) == len(c) + 1 and o[:len(c)] == c for o in paths)]
    dmax = max((len(c) for c in paths), default=0)
    retrieve = torch.full((len(leaves), dmax + 1), -1, dtype=torch.long)
    for r, c in enumerate(sorted(leaves, key=lambda c: (-len(c), c))):
        retrieve[r, 0] = 0
        for a in range(1, len(c) + 1):
            retrieve[r, a] = node_of[c[:a]]
    return {"attn_mask": mask, "tree_indices": tree_idx, "position_ids": depth, "retrieve_indices": retrieve}


class MedusaDecoder:
    def __init__(self, target, heads: MedusaHeads, choices: Optional[Sequence[Sequence[int]]] = None,
                 topk: int = TOPK):
        self.target, self.heads, self.topk = target, heads, topk
        bufs = medusa_tree_buffers(choices or DEFAULT_MEDUSA_CHOICES, topk)
        dev = target.device
        self.mask = bufs["attn_mask"].to(dev).bool()
        self.tree_idx = bufs["tree_indices"].to(dev)
        self.depth = bufs["position_ids"].to(dev)
        self.retrieve = bufs["retrieve_indices"].to(dev)
        self.last_stats: Dict[str, float] = {}

    def _topk(self, h: torch.Tensor) -> torch.Tensor:
        """final hidden [H] -> [num_heads, topk] candidate tokens."""
        return torch.topk(self.heads(h.view(1, -1)).float().squeeze(1), self.topk, -1).indices

    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, max_new_tokens: int, eos_token_id=None) -> torch.Tensor:
        tgt = self.target
        model = tgt.model
        dev = tgt.device
        assert input_ids.shape[0] == 1, "Medusa decoding runs batch size 1"
        ids = input_ids.to(dev)
        p = ids.shape[1]
        max_new_tokens = min(max_new_tokens, tgt.config.max_length - p)
        tgt.model.reset_kv_cache()
        logits, h = model.forward_tokens(ids, torch.arange(p, device=dev).view(1, p), torch.zeros(1, dtype=torch.long,
                                         device=dev), last_index=torch.tensor([p - 1], device=dev), prefill=True,
                                         return_hidden=True)
        root = argmax_rows(logits.float())[0]
        top = self._topk(h[0])
        out: List[int] = []
        rounds = 0
        eos = set(eos_token_id if isinstance(eos_token_id, (list, tuple)) else
                  ([eos_token_id] if eos_token_id is not None else []))
        ext = torch.full((1,), -1, dtype=torch.long, device=dev)
        while len(out) < max_new_tokens and p + int(self.depth.max()) + 1 < tgt.cache_len:
            flat = torch.cat([root.view(1), top.reshape(-1)])
            tree_tok = flat[self.tree_idx]                                      # [N]
            t_logits, t_h, kvs = model.forward_tree(tree_tok, p + self.depth, self.mask, p)
            pred = argmax_rows(t_logits.float())                                # target's next token per node
            ri = self.retrieve
            cand = torch.cat([tree_tok, ext])[ri]                               # [R, L] (-1 past a leaf)
            path_pred = torch.cat([pred, ext])[ri]
            ok = (cand[:, 1:] == path_pred[:, :-1]) & (cand[:, 1:] >= 0)
            acc = torch.cumprod(ok.long(), 1).sum(1)
            best = int(torch.argmax(acc))
            n = int(acc[best])
            nodes = ri[best, :n + 1]
            toks = cand[best, :n + 1].tolist()
            model.commit_tree_kv(kvs, nodes, p)
            out.extend(toks)
            p += n + 1
            last = int(nodes[-1])
            root = pred[last]
            top = self._topk(t_h[last])
            rounds += 1
            if eos and any(t in eos for t in toks):
                break
        out = out[:max_new_tokens]
        if eos:
            for i, t in enumerate(out):
                if t in eos:
                    out = out[:i + 1]
                    break
        self.last_stats = {"rounds": rounds, "tokens_per_round": len(out) / max(1, rounds)}
        return torch.cat([ids, torch.tensor(out, dtype=torch.long, device=dev).view(1, -1)], 1)
