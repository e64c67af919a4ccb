"""Full <-> tensor-parallel shard conversion driven by the parameters' own parallel attributes
(`tensor_model_parallel`, `partition_dim`, `partition_stride`, `qkv_split`), i.e. the generic
replacement of the reference's per-layer `preshard_hook`s
(src/neuronx_distributed/parallel_layers/layers.py:265-285, modules/qkv_linear.py:609-772,
trace/trace.py:618-649).

* plain TP tensors: the full tensor is split into `tp * stride` chunks along `partition_dim` and
  rank r keeps chunks r, r + tp, ... (interleaved fused projections such as gate_up, stride 2);
* fused GQA QKV (`qkv_split = (q_rows, kv_rows, kv_multiplier)`): Q rows are split contiguously,
  K and V are first replicated `kv_multiplier` times and then split, and the three local pieces
  are concatenated [q | k | v] — the same layout GQAQKVColumnParallelLinear creates.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Mapping, Optional

import torch


def _attrs(p) -> dict:
    return {
        "tp": bool(getattr(p, "tensor_model_parallel", False)),
        "dim": int(getattr(p, "partition_dim", 0) or 0),
        "stride": int(getattr(p, "partition_stride", 1) or 1),
        "qkv": getattr(p, "qkv_split", None),
    }


def shard_tensor(full: torch.Tensor, attrs: dict, tp: int, rank: int) -> torch.Tensor:
    if not attrs["tp"] or tp == 1 and attrs["qkv"] is None:
        return full
    if attrs["qkv"] is not None:
        q_rows, kv_rows, mult = attrs["qkv"]
        q, k, v = torch.split(full, [q_rows, kv_rows, kv_rows], dim=0)
        qp = q.shape[0] // tp
        kr = torch.cat([k] * mult, dim=0)
        vr = torch.cat([v] * mult, dim=0)
        kp = kr.shape[0] // tp
        return torch.cat([q[rank * qp:(rank + 1) * qp], kr[rank * kp:(rank + 1) * kp],
                          vr[rank * kp:(rank + 1) * kp]], dim=0)
    d, s = attrs["dim"], attrs["stride"]
    chunks = torch.chunk(full, tp * s, dim=d)
    return torch.cat(chunks[rank::tp], dim=d)


def merge_tensors(shards: List[torch.Tensor], attrs: dict) -> torch.Tensor:
    tp = len(shards)
    if not attrs["tp"] or tp == 1 and attrs["qkv"] is None:
        return shards[0]
    if attrs["qkv"] is not None:
        q_rows, kv_rows, mult = attrs["qkv"]
        qp, kp = q_rows // tp, kv_rows * mult // tp
        q = torch.cat([s[:qp] for s in shards], dim=0)
        k = torch.cat([s[qp:qp + kp] for s in shards], dim=0)[:kv_rows]
        v = torch.cat([s[qp + kp:] for s in shards], dim=0)[:kv_rows]
        return torch.cat([q, k, v], dim=0)
    d, s = attrs["dim"], attrs["stride"]
    pieces = [torch.chunk(sh, s, dim=d) for sh in shards]   # pieces[r][j] = chunk j*tp + r
    ordered = [pieces[r][j] for j in range(s) for r in range(tp)]
    return torch.cat(ordered, dim=d)


def shard_state_dict(model: torch.nn.Module, full_sd: Mapping[str, torch.Tensor], tp: int, rank: int,
                     strict: bool = True) -> Dict[str, torch.Tensor]:
    """Local shard (for `rank` of `tp`) of a full (unsharded) state dict, using `model`'s parameter
    attributes (model may live on the meta device)."""
    out = {}
    params = dict(model.named_parameters(remove_duplicate=False))
    for name, p in params.items():
        if name not in full_sd:
            if strict:
                raise KeyError(f"{name} missing from the full state dict")
            continue
        out[name] = shard_tensor(full_sd[name], _attrs(p), tp, rank).contiguous()
    for name, b in model.named_buffers():
        if name in full_sd:
            out[name] = full_sd[name]
    return out


def merge_state_dicts(model: torch.nn.Module, shard_sds: List[Mapping[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    """Full state dict from per-rank TP shards (inverse of shard_state_dict)."""
    out = {}
    params = dict(model.named_parameters(remove_duplicate=False))
    for name in shard_sds[0]:
        p = params.get(name)
        if p is None:
            out[name] = shard_sds[0][name]
            continue
        out[name] = merge_tensors([sd[name] for sd in shard_sds], _attrs(p))
    return out
