"""Full <-> tensor-parallel shard conversion driven by the parameters' own parallel attributes
(`tensor_model_parallel`, `partition_dim`, `partition_stride`, `qkv_split`), i.e. the generic
replacement of the reference's per-layer `preshard_hook`s
(src/neuronx_distributed/parallel_layers/layers.py:265-285, modules/qkv_linear.py:609-772,
trace/trace.py:618-649).

* plain TP tensors: the full tensor is split into `tp * stride` chunks along `partition_dim` and
  rank r keeps chunks r, r + tp, ... (interleaved fused projections such as gate_up, stride 2);
* fused GQA QKV (`qkv_split = (q_rows, kv_rows, kv_multiplier)`): K and V are replicated
  `kv_multiplier` times and then split, so rank r holds kv head r % num_kv_heads; Q rows are split
  into tp head groups and, when the kv heads are replicated, rank r receives the group
  `q_group_order(tp, m)[r]` whose heads attend to that kv head (reference
  scripts/checkpoint_converter.py:463-481); the local pieces are concatenated [q | k | v] — the
  layout GQAQKVColumnParallelLinear creates;
* the attention output projection of such a layer (row parallel, `qkv_qgroup_mult = m` on its
  weight) permutes its input-column head groups the same way.
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
        "qgroup_mult": int(getattr(p, "qkv_qgroup_mult", 1) or 1),
    }


def q_group_order(tp: int, mult: int) -> List[int]:
    """Q-head group held by each rank when every kv head is replicated on `mult` ranks
    (num_kv_heads * mult == tp; rank r holds kv head r % (tp // mult)): rank r gets the group whose
    heads belong to that kv head.  Identity without replication."""
    if mult <= 1:
        return list(range(tp))
    if tp % mult:
        raise ValueError(f"kv replication {mult} does not divide the TP degree {tp}")
    nkv = tp // mult
    return [j * mult + i for i in range(mult) for j in range(nkv)]


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
        gq = q_group_order(tp, mult)[rank]
        return torch.cat([q[gq * qp:(gq + 1) * qp], kr[rank * kp:(rank + 1) * kp],
                          vr[rank * kp:(rank + 1) * kp]], dim=0)
    d, s = attrs["dim"], attrs["stride"]
    if attrs.get("qgroup_mult", 1) > 1 and s == 1:
        g = q_group_order(tp, attrs["qgroup_mult"])[rank]
        return torch.chunk(full, tp, dim=d)[g]
    chunks = torch.chunk(full, tp * s, dim=d)
    return torch.cat(chunks[rank::tp], dim=d)


def merge_tensors(shards: List[torch.Tensor], attrs: dict) -> torch.Tensor:
    tp = len(shards)
    if not attrs["tp"] or tp == 1 and attrs["qkv"] is None:
        return shards[0]
    if attrs["qkv"] is not None:
        q_rows, kv_rows, mult = attrs["qkv"]
        qp, kp = q_rows // tp, kv_rows * mult // tp
        order = q_group_order(tp, mult)
        groups = [None] * tp
        for r, sh in enumerate(shards):
            groups[order[r]] = sh[:qp]
        q = torch.cat(groups, dim=0)
        k = torch.cat([s[qp:qp + kp] for s in shards], dim=0)[:kv_rows]
        v = torch.cat([s[qp + kp:] for s in shards], dim=0)[:kv_rows]
        return torch.cat([q, k, v], dim=0)
    d, s = attrs["dim"], attrs["stride"]
    if attrs.get("qgroup_mult", 1) > 1 and s == 1:
        order = q_group_order(tp, attrs["qgroup_mult"])
        groups = [None] * tp
        for r, sh in enumerate(shards):
            groups[order[r]] = sh
        return torch.cat(groups, dim=d)
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
