"""ZeRO-1 optimizer state through torch.distributed.checkpoint (DCP)
(reference: src/neuronx_distributed/optimizer/zero_dcp_utils.py:84-519).

Like the reference (`_tensor_to_sharded_tensor`, :84-140), every parameter's fp32 master / exp_avg /
exp_avg_sq is exposed to DCP as one ShardedTensor of the parameter's GLOBAL shape, row-sharded
along dim 0 over the data-parallel group (DP rank r owns rows [r c, (r + 1) c), c = ceil(rows /
DP): the torch_xla ZeRO shard without its padding).  Save writes each row once; load describes the
rows the CURRENT DP layout needs, so a checkpoint saved at one DP size loads at any other (DCP
re-slices), then the per-parameter rows are turned back into the flat ZeRO-1 buffer slices
(optimizer/zero_layout.py, one all-gather per bucket).  Keys carry the (TP, PP) coordinates
(`tpXX_ppXX.pN.field`, the reference's `|pp-XXXX|tp-XXXX` fqn suffix, :196-209) so ranks of
different model shards never collide; the step and param-group hyper-parameters are plain entries.
"""

from __future__ import annotations

import os
from typing import Any, Dict

import torch
import torch.distributed as dist
import torch.distributed.checkpoint as dcp
from torch.distributed._shard.sharded_tensor import Shard, ShardMetadata, init_from_local_shards

from ..parallel_layers import parallel_state as ps

_FIELDS = ("master", "exp_avg", "exp_avg_sq")


def _coords() -> str:
    if ps.model_parallel_is_initialized():
        return f"tp{ps.get_tensor_model_parallel_rank():02d}_pp{ps.get_pipeline_model_parallel_rank():02d}"
    return "tp00_pp00"


def _rows(d0: int, dp: int, r: int):
    c = -(-d0 // dp)
    return min(r * c, d0), min((r + 1) * c, d0)


def _sharded_param(t: torch.Tensor, shape, dp: int, r: int, group) -> Any:
    """ShardedTensor of global `shape` whose local shard is rows _rows(...) of `t` (full tensor)."""
    lo, hi = _rows(shape[0], dp, r)
    shards = []
    if hi > lo:
        off = [lo] + [0] * (len(shape) - 1)
        size = [hi - lo] + list(shape[1:])
        shards.append(Shard(tensor=t[lo:hi].contiguous(),
                            metadata=ShardMetadata(shard_offsets=off, shard_sizes=size,
                                                   placement=f"rank:{dist.get_rank()}/{t.device}")))
    return init_from_local_shards(shards, *shape, process_group=group)


def _group(b):
    return b.buf.dp_group if b.buf.dp > 1 else None


def _save_state(optimizer) -> Dict[str, Any]:
    from .zero_layout import full_states, param_entries

    c = _coords()
    sd: Dict[str, Any] = {f"{c}.step": torch.tensor(float(optimizer.step_count))}
    index = {id(p): i for (i, _, p, _) in param_entries(optimizer)}
    for b in optimizer.buffers:
        for p, full in full_states(b):
            i = index[id(p)]
            for f in _FIELDS:
                sd[f"{c}.p{i}.{f}"] = _sharded_param(full[f], tuple(full[f].shape), b.buf.dp, b.buf.dp_rank, _group(b))
    return sd


def save_optim_state_dict(path: str, optimizer, **kwargs) -> None:
    """Collective: every rank writes its own parameter rows under `path` (a directory)."""
    os.makedirs(path, exist_ok=True)
    dcp.save(_save_state(optimizer), checkpoint_id=path)
    if dist.get_rank() == 0:
        groups = [{k: v for k, v in g.items() if k != "params"} for g in optimizer.param_groups]
        torch.save({"param_groups": groups}, os.path.join(path, "nxd_param_groups.pt"))
    dist.barrier()


def load_optim_state_dict(path: str, optimizer, **kwargs) -> None:
    """Collective: reads the rows this rank's CURRENT DP layout owns (any DP size at save time),
    rebuilds the flat ZeRO-1 slices and refreshes the bf16 parameters from the loaded master."""
    from .zero_layout import load_full_states, param_entries

    c = _coords()
    entries = param_entries(optimizer)
    sd: Dict[str, Any] = {f"{c}.step": torch.tensor(0.0)}
    for (i, _, p, b) in entries:
        shape = tuple(p.shape) if p.dim() > 0 else (1,)
        for f in _FIELDS:
            buf = torch.zeros(shape, dtype=torch.float32, device=b.master.device)
            sd[f"{c}.p{i}.{f}"] = _sharded_param(buf, shape, b.buf.dp, b.buf.dp_rank, _group(b))
    dcp.load(sd, checkpoint_id=path)
    optimizer.step_count = int(sd[f"{c}.step"].item())
    meta = torch.load(os.path.join(path, "nxd_param_groups.pt"), weights_only=True)
    for g, sg in zip(optimizer.param_groups, meta["param_groups"]):
        g.update(sg)
    by_buf: Dict[int, Dict[int, Dict[str, torch.Tensor]]] = {}
    for (i, _, p, b) in entries:
        shape = tuple(p.shape) if p.dim() > 0 else (1,)
        rows = {}
        for f in _FIELDS:
            st = sd[f"{c}.p{i}.{f}"]
            lo, hi = _rows(shape[0], b.buf.dp, b.buf.dp_rank)
            padded = torch.zeros((-(-shape[0] // b.buf.dp),) + shape[1:], dtype=torch.float32, device=b.master.device)
            if hi > lo:
                padded[:hi - lo].copy_(st.local_shards()[0].tensor)
            rows[f] = padded
        by_buf.setdefault(id(b), {})[id(p)] = rows
    for b in optimizer.buffers:
        load_full_states(b, by_buf.get(id(b), {}), sharded=True)
    optimizer._after_load()
