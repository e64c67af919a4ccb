"""ZeRO-1 optimizer state through torch.distributed.checkpoint (DCP)
(reference: src/neuronx_distributed/optimizer/zero_dcp_utils.py:84-519).

Every flat optimizer buffer (fp32 master / exp_avg / exp_avg_sq of one (param group, kind) on one
(TP, PP) rank) is exposed to DCP as ONE global 1-D ShardedTensor whose local shards are exactly
this DP rank's bucket slices — so `save_optim_state_dict` writes each byte once (no gather) and
`load_optim_state_dict` reads whatever slices the CURRENT layout needs, i.e. loading with a
different DP size re-shards on the fly as long as the bucket plan is identical (same DP-agnostic
padding is not guaranteed across DP sizes: for DP changes use the DP-agnostic "full" format of
optimizer/convert_zero_checkpoints.py; DCP covers same-layout save/load and partial reads).
Keys carry the (TP, PP) coordinates so ranks of different model shards never collide.
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


def _sharded(buf_state, field: str, group) -> Any:
    t = getattr(buf_state, field)
    rank = dist.get_rank()
    shards = []
    for (s, e, lo) in buf_state.local:
        shards.append(Shard(tensor=t[lo:lo + e - s], metadata=ShardMetadata(shard_offsets=[s], shard_sizes=[e - s],
                                                                          placement=f"rank:{rank}/{t.device}")))
    return init_from_local_shards(shards, buf_state.buf.numel, process_group=group)


def _state(optimizer) -> Dict[str, Any]:
    c = _coords()
    sd: Dict[str, Any] = {f"{c}.step": torch.tensor(float(optimizer.step_count))}
    for i, b in enumerate(optimizer.buffers):
        group = b.buf.dp_group if b.buf.dp > 1 else None
        for f in _FIELDS:
            if b.buf.zero1:
                sd[f"{c}.buf{i}.{f}"] = _sharded(b, f, group)
            else:
                sd[f"{c}.buf{i}.{f}.r{dist.get_rank()}"] = getattr(b, f)
    return sd


def save_optim_state_dict(path: str, optimizer, **kwargs) -> None:
    """Collective: every rank writes its own slices under `path` (a directory)."""
    os.makedirs(path, exist_ok=True)
    dcp.save(_state(optimizer), checkpoint_id=path)
    if dist.get_rank() == 0:
        groups = [{k: v for k, v in g.items() if k != "params"} for g in optimizer.param_groups]
        torch.save({"param_groups": groups}, os.path.join(path, "nxd_param_groups.pt"))
    dist.barrier()


def load_optim_state_dict(path: str, optimizer, **kwargs) -> None:
    """Collective: fills every rank's master / moment slices in place, then refreshes the bf16
    parameters from the loaded master weights."""
    sd = _state(optimizer)
    dcp.load(sd, checkpoint_id=path)
    c = _coords()
    optimizer.step_count = int(sd[f"{c}.step"].item())
    meta = torch.load(os.path.join(path, "nxd_param_groups.pt"), weights_only=True)
    for g, sg in zip(optimizer.param_groups, meta["param_groups"]):
        g.update(sg)
    for b in optimizer.buffers:
        for (s, e, lo) in b.local:
            b.buf.param_data[s:e].copy_(b.master[lo:lo + e - s])
        b.buf.gather_params()
