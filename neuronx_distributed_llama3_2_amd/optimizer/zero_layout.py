"""Per-parameter optimizer-state layouts of the flat optimizers (reference checkpoint format).

The flat optimizers keep fp32 master weights and Adam moments in flat buffers, ZeRO-1-sharded in
contiguous bucket slices.  The reference's ZeRO-1 (torch_xla ZeroRedundancyOptimizer, wrapped by
src/neuronx_distributed/optimizer/zero_redundancy_optimizer.py:29-155 and re-sharded by
optimizer/convert_zero_checkpoints.py:54-144) shards EACH PARAMETER along dim 0 instead: the
parameter is zero-padded to a multiple of the DP size and DP rank r keeps chunk r.  Its state dict:

    {"state": {},                                   # the wrapper's own (empty) state
     "param_groups": [{...hyper-parameters..., "params": [i, ...]}],
     "base_state": {i: {"step": tensor, "exp_avg": shard, "exp_avg_sq": shard}},
     "shape_info": {i: torch.Size},
     "sharded_master_weights": {i: shard}}          # fp32 master (the reference's save_master_weights)

with i running over the trainable parameters in param-group order.  Without ZeRO-1 the plain torch
layout {"state": {i: {"step", "exp_avg", "exp_avg_sq"}}, "param_groups": [...]} plus
"master_weights": {i: fp32 tensor}.

Converting between the two needs the other DP ranks' slices of each bucket: `full_states` all-gathers
one bucket at a time over the buffer's DP group (a few hundred MB of transient device memory at the
default bucket size), `load_full_states` does the inverse from per-parameter rows.  Both are
collective over every buffer's DP group (all DP ranks call state_dict / load_state_dict together,
as they do through save_checkpoint / load_checkpoint).
"""

from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F

_KEYS = ("master", "exp_avg", "exp_avg_sq")


def _shape(p) -> torch.Size:
    return p.shape if p.dim() > 0 else torch.Size([1])


def param_entries(opt, buffers=None) -> List[Tuple[int, int, Any, Any]]:
    """(index, group index, param, buffer state) of every trainable parameter of `buffers` (default:
    all of the optimizer's), indexed in param-group order as torch_xla's get_shape_info does."""
    buffers = opt.buffers if buffers is None else buffers
    owner = {}
    for b in buffers:
        for p in b.buf.params:
            owner[id(p)] = b
    out, i = [], 0
    for gi, g in enumerate(opt.param_groups):
        for p in g["params"]:
            b = owner.get(id(p))
            if b is None:
                continue
            out.append((i, gi, p, b))
            i += 1
    return out


def _zero1(b) -> bool:
    """Buffer sharded in bucket slices (ZeRO-1 at DP > 1; FlatBuffer keeps DP = 1 whole)."""
    return bool(b.buf.zero1)


def _gather(b) -> bool:
    return bool(b.buf.zero1) and b.buf.dp > 1


def _local_bucket(b, bk, key: str) -> torch.Tensor:
    """This rank's slice of bucket `bk` of state `key` (a view into the flat state)."""
    t = getattr(b, key)
    for (s, e, lo) in b.local:
        if bk.start <= s < bk.end:
            return t[lo:lo + e - s]
    raise RuntimeError("bucket slice not found")


def _buckets(b):
    if _zero1(b):
        return b.buf.buckets
    return [_WholeBuffer(b.buf)]


class _WholeBuffer:
    def __init__(self, buf):
        self.start, self.end, self.params = 0, buf.numel, buf.params


def full_states(b) -> Iterator[Tuple[Any, Dict[str, torch.Tensor]]]:
    """(param, {master, exp_avg, exp_avg_sq: full fp32 tensor of the param's shape}) for every
    parameter of buffer state `b`, one bucket gathered at a time (collective over the DP group)."""
    for bk in _buckets(b):
        if _gather(b):
            full = {}
            for k in _KEYS:
                loc = _local_bucket(b, bk, k)
                g = torch.empty(loc.numel() * b.buf.dp, dtype=loc.dtype, device=loc.device)
                dist.all_gather_into_tensor(g, loc.contiguous(), group=b.buf.dp_group)
                full[k] = g
        elif _zero1(b):   # DP = 1: this rank's bucket slice is the whole bucket
            full = {k: _local_bucket(b, bk, k) for k in _KEYS}
        else:
            full = {k: getattr(b, k) for k in _KEYS}   # _WholeBuffer: start 0
        for p in bk.params:
            off, n = b.buf.offsets[id(p)]
            yield p, {k: full[k][off - bk.start:off - bk.start + n].view(_shape(p)) for k in _KEYS}


def dim0_shard(t: torch.Tensor, dp: int, rank: int) -> torch.Tensor:
    """torch_xla ZeRO shard: pad dim 0 to a multiple of dp, keep chunk `rank`."""
    if t.size(0) % dp:
        t = F.pad(t, [0, 0] * (t.dim() - 1) + [0, dp - t.size(0) % dp])
    return t.chunk(dp)[rank]


def load_full_states(b, rows: Dict[int, Dict[str, torch.Tensor]], sharded: bool) -> None:
    """Inverse of full_states: `rows[id(param)]` holds, per state key, either the full tensor
    (`sharded=False`) or this DP rank's padded dim-0 shard (`sharded=True`, gathered here over the DP
    group); fills this rank's slices of the flat master / moments."""
    for bk in _buckets(b):
        ps_ = [p for p in bk.params if id(p) in rows]
        if len(ps_) != len(bk.params):
            missing = len(bk.params) - len(ps_)
            raise KeyError(f"optimizer state missing for {missing} parameter(s) of buffer {b.buf.name}")
        for k in _KEYS:
            dev = getattr(b, k).device
            if sharded and b.buf.dp > 1:
                local = torch.cat([rows[id(p)][k].reshape(-1).to(dev, torch.float32) for p in ps_])
                g = torch.empty(local.numel() * b.buf.dp, dtype=torch.float32, device=dev)
                dist.all_gather_into_tensor(g, local.contiguous(), group=b.buf.dp_group)
                per_rank = g.view(b.buf.dp, -1)
            full_bucket = torch.zeros(bk.end - bk.start, dtype=torch.float32, device=dev)
            cur = 0
            for p in ps_:
                off, n = b.buf.offsets[id(p)]
                shp = _shape(p)
                if sharded and b.buf.dp > 1:
                    rows_per = -(-shp[0] // b.buf.dp)
                    m = rows_per * (n // shp[0] if shp[0] else 0)
                    full = per_rank[:, cur:cur + m].reshape(b.buf.dp * rows_per, *shp[1:])[:shp[0]]
                    cur += m
                else:
                    full = rows[id(p)][k].to(dev, torch.float32).reshape(shp)
                full_bucket[off - bk.start:off - bk.start + n].copy_(full.reshape(-1))
            if _zero1(b):
                _local_bucket(b, bk, k).copy_(_local_slice(b, bk, full_bucket))
            else:
                getattr(b, k)[bk.start:bk.end].copy_(full_bucket)


def _local_slice(b, bk, full_bucket: torch.Tensor) -> torch.Tensor:
    n = (bk.end - bk.start) // b.buf.dp
    r = b.buf.dp_rank
    return full_bucket[r * n:(r + 1) * n]


def reference_state_dict(opt, buffers=None, step: Optional[int] = None) -> Dict[str, Any]:
    """torch_xla ZeRO-1 layout (zero1 buffers) or plain torch layout (no ZeRO-1) of `buffers`."""
    entries = param_entries(opt, buffers)
    by_param = {id(p): (i, gi, b) for (i, gi, p, b) in entries}
    step_t = torch.tensor(float(opt.step_count if step is None else step))
    zero = bool(getattr(opt, "zero1", False))   # the torch_xla layout also at DP = 1 (whole shards)
    base, shapes, masters, plain = {}, {}, {}, {}
    seen = []
    for b in (opt.buffers if buffers is None else buffers):
        if b in seen:
            continue
        seen.append(b)
        for p, full in full_states(b):
            i = by_param[id(p)][0]
            shapes[i] = _shape(p)
            if zero:
                dp, r = b.buf.dp, b.buf.dp_rank
                sh = {k: dim0_shard(full[k], dp, r).detach().cpu().clone() for k in _KEYS}
                base[i] = {"step": step_t.clone(), "exp_avg": sh["exp_avg"], "exp_avg_sq": sh["exp_avg_sq"]}
                masters[i] = sh["master"]
            else:
                plain[i] = {"step": step_t.clone(), "exp_avg": full["exp_avg"].detach().cpu().clone(),
                            "exp_avg_sq": full["exp_avg_sq"].detach().cpu().clone()}
                masters[i] = full["master"].detach().cpu().clone()
    groups = []
    for gi, g in enumerate(opt.param_groups):
        d = {k: v for k, v in g.items() if k != "params"}
        d["params"] = [i for (i, ggi, _, _) in entries if ggi == gi]
        groups.append(d)
    if zero:
        return {"state": {}, "param_groups": groups, "base_state": base, "shape_info": shapes,
                "sharded_master_weights": masters}
    return {"state": plain, "param_groups": groups, "master_weights": masters}


def is_reference_layout(sd: Dict[str, Any]) -> bool:
    return isinstance(sd, dict) and "param_groups" in sd and ("base_state" in sd or (
        "state" in sd and not sd.get("flat_optimizer") and not sd.get("flat_optimizer_full")))


def load_reference_state_dict(opt, sd: Dict[str, Any], buffers=None) -> int:
    """Load a reference-layout state dict into `buffers` (default all); returns the step.  Master
    weights come from `sharded_master_weights` / `master_weights` when present, else from the
    current (bf16) parameters, as torch_xla's ZeRO does without save_master_weights."""
    entries = param_entries(opt, buffers)
    zero = "base_state" in sd
    per_idx = sd["base_state"] if zero else sd["state"]
    masters = sd.get("sharded_master_weights" if zero else "master_weights") or {}
    step = 0
    rows_by_buf: Dict[int, Dict[int, Dict[str, torch.Tensor]]] = {}
    for (i, gi, p, b) in entries:
        st = per_idx.get(i)
        if st is None:
            raise KeyError(f"optimizer state has no entry {i} (parameter of shape {tuple(p.shape)})")
        if "step" in st:
            step = int(float(st["step"]))
        if zero and "shape_info" in sd and tuple(sd["shape_info"][i]) != tuple(_shape(p)):
            raise ValueError(f"parameter {i}: checkpoint shape {tuple(sd['shape_info'][i])} != {tuple(p.shape)}")
        m = masters.get(i)
        if m is None:
            m = dim0_shard(p.detach().float(), b.buf.dp, b.buf.dp_rank) if (zero and _zero1(b)) else p.detach().float()
        rows_by_buf.setdefault(id(b), {})[id(p)] = {"master": m, "exp_avg": st["exp_avg"], "exp_avg_sq": st["exp_avg_sq"]}
    seen = []
    for (_, _, _, b) in entries:
        if b in seen:
            continue
        seen.append(b)
        load_full_states(b, rows_by_buf[id(b)], sharded=zero and _zero1(b))
    for gi, (g, sg) in enumerate(zip(opt.param_groups, sd["param_groups"])):
        for k, v in sg.items():
            if k != "params":
                g[k] = v
    return step
