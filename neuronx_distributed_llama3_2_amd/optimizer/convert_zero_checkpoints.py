"""Re-shard ZeRO-1 optimizer checkpoints across data-parallel sizes
(reference CLI / behaviour: src/neuronx_distributed/optimizer/convert_zero_checkpoints.py:54-223).

    python -m neuronx_distributed_llama3_2_amd.optimizer.convert_zero_checkpoints \\
        --input_dir <ckpt tag> --output_dir <out tag> (--convert_to_full | --convert_to_sharded --dp_size N)

Input: `optim/dp_rank_XX[_ep_rank_XX]_tp_rank_XX_pp_rank_XX.pt` in the reference's torch_xla ZeRO-1
layout (optimizer/zero_layout.py: per-parameter dim-0 shards, padded to a multiple of the DP size,
in `base_state` -- and `sharded_master_weights`, which the reference tool leaves unmerged and this
one merges like `base_state`).  --convert_to_full concatenates every parameter's shards over the DP
ranks and drops the padding (`shape_info`): `optim/full_[ep_rank_XX_]tp_rank_XX_pp_rank_XX.pt`;
--convert_to_sharded pads and re-chunks for the new DP size.  Files may be torch.save or xser.
Round-2 flat files (`flat_optimizer`) are still merged into the old DP-agnostic full format.
"""

from __future__ import annotations

import argparse
import concurrent.futures
import os
import re
import shutil
import time
from typing import Any, Dict, List

import torch
import torch.nn.functional as F

from ..parallel.grad_buffer import FlatBuffer, _bucket_elems, plan_flat_layout

_SHARD = re.compile(r"^dp_rank_(\d+)_(?:ep_rank_(\d+)_)?tp_rank_(\d+)_pp_rank_(\d+)\.pt$")
_FULL = re.compile(r"^full_(?:ep_rank_(\d+)_)?tp_rank_(\d+)_pp_rank_(\d+)\.pt$")


def _load(path: str):
    return torch.load(path, map_location="cpu", weights_only=True)


def get_parallel_info(input_dir: str):
    """(dp, tp, pp, is_full, ep) of the optimizer files under input_dir/optim (ep = 0 without EP)."""
    dp = tp = pp = ep = 0
    full = False
    for f in os.listdir(os.path.join(input_dir, "optim")):
        m = _SHARD.match(f)
        if m:
            dp = max(dp, int(m.group(1)) + 1)
            if m.group(2) is not None:
                ep = max(ep, int(m.group(2)) + 1)
            tp, pp = max(tp, int(m.group(3)) + 1), max(pp, int(m.group(4)) + 1)
        m = _FULL.match(f)
        if m:
            full = True
            if m.group(1) is not None:
                ep = max(ep, int(m.group(1)) + 1)
            tp, pp = max(tp, int(m.group(2)) + 1), max(pp, int(m.group(3)) + 1)
    return dp, tp, pp, full, ep


def _merge(values, shape):
    """Reference _merge: tensors are concatenated along dim 0 and un-padded to shape[0]; dicts are
    merged per key ("step" taken from the first shard); anything else from the first shard."""
    if isinstance(values[0], torch.Tensor):
        out = torch.cat(values)
        if out.shape[0] != shape[0]:
            out = out[:shape[0]]
        assert list(out.shape) == list(shape), (list(out.shape), list(shape))
        return out
    if isinstance(values[0], dict):
        return {k: (values[0][k] if k == "step" else _merge([v[k] for v in values], shape)) for k in values[0]}
    return values[0]


def _split(value, dp: int, idx: int):
    """Reference _split for one per-parameter entry: pad dim 0 to a multiple of dp, take chunk idx."""
    if isinstance(value, torch.Tensor):
        if value.size(0) % dp:
            value = F.pad(value, [0, 0] * (value.dim() - 1) + [0, dp - value.size(0) % dp])
        return value.chunk(dp)[idx].clone()
    if isinstance(value, dict):
        return {k: (v if k == "step" else _split(v, dp, idx)) for k, v in value.items()}
    return value


def merge_reference_shards(shards: List[Dict[str, Any]]) -> Dict[str, Any]:
    """ZeRO-1 shards (all DP ranks of one model shard) -> full per-parameter state."""
    merged = {k: v for k, v in shards[0].items() if k not in ("base_state", "sharded_master_weights")}
    shapes = shards[0]["shape_info"]
    base_shape = dict(shapes)
    if "ep_base_state_offset" in shards[0]:   # EP layout: base_state and shape_info offsets may differ
        bo, so = int(shards[0]["ep_base_state_offset"]), int(shards[0]["ep_shape_info_offset"])
        base_shape = {(k if k < so else k - so + bo): v for k, v in shapes.items()}
    merged["base_state"] = {k: _merge([c["base_state"][k] for c in shards], base_shape[k]) for k in shards[0]["base_state"]}
    if shards[0].get("sharded_master_weights"):
        merged["sharded_master_weights"] = {k: _merge([c["sharded_master_weights"][k] for c in shards], base_shape[k])
                                            for k in shards[0]["sharded_master_weights"]}
    return merged


def split_reference_full(full: Dict[str, Any], dp: int, idx: int) -> Dict[str, Any]:
    out = {k: v for k, v in full.items() if k not in ("base_state", "sharded_master_weights")}
    out["base_state"] = {k: _split(v, dp, idx) for k, v in full["base_state"].items()}
    if full.get("sharded_master_weights"):
        out["sharded_master_weights"] = {k: _split(v, dp, idx) for k, v in full["sharded_master_weights"].items()}
    return out


def merge_dp_shards(shards: List[Dict[str, Any]]) -> Dict[str, Any]:
    if not shards[0].get("flat_optimizer"):
        return merge_reference_shards(shards)
    return _merge_flat_shards(shards)


def _merge_flat_shards(shards: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Round-2 FlatMixedPrecisionAdamW shards of one (tp, pp) rank -> full per-parameter state."""
    base = shards[0]
    states = []
    for bi, b0 in enumerate(base["buffers"]):
        full = {k: torch.zeros(b0["numel"], dtype=torch.float32) for k in ("master", "exp_avg", "exp_avg_sq")}
        for sd in shards:
            b = sd["buffers"][bi]
            lo = 0
            for (s, e) in b["ranges"]:
                for k in full:
                    full[k][s:e] = b[k][lo:lo + e - s].float()
                lo += e - s
        for (gi, pi, off, n, shape) in b0["layout"]:
            states.append((gi, pi, {k: full[k][off:off + n].view(shape).clone() for k in full}))
    return {"flat_optimizer_full": True, "step": base["step"], "param_groups": base["param_groups"],
            "param_states": states, "buffer_names": [b["name"] for b in base["buffers"]],
            "buffer_params": [[(gi, pi, n, shape) for (gi, pi, _, n, shape) in b["layout"]] for b in base["buffers"]]}


def shard_full_state(full: Dict[str, Any], dp: int, dp_rank: int) -> Dict[str, Any]:
    """Full state -> the ZeRO-1 shard DP rank `dp_rank` of `dp` would save (same bucket planner as
    FlatBuffer; the bucket cap comes from NXD_DP_BUCKET_MB as in training)."""
    states = {(gi, pi): st for gi, pi, st in full["param_states"]}
    bufs = []
    for name, plist in zip(full["buffer_names"], full["buffer_params"]):
        order = list(reversed(plist))   # FlatBuffer lays parameters out in reverse registration order
        offs, spans, total = plan_flat_layout([n for (_, _, n, _) in order], dp, _bucket_elems(), FlatBuffer.ALIGN)
        flat = {k: torch.zeros(total, dtype=torch.float32) for k in ("master", "exp_avg", "exp_avg_sq")}
        layout = []
        off_of = {(gi, pi): o for (gi, pi, _, _), o in zip(order, offs)}
        for (gi, pi, n, shape) in plist:
            o = off_of[(gi, pi)]
            for k in flat:
                flat[k][o:o + n] = states[(gi, pi)][k].reshape(-1)
            layout.append((gi, pi, o, n, shape))
        if dp > 1:
            ranges = [(bs + dp_rank * ((be - bs) // dp), bs + (dp_rank + 1) * ((be - bs) // dp)) for (bs, be, _, _) in spans]
        else:
            ranges = [(0, total)]
        entry = {"name": name, "ranges": ranges, "layout": layout, "numel": total, "dp": dp, "dp_rank": dp_rank}
        for k in flat:
            entry[k] = torch.cat([flat[k][s:e] for (s, e) in ranges])
        bufs.append(entry)
    return {"flat_optimizer": True, "step": full["step"], "param_groups": full["param_groups"], "buffers": bufs,
            "zero1": dp > 1}


def _name(prefix: str, ep, tp_rank: int, pp_rank: int) -> str:
    e = f"ep_rank_{ep:02d}_" if ep is not None else ""
    return f"{prefix}{e}tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"


def _read(args, fn):
    path = os.path.join(args.input_dir, "optim", fn)
    if args.is_xser:
        from ..utils.serialization import xser_load

        return xser_load(path)
    return _load(path)


def _write(args, obj, fn):
    path = os.path.join(args.output_dir, "optim", fn)
    if args.is_xser:
        from ..utils.serialization import xser_save

        xser_save(obj, path)
    else:
        torch.save(obj, path)


def _shards(args, tp_rank, pp_rank, ep):
    return [_read(args, _name(f"dp_rank_{d:02d}_", ep, tp_rank, pp_rank)) for d in range(args.dp_size)]


def _to_sharded(args, full, tp_rank, pp_rank, ep):
    for d in range(args.new_dp_size):
        if full.get("flat_optimizer_full"):
            obj = shard_full_state(full, args.new_dp_size, d)
        else:
            obj = split_reference_full(full, args.new_dp_size, d)
        _write(args, obj, _name(f"dp_rank_{d:02d}_", ep, tp_rank, pp_rank))


def _sharded_to_full_task(args, tp_rank, pp_rank, ep=None):
    _write(args, merge_dp_shards(_shards(args, tp_rank, pp_rank, ep)), _name("full_", ep, tp_rank, pp_rank))


def _full_to_sharded_task(args, tp_rank, pp_rank, ep=None):
    _to_sharded(args, _read(args, _name("full_", ep, tp_rank, pp_rank)), tp_rank, pp_rank, ep)


def _sharded_to_sharded_task(args, tp_rank, pp_rank, ep=None):
    _to_sharded(args, merge_dp_shards(_shards(args, tp_rank, pp_rank, ep)), tp_rank, pp_rank, ep)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input_dir", type=str, required=True)
    p.add_argument("--output_dir", type=str, required=True)
    p.add_argument("--num_workers", type=int, default=1)
    p.add_argument("--dp_size", type=int, default=None, help="new DP size (convert_to_sharded)")
    g = p.add_mutually_exclusive_group(required=True)
    g.add_argument("--convert_to_full", action="store_true")
    g.add_argument("--convert_to_sharded", action="store_true")
    args, _ = p.parse_known_args(argv)
    args.new_dp_size = args.dp_size
    args.dp_size, args.tp_size, args.pp_size, is_full, args.ep_size = get_parallel_info(args.input_dir)
    args.is_xser = any(f.endswith(".tensors") for f in os.listdir(os.path.join(args.input_dir, "optim")))
    shutil.rmtree(os.path.join(args.output_dir, "optim"), ignore_errors=True)
    os.makedirs(os.path.join(args.output_dir, "optim"), exist_ok=True)
    if args.convert_to_full:
        if is_full:
            raise ValueError("Invalid inputs: convert full optim states to full optim states")
        task = _sharded_to_full_task
    else:
        assert args.new_dp_size, "--dp_size is required for --convert_to_sharded"
        task = _full_to_sharded_task if is_full else _sharded_to_sharded_task
    print(f"Task {task.__name__} started.")
    t0 = time.time()
    with concurrent.futures.ThreadPoolExecutor(max_workers=args.num_workers) as ex:
        eps = list(range(args.ep_size)) if args.ep_size else [None]
        futs = [ex.submit(task, args, t, pp, e) for t in range(args.tp_size) for pp in range(args.pp_size) for e in eps]
        for f in futs:
            f.result()
    print(f"Task {task.__name__} done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
