"""Re-shard ZeRO-1 optimizer checkpoints across data-parallel sizes
(reference CLI / behaviour: src/neuronx_distributed/optimizer/convert_zero_checkpoints.py:54-223).

    python -m neuronx_distributed_llama3_2_amd.optimizer.convert_zero_checkpoints \\
        --input_dir <ckpt tag> --output_dir <out tag> (--convert_to_full | --convert_to_sharded --dp_size N)

Input `optim/dp_rank_XX_tp_rank_XX_pp_rank_XX.pt` files (FlatMixedPrecisionAdamW ZeRO-1 shards: each
holds its slice of every DP bucket plus the buffer layout) are merged per (tp, pp) into a
DP-agnostic "full" state `optim/full_tp_rank_XX_pp_rank_XX.pt` (per-parameter fp32 master /
exp_avg / exp_avg_sq), which any DP size can load directly; `--convert_to_sharded` re-slices the
full state for a new DP size with the same bucket planner the flat buffers use.
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

from ..parallel.grad_buffer import FlatBuffer, _bucket_elems, plan_flat_layout

_SHARD = re.compile(r"^dp_rank_(\d+)_tp_rank_(\d+)_pp_rank_(\d+)\.pt$")
_FULL = re.compile(r"^full_tp_rank_(\d+)_pp_rank_(\d+)\.pt$")


def _load(path: str):
    return torch.load(path, map_location="cpu", weights_only=True)


def get_parallel_info(input_dir: str):
    dp = tp = pp = 0
    full = False
    for f in os.listdir(os.path.join(input_dir, "optim")):
        m = _SHARD.match(f)
        if m:
            dp, tp, pp = max(dp, int(m.group(1)) + 1), max(tp, int(m.group(2)) + 1), max(pp, int(m.group(3)) + 1)
        m = _FULL.match(f)
        if m:
            full = True
            tp, pp = max(tp, int(m.group(1)) + 1), max(pp, int(m.group(2)) + 1)
    return dp, tp, pp, full


def merge_dp_shards(shards: List[Dict[str, Any]]) -> Dict[str, Any]:
    """ZeRO-1 shards of one (tp, pp) rank (all DP ranks) -> full per-parameter state."""
    base = shards[0]
    assert base.get("flat_optimizer"), "expects FlatMixedPrecisionAdamW state dicts"
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


def _sharded_to_full_task(args, tp_rank, pp_rank):
    shards = [_load(os.path.join(args.input_dir, "optim", f"dp_rank_{d:02d}_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"))
              for d in range(args.dp_size)]
    torch.save(merge_dp_shards(shards),
               os.path.join(args.output_dir, "optim", f"full_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"))


def _full_to_sharded_task(args, tp_rank, pp_rank, full=None):
    full = full or _load(os.path.join(args.input_dir, "optim", f"full_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"))
    for d in range(args.new_dp_size):
        torch.save(shard_full_state(full, args.new_dp_size, d),
                   os.path.join(args.output_dir, "optim", f"dp_rank_{d:02d}_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"))


def _sharded_to_sharded_task(args, tp_rank, pp_rank):
    shards = [_load(os.path.join(args.input_dir, "optim", f"dp_rank_{d:02d}_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"))
              for d in range(args.dp_size)]
    _full_to_sharded_task(args, tp_rank, pp_rank, merge_dp_shards(shards))


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
    args.dp_size, args.tp_size, args.pp_size, is_full = get_parallel_info(args.input_dir)
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
        futs = [ex.submit(task, args, t, pp) for t in range(args.tp_size) for pp in range(args.pp_size)]
        for f in futs:
            f.result()
    print(f"Task {task.__name__} done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
