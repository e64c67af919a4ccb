"""Full <-> sharded (TP x PP x EP) checkpoint conversion for the framework's models
(reference CLI and behaviour: src/neuronx_distributed/scripts/checkpoint_converter.py:20-739).

    python -m neuronx_distributed_llama3_2_amd.scripts.checkpoint_converter \\
        --input_dir <hf dir | checkpoint.pt> --output_dir <ckpt> --config config.json \\
        --tp_size 8 --pp_size 1 --convert_from_full_state [--kv_size_multiplier 1] [--save_xser]
    python -m ... --input_dir <ckpt>/model --output_dir <dir> --config config.json \\
        --tp_size 8 --pp_size 1 --convert_to_full_state [--model_style hf]

Full states are HF-named (q/k/v/gate/up separate); sharded states use the framework's fused names
(`self_attn.qkv_proj.weight_qkv`, `mlp.gate_up_proj.weight`) and file layout
`model/dp_rank_00[_ep_rank_XX]_tp_rank_XX_pp_rank_XX.pt` (v2/v3; v1 `tp_rank_XX_pp_rank_XX/checkpoint.pt`
and xser directories are read too).  Partitioning rules are derived from parameter names:
vocab-sharded embedding / lm_head (dim 0), fused QKV (Q split, K/V replicated `kv_size_multiplier`
times then split), gate_up column-parallel with stride 2, o_proj / down_proj row-parallel (dim 1),
MoE experts sharded over EP on dim 0 and over TP on their I dim, norms / routers replicated; layers
are spread over PP stages like the pipeline partitioner (remainder to later stages).
"""

from __future__ import annotations

import argparse
import json
import os
import re
from typing import Dict, List, Optional, Tuple

import torch

from ..models.llama.convert import hf_to_nxd, nxd_to_hf
from ..parallel_layers.sharding import merge_tensors, shard_tensor
from ..pipeline.partition import create_partitions

_LAYER = re.compile(r"^model\.layers\.(\d+)\.")


class _Cfg:
    def __init__(self, d: dict):
        self.__dict__.update(d)
        self.num_key_value_heads = d.get("num_key_value_heads") or d["num_attention_heads"]
        self.head_dim = d.get("head_dim") or d["hidden_size"] // d["num_attention_heads"]
        self.tie_word_embeddings = d.get("tie_word_embeddings", False)


class CheckpointConverterBase:
    # ------------------------------------------------------------------ partition rules
    def get_partition_attrs(self, name: str, cfg: _Cfg, kv_mult: int) -> dict:
        """Sharding attributes of a framework-named parameter (see parallel_layers/sharding.py)."""
        rep = {"tp": False, "dim": 0, "stride": 1, "qkv": None}
        if name.endswith("embed_tokens.weight") or name == "lm_head.weight":
            return {"tp": True, "dim": 0, "stride": 1, "qkv": None}
        if "qkv_proj.weight_qkv" in name or "qkv_proj.bias_qkv" in name:
            return {"tp": True, "dim": 0, "stride": 1,
                    "qkv": (cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim, kv_mult)}
        if "experts" in name or "mlp_op" in name:
            if "gate_up_proj" in name:
                return {"tp": True, "dim": 2, "stride": 2, "qkv": None, "ep": True}
            if "down_proj" in name:
                return {"tp": True, "dim": 1, "stride": 1, "qkv": None, "ep": True}
        if "gate_up_proj.weight" in name:
            return {"tp": True, "dim": 0, "stride": 2, "qkv": None}
        if name.endswith("o_proj.weight"):   # head groups follow the Q reshuffle of replicated kv heads
            return {"tp": True, "dim": 1, "stride": 1, "qkv": None, "qgroup_mult": kv_mult}
        if name.endswith("down_proj.weight"):
            return {"tp": True, "dim": 1, "stride": 1, "qkv": None}
        return rep

    # ------------------------------------------------------------------ IO
    def load_full_state(self, args) -> Dict[str, torch.Tensor]:
        p = args.input_dir
        if os.path.isdir(p):
            cands = [os.path.join(p, "checkpoint.pt")]
            if os.path.exists(cands[0]):
                sd = torch.load(cands[0], map_location="cpu", weights_only=True)
            else:
                from ..inference.generation import load_hf_state_dict

                sd = load_hf_state_dict(p)
        else:
            sd = torch.load(p, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and args.model_key in sd and isinstance(sd[args.model_key], dict):
            sd = sd[args.model_key]
        return sd

    def get_input_filename(self, args, tp_rank, pp_rank, ep_rank, xser: bool) -> str:
        d = args.input_dir
        v1 = os.path.join(d, f"tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}")
        if xser and os.path.isdir(v1):
            return v1
        v1f = os.path.join(v1, "checkpoint.pt")
        v2 = os.path.join(d, f"dp_rank_00_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt")
        v3 = os.path.join(d, f"dp_rank_00_ep_rank_{ep_rank:02d}_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt")
        for f in (v1f, v2, v3):
            if os.path.exists(f):
                return f
        raise RuntimeError(f"Error: neither {v1f}, nor {v2}, nor {v3} exist")

    def get_output_filename(self, args, tp_rank, pp_rank, ep_rank, xser: bool) -> str:
        if args.ep_size > 1:
            fn = f"dp_rank_00_ep_rank_{ep_rank:02d}_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"
        else:
            fn = f"dp_rank_00_tp_rank_{tp_rank:02d}_pp_rank_{pp_rank:02d}.pt"
        return os.path.join(args.output_dir, "model", fn)

    def load_partial(self, args, tp_rank, pp_rank, ep_rank) -> Dict[str, torch.Tensor]:
        fn = self.get_input_filename(args, tp_rank, pp_rank, ep_rank, args.load_xser)
        if args.load_xser:
            from ..utils.serialization import xser_load

            return xser_load(fn)
        sd = torch.load(fn, map_location="cpu", weights_only=True)
        return sd.get(args.model_key, sd) if isinstance(sd.get(args.model_key, None), dict) else sd

    def save_partial(self, args, state, tp_rank, pp_rank, ep_rank) -> None:
        fn = self.get_output_filename(args, tp_rank, pp_rank, ep_rank, args.save_xser)
        os.makedirs(os.path.dirname(fn), exist_ok=True)
        if args.save_xser:
            from ..utils.serialization import xser_save

            xser_save(state, fn)
        else:
            torch.save(state, fn)

    def save_full(self, args, full_state) -> None:
        os.makedirs(args.output_dir, exist_ok=True)
        path = os.path.join(args.output_dir, "checkpoint.pt")
        print(f"Saving full checkpoint to {path}")
        torch.save(full_state, path)

    # ------------------------------------------------------------------ conversions
    def _stage_layers(self, n_layers: int, stages: int) -> List[Tuple[int, int]]:
        starts = [0] + create_partitions(stages, n_layers) + [n_layers]
        return [(starts[i], starts[i + 1]) for i in range(stages)]

    def _stage_of_key(self, key: str, ranges, stages: int) -> List[int]:
        m = _LAYER.match(key)
        if m:
            li = int(m.group(1))
            return [s for s, (a, b) in enumerate(ranges) if a <= li < b]
        if key.startswith("model.embed_tokens"):
            return [0]
        if key.startswith("model.norm") or key.startswith("lm_head"):
            return [stages - 1]
        return list(range(stages))

    def convert_full_state_to_tp(self, full: Dict[str, torch.Tensor], args, tp_rank, pp_rank, ep_rank,
                                 ranges, cfg: _Cfg) -> Dict[str, torch.Tensor]:
        stages = len(ranges)
        out = {}
        for k, v in full.items():
            owners = self._stage_of_key(k, ranges, stages)
            if args.pp_size * args.virtual_pp_size > 1:
                # virtual stage s lives on pp rank s % pp_size
                if not any(s % args.pp_size == pp_rank for s in owners):
                    continue
            a = self.get_partition_attrs(k, cfg, args.kv_size_multiplier)
            t = v
            if a.get("ep") and args.ep_size > 1:
                per = t.shape[0] // args.ep_size
                t = t[ep_rank * per:(ep_rank + 1) * per]
            out[k] = shard_tensor(t, a, args.tp_size, tp_rank).contiguous().clone()
        return out

    def convert_from_full_state(self, args) -> None:
        with open(args.config) as f:
            cfg = _Cfg(json.load(f))
        full = self.load_full_state(args)
        if args.model_style == "hf" and any(".q_proj." in k or ".gate_proj." in k for k in full):
            full = hf_to_nxd(full, cfg)
        if cfg.tie_word_embeddings and "lm_head.weight" not in full:
            full["lm_head.weight"] = full["model.embed_tokens.weight"]
        n_layers = args.n_layers or cfg.num_hidden_layers
        ranges = self._stage_layers(n_layers, args.pp_size * args.virtual_pp_size)
        print(f"pipeline stages (layer ranges): {ranges}")
        for tp in range(args.tp_size):
            for pp in range(args.pp_size):
                for ep in range(args.ep_size):
                    self.save_partial(args, self.convert_full_state_to_tp(full, args, tp, pp, ep, ranges, cfg), tp, pp,
                                      ep)

    def merge_tp_checkpoints(self, args) -> Dict[str, torch.Tensor]:
        with open(args.config) as f:
            cfg = _Cfg(json.load(f))
        full: Dict[str, torch.Tensor] = {}
        for pp in range(args.pp_size):
            parts = {}
            for ep in range(args.ep_size):
                shards = [self.load_partial(args, tp, pp, ep) for tp in range(args.tp_size)]
                for k in shards[0]:
                    a = self.get_partition_attrs(k, cfg, args.kv_size_multiplier)
                    t = merge_tensors([s[k] for s in shards], a)
                    if a.get("ep") and args.ep_size > 1:
                        parts.setdefault(k, []).append(t)
                    else:
                        parts[k] = [t]
            for k, ts in parts.items():
                full[k] = torch.cat(ts, 0) if len(ts) > 1 else ts[0]
        if args.model_style == "hf":
            full = nxd_to_hf(full, cfg)
        return full

    def convert_to_full_state(self, args) -> None:
        self.save_full(args, self.merge_tp_checkpoints(args))

    def convert_from_xser(self, args) -> None:
        from ..utils.serialization import xser_load

        for tp in range(args.tp_size):
            for pp in range(args.pp_size):
                for ep in range(args.ep_size):
                    st = xser_load(self.get_input_filename(args, tp, pp, ep, True))
                    fn = self.get_output_filename(args, tp, pp, ep, False)
                    os.makedirs(os.path.dirname(fn), exist_ok=True)
                    torch.save(st, fn)

    def convert_to_xser(self, args) -> None:
        from ..utils.serialization import xser_save

        for tp in range(args.tp_size):
            for pp in range(args.pp_size):
                for ep in range(args.ep_size):
                    st = torch.load(self.get_input_filename(args, tp, pp, ep, False), map_location="cpu",
                                    weights_only=True)
                    fn = self.get_output_filename(args, tp, pp, ep, True)
                    os.makedirs(os.path.dirname(fn), exist_ok=True)
                    xser_save(st, fn)

    # ------------------------------------------------------------------ CLI
    def get_arg_parser(self):
        p = argparse.ArgumentParser()
        p.add_argument("--input_dir", type=str, required=True)
        p.add_argument("--output_dir", type=str, required=True)
        p.add_argument("--config", type=str)
        p.add_argument("--model_key", type=str, default="model")
        p.add_argument("--tp_size", type=int, default=1)
        p.add_argument("--pp_size", type=int, default=1)
        p.add_argument("--ep_size", type=int, default=1)
        p.add_argument("--virtual_pp_size", type=int, default=1)
        p.add_argument("--n_layers", type=int, default=0)
        p.add_argument("--coalesce_qkv", type=bool, default=False)
        p.add_argument("--kv_size_multiplier", type=int, default=1)
        p.add_argument("--qkv_linear", type=bool, default=True)
        p.add_argument("--fuse_qkv", type=bool, default=True)
        p.add_argument("--load_xser", type=bool, default=False)
        p.add_argument("--save_xser", type=bool, default=False)
        p.add_argument("--convert_from_xser", action="store_true")
        p.add_argument("--convert_to_xser", action="store_true")
        p.add_argument("--convert_from_full_state", action="store_true")
        p.add_argument("--convert_to_full_state", action="store_true")
        p.add_argument("--model_style", type=str, choices=["hf", "megatron", "nxd"], default="hf")
        return p

    def run(self, args) -> None:
        flags = ["convert_from_full_state", "convert_to_full_state", "convert_from_xser", "convert_to_xser"]
        assert sum(int(getattr(args, f)) for f in flags) == 1, "Exactly one '--convert_*' flag must be specified"
        getattr(self, [f for f in flags if getattr(args, f)][0])(args)


def main(argv: Optional[List[str]] = None) -> None:
    conv = CheckpointConverterBase()
    conv.run(conv.get_arg_parser().parse_args(argv))


if __name__ == "__main__":
    main()
