"""ZeRO-1 optimizers with the reference's class names and constructor
(src/neuronx_distributed/optimizer/zero_redundancy_optimizer.py:29-362).

`NeuronZero1Optimizer(params, optimizer_class, grad_clipping=True, max_norm=..., sharding_groups=...,
grad_norm_groups=..., pin_layout=..., coalesce_cc=..., use_grad_acc_hook=..., higher_cc_precision=...,
save_master_weights=..., **defaults)`:

* AdamW family (torch.optim.AdamW / Adam, AdamW_FP32OptimParams): the native flat path
  (FlatMixedPrecisionAdamW, zero1=True) — bucketed backward-overlapped reduce-scatter, fused
  AdamW kernel on this rank's fp32 shard, bucket all-gather of the bf16 weights.
* Any other optimizer class: generic ZeRO-1 on the same flat buffers — this rank's fp32 master
  shard of every bucket becomes one parameter of an `optimizer_class` instance whose `.grad` is the
  reduce-scattered fp32 gradient slice (elementwise optimizers are exact; per-tensor statistics
  such as LAMB trust ratios are computed per bucket slice).
* Expert-parallel parameters (`expert_model_parallel`) are sharded over the expert-data-parallel
  group (NeuronEPZero1Optimizer semantics) automatically.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import torch
import torch.distributed as dist

from .. import ops
from ..parallel.grad_buffer import KIND_DUP_SP, KIND_SHARDED, FlatBuffer, param_kind
from ..parallel_layers import parallel_state as ps
from ..parallel_layers import stream_split
from .flat_optimizer import FlatMixedPrecisionAdamW, replica_slices

_ADAM_NAMES = {"AdamW", "Adam", "AdamW_FP32OptimParams", "FusedAdam"}


def _is_adam_family(cls) -> bool:
    return getattr(cls, "__name__", "") in _ADAM_NAMES


class _GenericZero1(torch.optim.Optimizer):
    def __init__(self, params, optimizer_class, dp_group=None, grad_clipping=True, max_norm=1.0, **defaults):
        super().__init__(params, dict(defaults))
        self.dp_group = dp_group if dp_group is not None else (
            ps.get_data_parallel_group() if ps.model_parallel_is_initialized() else None)
        self.grad_clipping, self.max_norm = grad_clipping, max_norm
        self.buffers = []
        inner_groups = []
        for g in self.param_groups:
            plist = [p for p in g["params"] if p.requires_grad]
            if not plist:
                continue
            kinds = {}
            for p in plist:   # expert-parallel params get their own (EDP-sharded) buffers
                kinds.setdefault((param_kind(p), bool(getattr(p, "expert_model_parallel", False))), []).append(p)
            for kind, ps_ in kinds.items():
                group, avg = self.dp_group, None
                if any(getattr(p, "expert_model_parallel", False) for p in ps_) and ps.model_parallel_is_initialized():
                    group, avg = ps.get_expert_data_parallel_group(), ps.get_data_parallel_size()
                buf = FlatBuffer(ps_, dp_group=group, zero1=True, name=kind, avg_world=avg)
                buf.kind = kind[0]
                masters = []
                for s, e in buf.shard_ranges():
                    m = torch.nn.Parameter(buf.param_data[s:e].detach().float().clone())
                    m._range = (s, e)
                    masters.append(m)
                self.buffers.append((buf, masters))
                gi = {k: v for k, v in g.items() if k != "params"}
                gi["params"] = masters
                inner_groups.append(gi)
        self.inner = optimizer_class(inner_groups, **defaults)
        self.grad_norm = None

    def set_grad_sync(self, enabled: bool) -> None:
        for b, _ in self.buffers:
            b.set_sync(enabled)

    def zero_grad(self, set_to_none: bool = True) -> None:
        stream_split.join()
        for b, _ in self.buffers:
            b.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        stream_split.join()   # main_grad is written by the SP halves' streams
        for b, _ in self.buffers:
            b.finish_grad_sync()
        tp = ps.get_tensor_model_parallel_size() if ps.model_parallel_is_initialized() else 1
        if tp > 1:
            for b, _ in self.buffers:
                if b.kind == KIND_DUP_SP:
                    dist.all_reduce(b.grad_data, group=ps.get_tensor_model_parallel_group())
        for b, masters in self.buffers:
            for m in masters:
                s, e = m._range
                m.grad = b.grad_data[s:e]
        if self.grad_clipping:
            dev = self.buffers[0][0].grad_data.device
            sq = torch.zeros(1, dtype=torch.float32, device=dev)
            tp_rank = ps.get_tensor_model_parallel_rank() if ps.model_parallel_is_initialized() else 0
            for b, masters in self.buffers:
                if b.kind != KIND_SHARDED and tp_rank != 0:
                    continue
                for m in masters:
                    ops.flat_sumsq(m.grad, out=sq, accumulate=True)
                for lo, hi, w in replica_slices(b, [m._range for m in masters]):   # replicated K/V rows
                    tmp = torch.zeros(1, dtype=torch.float32, device=dev)
                    ops.flat_sumsq(b.grad_data[lo:hi], out=tmp, accumulate=True)
                    sq.add_(tmp, alpha=w - 1.0)
            if tp > 1:
                dist.all_reduce(sq, group=ps.get_tensor_model_parallel_group())
            if self.dp_group is not None and dist.get_world_size(group=self.dp_group) > 1:
                dist.all_reduce(sq, group=self.dp_group)
            coef = ops.clip_coefficient(sq, self.max_norm)
            self.grad_norm = coef[1]
            for b, masters in self.buffers:
                for m in masters:
                    m.grad.mul_(coef[0])
        loss = self.inner.step(closure)
        for b, masters in self.buffers:
            for m in masters:
                s, e = m._range
                b.param_data[s:e].copy_(m.detach())
            b.gather_params()
        return loss

    def state_dict(self) -> Dict[str, Any]:
        return {"generic_zero1": True, "inner": self.inner.state_dict(),
                "masters": [[m.detach() for m in ms] for _, ms in self.buffers]}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.inner.load_state_dict(sd["inner"])
        for (b, ms), saved in zip(self.buffers, sd["masters"]):
            for m, t in zip(ms, saved):
                m.data.copy_(t)
                s, e = m._range
                b.param_data[s:e].copy_(m.detach())
            b.gather_params()


def NeuronZero1Optimizer(params, optimizer_class=torch.optim.AdamW, grad_clipping: bool = True, max_norm: float = 1.0,
                         sharding_groups=None, grad_norm_groups=None, pin_layout: bool = False, coalesce_cc: bool = True,
                         use_grad_acc_hook: bool = True, higher_cc_precision: bool = True,
                         save_master_weights: bool = False, lazy_init: bool = False, optimizer_dtype=None,
                         shared_param_ids: Optional[set] = None, **defaults):
    """Factory with the reference signature; returns the MI355X-native implementation."""
    dp_group = None
    if isinstance(sharding_groups, (torch.distributed.ProcessGroup,)):
        dp_group = sharding_groups
    elif ps.model_parallel_is_initialized():
        dp_group = ps.get_data_parallel_group()
    if _is_adam_family(optimizer_class):
        kw = {k: v for k, v in defaults.items() if k in ("lr", "betas", "eps", "weight_decay")}
        opt = FlatMixedPrecisionAdamW(params, zero1=True, dp_group=dp_group, grad_clipping=grad_clipping,
                                      max_grad_norm=max_norm, shared_param_ids=shared_param_ids, **kw)
    else:
        opt = _GenericZero1(params, optimizer_class, dp_group=dp_group, grad_clipping=grad_clipping, max_norm=max_norm,
                            **defaults)
    opt.save_master_weights = save_master_weights
    return opt


class _FlatEPZero1(FlatMixedPrecisionAdamW):
    """AdamW-family ZeRO-1 with expert parallelism (reference NeuronEPZero1Optimizer,
    optimizer/zero_redundancy_optimizer.py:158-362): dense parameters are sharded over the DP group,
    expert parameters over the expert-data-parallel group (their own flat buffers, gradients averaged
    over the whole DP world); ONE gradient norm over both (every shard counted once) clips both.

    state_dict() has the reference's combined layout (optimizer/zero_layout.py per part): the dense
    optimizer's torch_xla ZeRO entries first, the expert optimizer's after them at
    `ep_param_id_offset` / `ep_param_group_offset` / `ep_base_state_offset` / `ep_shape_info_offset`
    (reference zero_redundancy_optimizer.py:281-362)."""

    def _split(self):
        dense = [b for b in self.buffers if not b.buf.name.endswith(":ep")]
        expert = [b for b in self.buffers if b.buf.name.endswith(":ep")]
        return dense, expert

    def state_dict(self) -> Dict[str, Any]:
        from .zero_layout import reference_state_dict

        dense, expert = self._split()
        d = reference_state_dict(self, dense)
        e = reference_state_dict(self, expert)

        def offset(dct):
            return max(dct) + 1 if len(dct) > 0 else 1

        ep_pid, ep_base, ep_shape = offset(d["state"]), offset(d["base_state"]), offset(d["shape_info"])
        out = {"ep_param_id_offset": ep_pid, "ep_param_group_offset": len(d["param_groups"]),
               "ep_base_state_offset": ep_base, "ep_shape_info_offset": ep_shape,
               "param_groups": d["param_groups"] + e["param_groups"],
               "state": dict(d["state"]), "base_state": dict(d["base_state"]), "shape_info": dict(d["shape_info"]),
               "sharded_master_weights": dict(d["sharded_master_weights"])}
        for k, v in e["state"].items():
            out["state"][ep_pid + k] = v
        for k, v in e["base_state"].items():
            out["base_state"][ep_base + k] = v
            out["sharded_master_weights"][ep_base + k] = e["sharded_master_weights"][k]
        for k, v in e["shape_info"].items():
            out["shape_info"][ep_shape + k] = v
        return out

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        from .zero_layout import load_reference_state_dict

        if sd.get("flat_optimizer") or sd.get("flat_optimizer_full"):
            return super().load_state_dict(sd)
        keys = ("ep_param_id_offset", "ep_param_group_offset", "ep_base_state_offset", "ep_shape_info_offset")
        if any(k not in sd for k in keys):
            raise ValueError("state_dict is not compatible with expert parallelism and Zero-1.")
        pid, goff = int(sd["ep_param_id_offset"]), int(sd["ep_param_group_offset"])
        boff, soff = int(sd["ep_base_state_offset"]), int(sd["ep_shape_info_offset"])

        def split(key, off):
            lo, hi = {}, {}
            for k, v in (sd.get(key) or {}).items():
                (lo if k < off else hi)[k if k < off else k - off] = v
            return lo, hi

        st_d, st_e = split("state", pid)
        bs_d, bs_e = split("base_state", boff)
        sh_d, sh_e = split("shape_info", soff)
        mw_d, mw_e = split("sharded_master_weights", boff)
        dense, expert = self._split()
        step = load_reference_state_dict(self, {"state": st_d, "base_state": bs_d, "shape_info": sh_d,
                                                "sharded_master_weights": mw_d,
                                                "param_groups": sd["param_groups"][:goff]}, dense)
        if expert:
            step = load_reference_state_dict(self, {"state": st_e, "base_state": bs_e, "shape_info": sh_e,
                                                    "sharded_master_weights": mw_e,
                                                    "param_groups": sd["param_groups"][goff:]}, expert)
        self.step_count = step
        self._after_load()


def NeuronEPZero1Optimizer(params, optimizer_class=torch.optim.AdamW, grad_clipping: bool = True,
                           max_norm: float = 1.0, sharding_groups=None, shared_param_ids: Optional[set] = None,
                           save_master_weights: bool = False, **kwargs):
    """Expert-parallel ZeRO-1: expert params sharded over the expert-data-parallel group, dense params
    over the DP group, one combined gradient norm, reference-layout merged state dict."""
    if sharding_groups is not None and not isinstance(sharding_groups, torch.distributed.ProcessGroup) and \
            ps.model_parallel_is_initialized() and sharding_groups != ps.get_data_parallel_group(as_list=True):
        raise ValueError("Custom sharding group for Zero-1 with expert parallelism is not supported.")
    if not _is_adam_family(optimizer_class):
        return NeuronZero1Optimizer(params, optimizer_class, grad_clipping=grad_clipping, max_norm=max_norm,
                                    shared_param_ids=shared_param_ids, save_master_weights=save_master_weights,
                                    **kwargs)
    kw = {k: v for k, v in kwargs.items() if k in ("lr", "betas", "eps", "weight_decay")}
    dp_group = ps.get_data_parallel_group() if ps.model_parallel_is_initialized() else None
    opt = _FlatEPZero1(params, zero1=True, dp_group=dp_group, grad_clipping=grad_clipping, max_grad_norm=max_norm,
                       shared_param_ids=shared_param_ids, **kw)
    opt.save_master_weights = save_master_weights
    return opt
