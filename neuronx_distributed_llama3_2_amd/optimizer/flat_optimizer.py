"""Native mixed-precision AdamW / ZeRO-1 over flat buffers.

Replaces, for the AdamW family, the reference's torch_xla ZeroRedundancyOptimizer + per-parameter
AdamW_FP32OptimParams loop (src/neuronx_distributed/optimizer/zero_redundancy_optimizer.py:29-155,
src/neuronx_distributed/utils/adamw_fp32_optim_params.py:31-155):

* bf16 model parameters, fp32 master weights and fp32 Adam moments, all flat; each DP rank owns
  one slice of every gradient bucket (ZeRO-1) — or everything when DP = 1;
* one step = (finish the backward-overlapped bucket reduce-scatters) -> one coalesced TP all-reduce
  of sequence-parallel norm grads -> flat grad-norm kernel (TP-replicated params counted once,
  partial sums all-reduced over TP / DP / PP; the clip coefficient never leaves the device) ->
  fused AdamW kernel per bucket slice that also writes the bf16 weights -> bucket all-gathers;
* state_dict() saves per-parameter unflattened state on DP=1, or this rank's flat shards plus
  the shard map under ZeRO-1 (one file per DP rank, like the reference's ZeRO checkpoints).
"""

from __future__ import annotations

import math
import os
from collections import defaultdict
from typing import Any, Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

from .. import ops
from ..parallel import comm
from ..parallel.grad_buffer import KIND_DUP, KIND_DUP_SP, KIND_SHARDED, FlatBuffer, find_shared_params, param_kind
from ..parallel_layers import parallel_state as ps
from ..parallel_layers import stream_split


class _BufferState:
    def __init__(self, buf: FlatBuffer, group: dict):
        self.buf = buf
        self.group = group
        self.ranges = buf.shard_ranges()
        n = sum(e - s for s, e in self.ranges)
        dev = buf.param_data.device
        self.master = torch.empty(n, dtype=torch.float32, device=dev)
        off = 0
        self.local = []  # (buffer start, buffer end, local start)
        for s, e in self.ranges:
            self.master[off:off + e - s].copy_(buf.param_data[s:e].float())
            self.local.append((s, e, off))
            off += e - s
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)


def replica_slices(buf, ranges):
    """(start, end, weight) pieces of `ranges` (flat offsets of `buf`) that hold the K/V rows of a
    GQA QKV projection whose kv heads are replicated on m TP ranks (weight 1/m, grads.py)."""
    from ..parallel_layers.grads import kv_replica_slices

    out = []
    for p in buf.params:
        kv = kv_replica_slices(p)
        if kv is None:
            continue
        off, n = buf.offsets[id(p)]
        cols = p.shape[1] if p.dim() > 1 else 1
        ks, ke = off + kv[0] * cols, off + n
        for s, e in ranges:
            lo, hi = max(s, ks), min(e, ke)
            if lo < hi:
                out.append((lo, hi, kv[1]))
    return out


class FlatMixedPrecisionAdamW(torch.optim.Optimizer):
    """AdamW (decoupled weight decay) with fp32 master weights over flat buffers; optional ZeRO-1.

    `params` may be an iterable of parameters or of param-group dicts (lr, betas, eps, weight_decay).
    """

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 zero1: bool = False, dp_group=None, grad_clipping: bool = True, max_grad_norm: float = 1.0,
                 shared_param_ids: Optional[set] = None, sp_reduce: bool = True, bias_correction: bool = True,
                 stochastic_rounding: Optional[bool] = None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if dp_group is None and ps.model_parallel_is_initialized():
            dp_group = ps.get_data_parallel_group()
        self.dp_group = dp_group
        self.zero1 = zero1
        self.grad_clipping = grad_clipping
        self.max_grad_norm = max_grad_norm
        self.bias_correction = bias_correction
        # stochastic rounding of the bf16 weight copy-out (reference: NEURON_RT_STOCHASTIC_ROUNDING_EN)
        if stochastic_rounding is None:
            env = os.environ.get("NXD_STOCHASTIC_ROUNDING", os.environ.get("NEURON_RT_STOCHASTIC_ROUNDING_EN", "0"))
            stochastic_rounding = env == "1"
        self.stochastic_rounding = stochastic_rounding
        self.step_count = 0
        self.grad_norm: Optional[torch.Tensor] = None
        self.buffers: List[_BufferState] = []
        shared = shared_param_ids or set()
        for gi, g in enumerate(self.param_groups):
            by_kind = defaultdict(list)
            index_of = {}
            for pi, p in enumerate(g["params"]):
                if p.requires_grad:   # expert-parallel params get their own (EDP-reduced) buffers
                    by_kind[(param_kind(p, sp_reduce), p.dtype, p.device,
                             bool(getattr(p, "expert_model_parallel", False)))].append(p)
                    index_of[id(p)] = pi
            for (kind, _, _, is_ep), plist in by_kind.items():
                group, avg = self.dp_group, None
                if any(getattr(p, "expert_model_parallel", False) for p in plist) and ps.model_parallel_is_initialized():
                    group, avg = ps.get_expert_data_parallel_group(), ps.get_data_parallel_size()
                buf = FlatBuffer(plist, dp_group=group, zero1=zero1, shared_ids=shared, name=f"g{gi}:{kind}" + (":ep" if is_ep else ""),
                                 avg_world=avg)
                buf.kind = kind
                buf.is_expert = is_ep
                st = _BufferState(buf, g)
                st.group_index = gi
                st.param_index = [index_of[id(p)] for p in plist]   # registration order
                self.buffers.append(st)

    # ---------------------------------------------------------------- graph capture
    @property
    def capturable(self) -> bool:
        return getattr(self, "_capturable", False)

    def make_capturable(self) -> None:
        """Move the per-step scalars to the device so step() can be captured in a hipGraph: the
        step counter lives in a device tensor, bias corrections are computed on the device each
        step, and the kernels read [lr, 1-beta1^t, 1-beta2^t] from memory.  Learning rates set in
        param_groups reach the device through sync_lr() (called by GraphedTrainStep per replay)."""
        dev = self.buffers[0].master.device
        self._capturable = True
        self._dev_step = torch.full((1,), float(self.step_count), dtype=torch.float32, device=dev)
        self._dev_hyper = torch.zeros(len(self.param_groups), 3, dtype=torch.float32, device=dev)
        self._dev_betas = torch.tensor([list(g["betas"]) for g in self.param_groups], dtype=torch.float32, device=dev)
        self.sync_lr()

    def sync_lr(self) -> None:
        if self.capturable:
            lrs = torch.tensor([float(g["lr"]) for g in self.param_groups], dtype=torch.float32)
            self._dev_hyper[:, 0].copy_(lrs, non_blocking=True)

    def _device_hyper_step(self) -> torch.Tensor:
        self._dev_step.add_(1.0)
        if self.bias_correction:
            self._dev_hyper[:, 1:].copy_(1.0 - torch.pow(self._dev_betas, self._dev_step))
        else:
            self._dev_hyper[:, 1:].fill_(1.0)
        return self._dev_hyper

    # ---------------------------------------------------------------- helpers
    def set_grad_sync(self, enabled: bool) -> None:
        for b in self.buffers:
            b.buf.set_sync(enabled)

    def zero_grad(self, set_to_none: bool = True) -> None:
        stream_split.join()
        for b in self.buffers:
            b.buf.zero_grad()

    def _tp(self):
        if ps.model_parallel_is_initialized() and ps.get_tensor_model_parallel_size() > 1:
            return ps.get_tensor_model_parallel_group(), ps.get_tensor_model_parallel_rank()
        return None, 0

    def _sync_grads(self):
        for b in self.buffers:
            b.buf.finish_grad_sync(average=True)
        tp_group, _ = self._tp()
        if tp_group is not None:
            # sequence-parallel norm-weight gradients: partial sums over TP (reference
            # grads.py:313-329), all buffers in one coalesced all-reduce
            comm.all_reduce_coalesced([b.buf.grad_data for b in self.buffers if b.buf.kind == KIND_DUP_SP],
                                      group=tp_group)

    def _grad_norm_sq(self) -> torch.Tensor:
        tp_group, tp_rank = self._tp()
        dev = self.buffers[0].master.device
        total = torch.zeros(1, dtype=torch.float32, device=dev)
        # without ZeRO-1 every DP rank holds whole buffers: dense ones are replicated over DP, but
        # expert buffers hold only this EP rank's experts, so their part is summed over EP first
        # (otherwise each EP rank clips with its own norm and the replicated dense params drift)
        ep_group = None
        if not self.zero1 and ps.model_parallel_is_initialized() and ps.get_expert_model_parallel_size() > 1:
            ep_group = ps.get_expert_model_parallel_group()
        ep_total = torch.zeros(1, dtype=torch.float32, device=dev) if ep_group is not None else total
        for b in self.buffers:
            if b.buf.kind != KIND_SHARDED and tp_rank != 0:
                continue
            acc = ep_total if getattr(b.buf, "is_expert", False) else total
            for s, e in b.ranges:
                ops.flat_sumsq(b.buf.grad_data[s:e], out=acc, accumulate=True)
            for lo, hi, w in self._replica_slices(b):   # replicated K/V rows count 1/m (grads.py)
                tmp = torch.zeros(1, dtype=torch.float32, device=dev)
                ops.flat_sumsq(b.buf.grad_data[lo:hi], out=tmp, accumulate=True)
                acc.add_(tmp, alpha=w - 1.0)
        if ep_group is not None:
            dist.all_reduce(ep_total, group=ep_group)
            total.add_(ep_total)
        if tp_group is not None:
            dist.all_reduce(total, group=tp_group)
        if self.zero1 and self.dp_group is not None and dist.get_world_size(group=self.dp_group) > 1:
            dist.all_reduce(total, group=self.dp_group)
        if ps.model_parallel_is_initialized() and ps.get_pipeline_model_parallel_size() > 1:
            dist.all_reduce(total, group=ps.get_pipeline_model_parallel_group())
        return total

    def _replica_slices(self, b):
        """Flat (start, end, weight) pieces of this rank's shard that hold kv-replicated K/V rows."""
        cached = getattr(b, "_replica_cache", None)
        if cached is None:
            cached = b._replica_cache = replica_slices(b.buf, b.ranges)
        return cached

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        stream_split.join()   # the two-stream SP halves' last weight gradients
        self._sync_grads()
        coef = None
        if self.grad_clipping:
            sq = self._grad_norm_sq()
            coef = ops.clip_coefficient(sq, self.max_grad_norm, is_sumsq=True)
            self.grad_norm = coef[1]
        self.step_count += 1
        seed = ops.sr_seed_for_step(self.step_count) if self.stochastic_rounding else 0
        hyper = self._device_hyper_step() if self.capturable else None
        for bi, b in enumerate(self.buffers):
            g = b.group
            beta1, beta2 = g["betas"]
            fp32_params = b.buf.param_data.dtype == torch.float32   # e.g. MoE routers kept in fp32
            for (s, e, lo) in b.local:
                n = e - s
                ops.adamw_flat_(b.master[lo:lo + n], b.buf.grad_data[s:e], b.exp_avg[lo:lo + n], b.exp_avg_sq[lo:lo + n],
                                None if fp32_params else b.buf.param_data[s:e], g["lr"], beta1, beta2, g["eps"],
                                g["weight_decay"], self.step_count,
                                grad_scale=coef, bias_correction=self.bias_correction,
                                sr_seed=(((seed ^ (bi * 0x9E3779B1 + s)) & 0xFFFFFFFF) or 1) if seed else 0,
                                hyper=hyper[b.group_index] if hyper is not None else None)
                if fp32_params:
                    b.buf.param_data[s:e].copy_(b.master[lo:lo + n])
        for b in self.buffers:
            b.buf.gather_params()
        return loss

    # ---------------------------------------------------------------- checkpointing
    def state_dict(self) -> Dict[str, Any]:
        """The reference's layout (optimizer/zero_layout.py): torch_xla ZeRO-1 per-parameter dim-0
        shards with `base_state` / `shape_info` / `sharded_master_weights` under ZeRO-1, the plain
        torch layout (+ `master_weights`) without.  Collective over the DP group under ZeRO-1."""
        from .zero_layout import reference_state_dict

        return reference_state_dict(self)

    def flat_state_dict(self) -> Dict[str, Any]:
        """This rank's flat buffers as they are (no communication; the layout of round-2 files)."""
        groups = [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]
        bufs = []
        for b in self.buffers:
            layout = [(b.group_index, pi, b.buf.offsets[id(p)][0], p.numel(), tuple(p.shape))
                      for pi, p in zip(b.param_index, b.buf.params)]
            bufs.append({"name": b.buf.name, "ranges": b.ranges, "master": b.master, "exp_avg": b.exp_avg,
                         "exp_avg_sq": b.exp_avg_sq, "layout": layout, "numel": b.buf.numel, "dp": b.buf.dp,
                         "dp_rank": b.buf.dp_rank})
        return {"flat_optimizer": True, "step": self.step_count, "param_groups": groups, "buffers": bufs,
                "zero1": self.zero1}

    def _after_load(self) -> None:
        if self.capturable:
            self._dev_step.fill_(float(self.step_count))
        self.sync_lr()
        for b in self.buffers:
            for (s, e, lo) in b.local:
                b.buf.param_data[s:e].copy_(b.master[lo:lo + e - s])
            b.buf.gather_params()

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        from .zero_layout import is_reference_layout, load_reference_state_dict

        if sd.get("flat_optimizer_full"):
            return self._load_full_state_dict(sd)
        if not sd.get("flat_optimizer") and is_reference_layout(sd):
            self.step_count = load_reference_state_dict(self, sd)
            self._after_load()
            return
        assert sd.get("flat_optimizer"), "not a FlatMixedPrecisionAdamW state dict"
        self.step_count = int(sd["step"])
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                g[k] = v
        for b, sb in zip(self.buffers, sd["buffers"]):
            assert b.buf.name == sb["name"] and b.master.numel() == sb["master"].numel(), "optimizer layout mismatch"
            b.master.copy_(sb["master"])
            b.exp_avg.copy_(sb["exp_avg"])
            b.exp_avg_sq.copy_(sb["exp_avg_sq"])
        self._after_load()

    def _load_full_state_dict(self, sd: Dict[str, Any]) -> None:
        """DP-agnostic state (optimizer/convert_zero_checkpoints.py "full" format): per-parameter
        master / exp_avg / exp_avg_sq, scattered into this rank's flat shards."""
        self.step_count = int(sd["step"])
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                g[k] = v
        states = {(int(gi), int(pi)): st for gi, pi, st in sd["param_states"]}
        for b in self.buffers:
            full = {k: torch.zeros(b.buf.numel, dtype=torch.float32) for k in ("master", "exp_avg", "exp_avg_sq")}
            for pi, p in zip(b.param_index, b.buf.params):
                st = states[(b.group_index, pi)]
                off, n = b.buf.offsets[id(p)]
                for k in full:
                    full[k][off:off + n] = st[k].reshape(-1).float()
            for (s, e, lo) in b.local:
                b.master[lo:lo + e - s].copy_(full["master"][s:e])
                b.exp_avg[lo:lo + e - s].copy_(full["exp_avg"][s:e])
                b.exp_avg_sq[lo:lo + e - s].copy_(full["exp_avg_sq"][s:e])
                b.buf.param_data[s:e].copy_(b.master[lo:lo + e - s])
            b.buf.gather_params()
