"""Expert MLPs: token dispatch + batched expert GEMMs
(reference: src/neuronx_distributed/modules/moe/expert_mlps.py:13-357, experts.py:23-163).

Dispatch modes (same selection rules as the reference):
* capacity factor (static shapes): every expert holds C = ceil(T * top_k * cf / E) tokens, later
  tokens are dropped (their affinity contribution is zero) — position-in-expert by an exact
  integer cumsum over the token dim; expert-aligned [E, C, H] tokens go through one batched GEMM
  per projection and, with expert parallelism, through an all-to-all over the EP group;
* full capacity ("dropless"): the reference runs every token through every expert (E x the
  FLOPs); here tokens are sorted by expert and each expert multiplies only its own rows (grouped
  GEMMs over contiguous segments) — same result, top_k / E of the work;
* selective loading (token generation with few tokens): only the chosen experts' weights are read.
"""

from __future__ import annotations

import math
from typing import Any, Callable, Optional, Union

import torch
import torch.nn.functional as F
from torch import nn

from ... import ops
from ...parallel_layers import parallel_state as ps
from ...parallel_layers.mappings import (
    copy_to_tensor_model_parallel_region,
    enter_expert_parallel_region,
    exit_expert_parallel_region,
)
from ...utils.tensor_utils import cumsum
from .model_utils import ACT2FN
from .moe_parallel_layers import ExpertFusedColumnParallelLinear, ExpertFusedRowParallelLinear


class Experts(nn.Module):
    """E MLPs with fused 3-D weights: gate_up [E, H, 2I/tp] (GLU) or up [E, H, I/tp], down [E, I/tp, H]."""

    def __init__(self, num_experts: int, hidden_size: int, intermediate_size: int, glu: bool, activation_fn,
                 dtype: torch.dtype = torch.float32, device: Optional[torch.device] = None,
                 input_layer_init_method=None, output_layer_init_method=None):
        super().__init__()
        self.num_experts, self.hidden_size, self.intermediate_size, self.glu = num_experts, hidden_size, \
            intermediate_size, glu
        self.activation_fn = activation_fn
        self.gate_up_proj = ExpertFusedColumnParallelLinear(num_experts, hidden_size,
                                                            (2 if glu else 1) * intermediate_size,
                                                            dtype=dtype, device=device, stride=2 if glu else 1,
                                                            init_method=input_layer_init_method)
        self.down_proj = ExpertFusedRowParallelLinear(num_experts, intermediate_size, hidden_size, reduce_output=False,
                                                      dtype=dtype, device=device,
                                                      init_method=output_layer_init_method)

    def _activation(self, x: torch.Tensor) -> torch.Tensor:
        if self.glu:
            if self.activation_fn is F.silu:
                return ops.swiglu(x)
            g, u = x.chunk(2, dim=-1)
            return self.activation_fn(g) * u
        return self.activation_fn(x)

    def forward(self, hidden_states: torch.Tensor, expert_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        """hidden_states [E or 1, ..., H] -> [E, ..., H] (partial sums over TP)."""
        h = self.gate_up_proj(hidden_states, expert_indices)
        return self.down_proj(self._activation(h), expert_indices)


class ExpertMLPs(nn.Module):
    SELECTIVE_LOADING_THRESHOLD = 1.0

    def __init__(self, num_experts: int, top_k: int, hidden_size: int, intermediate_size: int, hidden_act: str,
                 glu_mlp: bool, capacity_factor: Union[None, float], normalize_top_k_affinities: bool = False,
                 return_bias: bool = False, init_method: Optional[Callable[..., Any]] = None,
                 output_layer_init_method: Optional[Callable[..., Any]] = None, dtype: torch.dtype = torch.float32,
                 device: Optional[torch.device] = None):
        super().__init__()
        if not (0 < top_k <= num_experts):
            raise ValueError(f"Invalid top_k={top_k} for num_experts={num_experts}")
        if hidden_act not in ACT2FN:
            raise ValueError(f"Unknown activation: {hidden_act} ; Supported: {list(ACT2FN)}")
        if capacity_factor is None or capacity_factor >= num_experts / top_k:
            capacity_factor = None
        if normalize_top_k_affinities and top_k == 1:
            raise ValueError("top_k must be greater than 1 for normalizing top-k expert affinities")
        if return_bias:
            raise NotImplementedError("bias is currently unsupported for MoE")
        self.num_experts, self.top_k, self.hidden_size, self.intermediate_size = num_experts, top_k, hidden_size, \
            intermediate_size
        self.act_fn = ACT2FN[hidden_act]
        self.glu_mlp = glu_mlp
        self.capacity_factor = capacity_factor
        self.normalize_top_k_affinities = normalize_top_k_affinities
        self.return_bias = return_bias
        self.mlp_op = Experts(num_experts, hidden_size, intermediate_size, glu_mlp, self.act_fn, dtype=dtype,
                              device=device, input_layer_init_method=init_method,
                              output_layer_init_method=output_layer_init_method)
        self.dtype, self.device = dtype, device
        self.input_grad_reduced_by_caller = False

    def set_input_grad_reduced_by_caller(self, flag: bool = True) -> None:
        """The MoE layer reduces the (TP-partial) input gradient once for router + experts."""
        self.input_grad_reduced_by_caller = flag
        self.mlp_op.gate_up_proj.async_tensor_model_parallel_allreduce = \
            (not flag) and ps.get_tensor_model_parallel_size() > 1
        self.mlp_op.gate_up_proj.skip_input_copy = flag

    # ------------------------------------------------------------------ helpers
    def get_expert_mask(self, expert_index: torch.Tensor) -> torch.Tensor:
        """top_k-hot [T, E] (int32)."""
        mask = torch.zeros(expert_index.shape[0], self.num_experts, device=expert_index.device, dtype=torch.int32)
        mask.scatter_add_(1, expert_index, torch.ones_like(expert_index, dtype=torch.int32))
        return mask

    def get_expert_affinities_masked(self, expert_affinities: torch.Tensor, expert_mask: torch.Tensor) -> torch.Tensor:
        masked = expert_affinities.masked_fill(expert_mask == 0, 0)
        if self.normalize_top_k_affinities:
            masked = F.normalize(masked, p=1.0, dim=1)
        return masked

    def _chosen_affinities(self, expert_affinities, expert_index):
        ch = expert_affinities.gather(1, expert_index)
        if self.normalize_top_k_affinities:
            ch = F.normalize(ch, p=1.0, dim=1)
        return ch

    # ------------------------------------------------------------------ dispatch modes
    def forward_dropless(self, hidden_states, expert_affinities, expert_index):
        """Sort tokens by expert; each expert computes only its own tokens (full capacity)."""
        if ps.get_expert_model_parallel_size() > 1:
            raise NotImplementedError("Expert parallelism requires a capacity factor (static all-to-all shapes)")
        T, H = hidden_states.shape
        k = self.top_k
        if ps.get_tensor_model_parallel_size() > 1 and not self.input_grad_reduced_by_caller:
            # experts are TP-sharded on I: input grads are partial sums over TP
            hidden_states = copy_to_tensor_model_parallel_region(hidden_states)
        # device-side permutation: stable sort of the T*k slots by expert, group offsets by a
        # cumsum of the per-expert counts -- no group size ever reaches the host
        order, inverse, offs = ops.moe_permutation(expert_index, self.num_experts)
        x_sorted = ops.moe_dispatch(hidden_states, order, inverse, k)
        w_gu, w_d = self.mlp_op.gate_up_proj.weight, self.mlp_op.down_proj.weight
        # grouped backend (default): the sync-free grouped kernel; NXD_MOE_GEMM=loop|auto: one host
        # read of the group sizes per layer, per-expert hipBLASLt GEMMs (profiles/r2_moe_layer_v1.md)
        bounds = ops.grouped_gemm.host_group_bounds(offs)
        h = self.mlp_op._activation(ops.grouped_linear(x_sorted, w_gu, offs, bounds))
        y_sorted = ops.grouped_linear(h, w_d, offs, bounds)    # [T*k, H] TP-partial
        # un-permute each (token, choice) slot and take the affinity-weighted sum over k (one kernel)
        aff = self._chosen_affinities(expert_affinities, expert_index)
        return ops.moe_unpermute_combine(y_sorted, inverse, aff)

    def forward_all_experts(self, hidden_states, expert_affinities, expert_index):
        """Every token through every expert (reference semantics; used for tiny batches)."""
        if ps.get_expert_model_parallel_size() > 1:
            raise NotImplementedError("Expert parallelism is not supported without capacity factor.")
        mask = self.get_expert_mask(expert_index)
        aff = self.get_expert_affinities_masked(expert_affinities, mask)
        y = self.mlp_op(hidden_states.unsqueeze(0))            # [E, T, H]
        return torch.einsum("eth,te->th", y, aff.to(y.dtype))

    def forward_capacity_factor(self, hidden_states, expert_affinities, expert_index):
        T, H = hidden_states.shape
        E, k = self.num_experts, self.top_k
        cf = self.capacity_factor if self.capacity_factor is not None else E / k   # None: full capacity
        C = min(T, math.ceil(T * k * cf / E))
        mask = self.get_expert_mask(expert_index)              # [T, E]
        pos = cumsum(mask)                                     # 1-based position in expert
        mask = mask.masked_fill(pos > C, 0)
        aff = self.get_expert_affinities_masked(expert_affinities, mask)
        slot = (pos - 1 + torch.arange(E, device=hidden_states.device, dtype=pos.dtype) * C)
        slot = slot.masked_fill(mask == 0, -1)                 # [T, E] flat slot or -1 if dropped
        tslot = slot.gather(1, expert_index)                   # [T, k]
        assign = torch.full((E * C,), T, dtype=torch.long, device=hidden_states.device)  # T = "empty" row
        valid = tslot >= 0
        tok_ids = torch.arange(T, device=hidden_states.device).unsqueeze(1).expand(T, k)
        assign[tslot[valid].long()] = tok_ids[valid]
        padded = torch.cat([hidden_states, hidden_states.new_zeros(1, H)], 0)
        x = padded[assign].view(E, C, H)
        ep = ps.get_expert_model_parallel_size()
        if ep > 1:
            x = enter_expert_parallel_region(x)                # [E/ep, ep*C, H]
        y = self.mlp_op(x)
        if ep > 1:
            y = exit_expert_parallel_region(y)                 # [E, C, H]
        y = torch.cat([y.reshape(E * C, H), y.new_zeros(1, H)], 0)
        idx = torch.where(valid, tslot.long(), torch.full_like(tslot.long(), E * C))
        a = aff.gather(1, expert_index).to(y.dtype)            # zero for dropped tokens
        out = (y[idx] * a.unsqueeze(-1)).sum(1)
        return out

    def forward_selective_loading(self, hidden_states, expert_affinities, expert_index):
        ch = self._chosen_affinities(expert_affinities, expert_index)
        outs = []
        for t in range(hidden_states.shape[0]):
            y = self.mlp_op(hidden_states[t].view(1, 1, -1), expert_indices=expert_index[t])  # [k, 1, H]
            outs.append((y.squeeze(1) * ch[t].unsqueeze(1).to(y.dtype)).sum(0))
        return torch.stack(outs, 0)

    def forward(self, hidden_states, expert_affinities, expert_index, seq_len: int):
        if ps.get_expert_model_parallel_size() > 1:
            # the EP all-to-all needs static per-expert capacity (full capacity when cf is None)
            return self.forward_capacity_factor(hidden_states, expert_affinities, expert_index)
        if self.training:
            if self.capacity_factor is None:
                return self.forward_dropless(hidden_states, expert_affinities, expert_index)
            return self.forward_capacity_factor(hidden_states, expert_affinities, expert_index)
        T = hidden_states.shape[0]
        if seq_len > 1:   # context encoding
            if self.capacity_factor is None:
                return self.forward_dropless(hidden_states, expert_affinities, expert_index)
            return self.forward_capacity_factor(hidden_states, expert_affinities, expert_index)
        if T * self.top_k / self.num_experts < self.SELECTIVE_LOADING_THRESHOLD:
            return self.forward_selective_loading(hidden_states, expert_affinities, expert_index)
        return self.forward_dropless(hidden_states, expert_affinities, expert_index)
