"""Mixture-of-Experts layer (reference: src/neuronx_distributed/modules/moe/model.py:7-160).

hidden [S(/tp), B, H] (training, SP shard) or [B, S, H] (inference) -> same shape; the router and
the expert dispatch see the full token set (SP is exited with an all-gather and re-entered with a
reduce-scatter of the TP-partial expert outputs, exactly like a dense TP MLP).
"""

from __future__ import annotations

import torch

from ...parallel_layers import mappings
from ...parallel_layers import parallel_state as ps
from .experts import ExpertMLPs
from .routing import RouterBase


class MoE(torch.nn.Module):
    is_test = False

    def __init__(self, router: RouterBase, expert_mlps: ExpertMLPs, sequence_parallel_enabled: bool = False,
                 return_router_logits: bool = False):
        super().__init__()
        for attr in ("num_experts", "top_k", "hidden_size"):
            if getattr(router, attr) != getattr(expert_mlps, attr):
                raise ValueError(f"Inconsistent {attr} across the router and expert_mlps")
        self.router = router
        self.expert_mlps = expert_mlps
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.return_router_logits = return_router_logits
        self.ep_enabled = ps.get_expert_model_parallel_size() > 1
        if ps.get_tensor_model_parallel_size() > 1:
            # router + experts both see TP-partial gradients: reduce the input grad ONCE here
            self.expert_mlps.set_input_grad_reduced_by_caller(True)
            self.router.linear_router.reduce_weight_grad = True

    def forward(self, hidden_states: torch.Tensor):
        if not self.training:
            assert not self.sequence_parallel_enabled, "SP is not currently supported for inference"
        sp = self.sequence_parallel_enabled and ps.get_tensor_model_parallel_size() > 1
        if sp:   # backward: reduce-scatter of the TP-partial input grads
            full = mappings.gather_from_sequence_parallel_region(hidden_states, to_model_parallel=True)
        elif ps.get_tensor_model_parallel_size() > 1:
            full = mappings.copy_to_tensor_model_parallel_region(hidden_states)
        else:
            full = hidden_states
        shape = full.shape
        seq_len = shape[0] if self.training else shape[1]
        x = full.reshape(-1, shape[-1])
        router_logits, expert_affinities, expert_index = self.router(x)
        out = self.expert_mlps(hidden_states=x, expert_affinities=expert_affinities, expert_index=expert_index,
                               seq_len=seq_len)
        out = out.view(shape)
        if sp:
            out = mappings.reduce_scatter_to_sequence_parallel_region(out)
        elif ps.get_tensor_model_parallel_size() > 1:
            out = mappings.reduce_from_tensor_model_parallel_region(out)
        res = (out,)
        if self.return_router_logits:
            res += (router_logits,)
        if self.is_test:
            res += (expert_index,)
        return res[0] if len(res) == 1 else res
