"""MoE routers (reference: src/neuronx_distributed/modules/moe/routing.py:9-218).

Same contract: forward(hidden [T, H]) -> (router_logits [T, E], expert_affinities [T, E],
expert_index [T, top_k]).  Affinities are computed in fp32 (the reference's fp64 only guards
against XLA's bf16 auto-downcast); Sinkhorn balancing runs a fixed number of fp32 iterations.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import torch
import torch.nn.functional as F

from .moe_parallel_layers import LinearRouter


class RouterBase(torch.nn.Module, ABC):
    def __init__(self, num_experts: int, top_k: int, hidden_size: int, act_fn: str, dtype: torch.dtype,
                 device: torch.device):
        super().__init__()
        if not (0 < top_k <= num_experts):
            raise ValueError(f"Invalid top_k={top_k} for num_experts={num_experts}")
        if act_fn not in ("sigmoid", "softmax"):
            raise ValueError("act_fn must be either 'sigmoid' or 'softmax'")
        self.num_experts, self.top_k, self.hidden_size, self.act_fn = num_experts, top_k, hidden_size, act_fn
        self.dtype, self.device = dtype, device
        self.linear_router = LinearRouter(input_size=hidden_size, output_size=num_experts, dtype=dtype, device=device)

    def get_router_logits_and_expert_affinities(self, hidden_states: torch.Tensor):
        router_logits = self.linear_router(hidden_states)
        if self.act_fn == "sigmoid":
            aff = torch.sigmoid(router_logits.float())
        else:
            aff = F.softmax(router_logits, dim=1, dtype=torch.float32)
        return router_logits, aff.to(hidden_states.dtype)

    @abstractmethod
    def forward(self, hidden_states: torch.Tensor):
        ...


class RouterTopK(RouterBase):
    """Softmax affinities, top-k experts per token by logit (pair with load_balancing_loss_func)."""

    def __init__(self, num_experts: int, top_k: int, hidden_size: int, dtype: torch.dtype = torch.float32,
                 device: torch.device = torch.device("cpu")):
        super().__init__(num_experts, top_k, hidden_size, "softmax", dtype, device)

    def forward(self, hidden_states):
        router_logits, aff = self.get_router_logits_and_expert_affinities(hidden_states)
        _, expert_index = torch.topk(router_logits, self.top_k)
        return router_logits, aff, expert_index.detach().long()


class RouterSinkhorn(RouterBase):
    """Top-1 routing on Sinkhorn-balanced logits during training (fixed iteration count)."""

    DEFAULT_SINKHORN_ITERS = 30

    def __init__(self, num_experts: int, top_k: int, hidden_size: int, act_fn: str = "sigmoid",
                 dtype: torch.dtype = torch.float32, device: torch.device = torch.device("cpu"),
                 sinkhorn_iterations: Optional[int] = None, sinkhorn_tol: Optional[float] = None):
        if top_k != 1:
            raise NotImplementedError("RouterSinkhorn only supports Top-1 routing")
        super().__init__(num_experts, top_k, hidden_size, act_fn, dtype, device)
        self.sinkhorn_iterations = sinkhorn_iterations if sinkhorn_iterations is not None else self.DEFAULT_SINKHORN_ITERS
        self.sinkhorn_tol = sinkhorn_tol

    def forward(self, hidden_states):
        router_logits, aff = self.get_router_logits_and_expert_affinities(hidden_states)
        with torch.no_grad():
            route = (self._sinkhorn(router_logits.detach().float(), self.sinkhorn_iterations, self.sinkhorn_tol)
                     if self.training else router_logits.detach())
            expert_index = torch.argmax(route, dim=1, keepdim=True)
        return router_logits, aff, expert_index.long()

    @staticmethod
    def _sinkhorn(cost: torch.Tensor, num_iters: int, tol: Optional[float] = None) -> torch.Tensor:
        """Alternating row/column normalisation of exp(cost) (Megatron-style, fixed iterations)."""
        if num_iters == 0:
            return cost
        cost = torch.exp(cost - cost.max())
        d0 = torch.ones(cost.shape[0], device=cost.device, dtype=cost.dtype)
        d1 = torch.ones(cost.shape[1], device=cost.device, dtype=cost.dtype)
        eps = 1e-8
        d1_old = d1
        for _ in range(num_iters):
            d0 = (1.0 / d0.shape[0]) / (torch.sum(d1 * cost, 1) + eps)
            d1 = (1.0 / d1.shape[0]) / (torch.sum(d0.unsqueeze(1) * cost, 0) + eps)
            if tol is not None:
                err = torch.mean(torch.abs(d1_old - d1))
                d1_old = d1
        if tol is not None:
            assert float(err) < tol, f"Sinkhorn error {float(err)} above tolerance {tol}"
        return d1 * cost * d0.unsqueeze(1)
