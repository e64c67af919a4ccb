"""AdamW with fp32 optimizer state for low-precision parameters
(reference: src/neuronx_distributed/utils/adamw_fp32_optim_params.py:31-155).

The reference keeps Adam moments in fp64 only to survive XLA_DOWNCAST_BF16; here the moments
are fp32 and the per-tensor update runs the fused CDNA4 AdamW kernel (ops.adamw_flat_) on GPU
tensors.  Inside `initialize_parallel_optimizer` / NeuronZero1Optimizer this class is recognised
and replaced by the flat-buffer implementation (one kernel per bucket instead of per tensor).
"""

from __future__ import annotations

import math

import torch
from torch.optim import Optimizer

from .. import ops


class AdamW_FP32OptimParams(Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-6, weight_decay: float = 0.0,
                 correct_bias: bool = True, no_decay_params=None):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, correct_bias=correct_bias)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                g = getattr(p, "main_grad", None)
                g = p.grad if g is None else g
                if g is None:
                    continue
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                    state["exp_avg_sq"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                    if p.dtype != torch.float32:
                        state["master"] = p.detach().float().reshape(-1).clone()
                state["step"] += 1
                b1, b2 = group["betas"]
                master = state.get("master")
                if master is not None:
                    ops.adamw_flat_(master, g.detach().reshape(-1).contiguous(), state["exp_avg"], state["exp_avg_sq"],
                                    None, group["lr"], b1, b2, group["eps"], group["weight_decay"], state["step"],
                                    bias_correction=group["correct_bias"])
                    p.data.copy_(master.view_as(p))
                else:
                    flat = p.data.view(-1)
                    ops.adamw_flat_(flat, g.detach().reshape(-1).contiguous(), state["exp_avg"], state["exp_avg_sq"], None,
                                    group["lr"], b1, b2, group["eps"], group["weight_decay"], state["step"],
                                    bias_correction=group["correct_bias"])
        return loss
