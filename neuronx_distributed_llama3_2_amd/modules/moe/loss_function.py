"""Switch-Transformer load-balancing loss (reference: src/neuronx_distributed/modules/moe/loss_function.py:5-48)."""

import torch
import torch.nn.functional as F


def load_balancing_loss_func(router_logits: torch.Tensor, num_experts: int, top_k: int) -> torch.Tensor:
    """router_logits: [tokens * layers, E] -> E/top_k * sum_e f_e * P_e (f: routed fraction per
    top-k slot, P: mean router probability)."""
    aff = F.softmax(router_logits, dim=-1, dtype=torch.float32)
    _, sel = torch.topk(aff, top_k)
    mask = F.one_hot(sel, num_experts).float()          # [N, top_k, E]
    tokens_per_expert = mask.mean(0)                     # [top_k, E]
    prob_per_expert = aff.mean(0)                        # [E]
    return (tokens_per_expert * prob_per_expert.unsqueeze(0)).sum() * (num_experts / top_k)
