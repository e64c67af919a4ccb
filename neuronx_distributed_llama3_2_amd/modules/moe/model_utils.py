"""Activation table for MoE MLPs (reference: src/neuronx_distributed/modules/moe/model_utils.py:4-11)."""

import torch
import torch.nn.functional as F

ACT2FN = {
    "gelu": F.gelu,
    "leaky_relu": F.leaky_relu,
    "relu": F.relu,
    "sigmoid": torch.sigmoid,
    "silu": F.silu,
    "tanh": torch.tanh,
}
