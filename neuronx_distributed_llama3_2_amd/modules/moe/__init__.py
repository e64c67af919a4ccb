"""Mixture of Experts (reference: src/neuronx_distributed/modules/moe/)."""

from .experts import ExpertMLPs, Experts  # noqa: F401
from .loss_function import load_balancing_loss_func  # noqa: F401
from .model import MoE  # noqa: F401
from .model_utils import ACT2FN  # noqa: F401
from .moe_parallel_layers import (  # noqa: F401
    ExpertFusedColumnParallelLinear,
    ExpertFusedLinearWithAsyncCommunication,
    ExpertFusedRowParallelLinear,
    LinearRouter,
    LinearWithWeightGradAR,
)
from .routing import RouterBase, RouterSinkhorn, RouterTopK  # noqa: F401
