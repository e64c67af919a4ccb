"""Tensor/sequence-parallel building blocks (reference: src/neuronx_distributed/parallel_layers/__init__.py)."""

from . import parallel_state  # noqa: F401
from .checkpointing import load, save  # noqa: F401
from .grads import clip_grad_norm  # noqa: F401
from .layers import ColumnParallelLinear, ParallelEmbedding, RowParallelLinear  # noqa: F401
from .layers import InputChannelParallelConv2d, OutputChannelParallelConv2d  # noqa: F401
from .loss_functions import parallel_cross_entropy  # noqa: F401
from .mappings import (  # noqa: F401
    copy_to_tensor_model_parallel_region,
    gather_from_tensor_model_parallel_region,
    reduce_from_tensor_model_parallel_region,
    scatter_to_tensor_model_parallel_region,
)
from .parallel_state import initialize_model_parallel  # noqa: F401
from .random import get_rng_tracker, get_xla_rng_tracker, model_parallel_manual_seed, model_parallel_xla_manual_seed  # noqa: F401
from .utils import (  # noqa: F401
    copy_tensor_model_parallel_attributes,
    move_model_to_device,
    set_defaults_if_not_set_tensor_model_parallel_attributes,
    set_tensor_model_parallel_attributes,
    split_tensor_along_last_dim,
)

# modules / functions treated as leaves when the pipeline tracer partitions a model
PARALLEL_MODULES = [ColumnParallelLinear, RowParallelLinear, ParallelEmbedding]
PARALLEL_FUNCTIONS = [
    parallel_cross_entropy,
    copy_to_tensor_model_parallel_region,
    gather_from_tensor_model_parallel_region,
    reduce_from_tensor_model_parallel_region,
    scatter_to_tensor_model_parallel_region,
]
