"""Training API (reference: src/neuronx_distributed/trainer/)."""

from .post_partition_hooks import PostPartitionHooks

hooks = PostPartitionHooks()

from .checkpoint import (  # noqa: E402,F401
    CheckpointIOState,
    finalize_checkpoint,
    has_checkpoint,
    load_checkpoint,
    save_checkpoint,
)
from .model import NxDModel  # noqa: E402,F401
from .optimizer import NxDOptimizer  # noqa: E402,F401
from .trainer import (  # noqa: E402,F401
    initialize_parallel_model,
    initialize_parallel_optimizer,
    neuronx_distributed_config,
)
