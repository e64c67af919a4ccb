"""Inference trace / SPMD runtime API (reference: src/neuronx_distributed/trace/__init__.py)."""

from .model_builder import BaseModelInstance, ModelBuilder, ModelContainer  # noqa: F401
from .spmd import GraphRunner, NxDModel, NxDModelExecutor, SPMDBucketModel, SPMDBucketModelScript, StateInitializer  # noqa: F401
from .trace import (  # noqa: F401
    ParallelModel,
    TensorParallelModel,
    TensorParallelNeuronModel,
    create_local_weight,
    create_local_weight_qkv,
    get_sharded_checkpoint,
    parallel_model_load,
    parallel_model_save,
    parallel_model_trace,
    shard_children,
)
