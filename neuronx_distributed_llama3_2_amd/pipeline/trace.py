"""Symbolic tracing of a model for pipeline partitioning
(reference: src/neuronx_distributed/pipeline/trace.py:32-217).

torch.fx tracing with the transformer-layer class, the tensor-parallel layers, norms and any
user `leaf_module_cls` kept as leaves (their internals — HIP kernels, RCCL collectives — are never
traced), and the parallel loss / mapping functions auto-wrapped as leaf calls.
"""

from __future__ import annotations

import inspect
from typing import Any, Dict, List, Optional, Sequence, Type

import torch
import torch.fx as fx


def _default_leaf_classes():
    from ..modules.qkv_linear import GQAQKVColumnParallelLinear
    from ..parallel_layers import PARALLEL_MODULES
    from ..parallel_layers.layer_norm import LayerNorm, RMSNorm

    return list(PARALLEL_MODULES) + [GQAQKVColumnParallelLinear, RMSNorm, LayerNorm]


def _default_autowrap_functions():
    from ..parallel_layers import PARALLEL_FUNCTIONS

    return list(PARALLEL_FUNCTIONS)


class NxDTracer(fx.Tracer):
    def __init__(self, leaf_modules: Sequence[Type[torch.nn.Module]] = (), autowrap_functions=(), autowrap_modules=(),
                 **kwargs):
        import math

        super().__init__(autowrap_modules=(math,) + tuple(autowrap_modules), autowrap_functions=tuple(autowrap_functions))
        self._leaf = tuple(leaf_modules)

    def is_leaf_module(self, m: torch.nn.Module, qualname: str) -> bool:
        if isinstance(m, self._leaf):
            return True
        return super().is_leaf_module(m, qualname)


def get_concrete_args(model: torch.nn.Module, input_names: Optional[List[str]]) -> Dict[str, Any]:
    """Every forward argument not in `input_names` is frozen to its default value."""
    sig = inspect.signature(model.forward)
    if input_names is None:
        return {}
    concrete = {}
    for name, p in sig.parameters.items():
        if name in input_names or p.kind in (inspect.Parameter.VAR_POSITIONAL, inspect.Parameter.VAR_KEYWORD):
            continue
        concrete[name] = p.default if p.default is not inspect.Parameter.empty else None
    return concrete


def trace_model(model: torch.nn.Module, input_names: Optional[List[str]] = None,
                leaf_modules: Sequence[Type[torch.nn.Module]] = (), autowrap_functions: Sequence = (),
                autowrap_modules: Sequence = (), tracer_cls=None) -> fx.GraphModule:
    leaves = list(leaf_modules) + _default_leaf_classes()
    wraps = list(autowrap_functions) + _default_autowrap_functions()
    tracer = (tracer_cls or NxDTracer)(leaf_modules=leaves, autowrap_functions=wraps, autowrap_modules=autowrap_modules)
    concrete = get_concrete_args(model, input_names)
    graph = tracer.trace(model, concrete_args=concrete or None)
    gm = fx.GraphModule(tracer.root, graph, model.__class__.__name__)
    gm.graph.eliminate_dead_code()
    gm.recompile()
    return gm
