"""Float -> quantized module mapping (reference: src/neuronx_distributed/quantization/quantization_mappings.py:11-16)."""

from typing import Any, Callable, Dict

from ..modules.moe import moe_parallel_layers
from ..parallel_layers import layers as parallel_layers
from . import quantization_layers as q_layers

DEFAULT_QUANT_MODULE_MAPPINGS: Dict[Callable, Any] = {
    parallel_layers.ColumnParallelLinear: q_layers.QuantizedColumnParallel,
    parallel_layers.RowParallelLinear: q_layers.QuantizedRowParallel,
    moe_parallel_layers.ExpertFusedColumnParallelLinear: q_layers.QuantizedExpertFusedColumnParallel,
    moe_parallel_layers.ExpertFusedRowParallelLinear: q_layers.QuantizedExpertFusedRowParallel,
}


def get_default_quant_module_mappings() -> Dict[Callable, Any]:
    return DEFAULT_QUANT_MODULE_MAPPINGS
