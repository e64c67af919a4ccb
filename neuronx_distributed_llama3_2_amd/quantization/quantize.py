"""Module swapping float -> int8 weight-only layers (reference: src/neuronx_distributed/quantization/quantize.py:13-35)."""

from __future__ import annotations

import copy
from typing import Any, Callable, Dict

from .quantization_config import BASE_QCONFIG_DICT_TYPE, get_default_custom_qconfig_dict
from .quantization_mappings import get_default_quant_module_mappings


def convert(module: Any, q_config: BASE_QCONFIG_DICT_TYPE = None, inplace: bool = False,
            mapping: Dict[Callable, Any] = None) -> Any:
    """Replace every mapped layer by its quantized version (float weights, if materialised, are
    quantized symmetric int8 per the q_config; otherwise load an int8 or float state dict later)."""
    if not inplace:
        module = copy.deepcopy(module)
    q_config = q_config or get_default_custom_qconfig_dict()
    mapping = mapping or get_default_quant_module_mappings()
    _swap(module, q_config, mapping)
    return module


def _swap(module, q_config, mapping):
    for name, child in list(module.named_children()):
        if type(child) in mapping:
            module._modules[name] = mapping[type(child)].from_float(child, q_config=q_config)
        else:
            _swap(child, q_config, mapping)
    return module
