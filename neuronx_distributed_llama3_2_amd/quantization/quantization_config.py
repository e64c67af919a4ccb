"""Quantization config types (reference: src/neuronx_distributed/quantization/quantization_config.py:9-57)."""

import enum
from enum import Enum
from typing import TypedDict

import torch


class _ContainsEnumMeta(enum.EnumMeta):
    def __contains__(cls, item):
        try:
            cls(item)
        except ValueError:
            return False
        return True


class QuantizationType(Enum, metaclass=_ContainsEnumMeta):
    PER_TENSOR_SYMMETRIC = "per_tensor_symmetric"
    PER_CHANNEL_SYMMETRIC = "per_channel_symmetric"


class QuantizedDtype(Enum, metaclass=_ContainsEnumMeta):
    INT8 = torch.int8


class BASE_QCONFIG_DICT_TYPE(TypedDict):
    quantization_type: QuantizationType
    quantized_dtype: QuantizedDtype


class PER_CHANNEL_QCONFIG_DICT_TYPE(BASE_QCONFIG_DICT_TYPE):
    quantization_per_channel_axis: int


_DEFAULT_CUSTOM_QCONFIG_DICT: BASE_QCONFIG_DICT_TYPE = {
    "quantization_type": QuantizationType.PER_TENSOR_SYMMETRIC,
    "quantized_dtype": QuantizedDtype.INT8,
}
_DEFAULT_PER_CHANNEL_QCONFIG_DICT: PER_CHANNEL_QCONFIG_DICT_TYPE = {
    "quantization_type": QuantizationType.PER_CHANNEL_SYMMETRIC,
    "quantized_dtype": QuantizedDtype.INT8,
    "quantization_per_channel_axis": 0,
}


def get_default_custom_qconfig_dict() -> BASE_QCONFIG_DICT_TYPE:
    return dict(_DEFAULT_CUSTOM_QCONFIG_DICT)


def get_default_per_channel_custom_qconfig_dict() -> PER_CHANNEL_QCONFIG_DICT_TYPE:
    return dict(_DEFAULT_PER_CHANNEL_QCONFIG_DICT)
