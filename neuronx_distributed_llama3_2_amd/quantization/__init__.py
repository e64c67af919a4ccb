"""int8 weight-only quantization (reference: src/neuronx_distributed/quantization/)."""

from .dequantize import direct_cast_dequantize, scale_dequantize  # noqa: F401
from .observer import PerChannelAbsMaxObserver  # noqa: F401
from .quantization_config import (  # noqa: F401
    QuantizationType,
    QuantizedDtype,
    get_default_custom_qconfig_dict,
    get_default_per_channel_custom_qconfig_dict,
)
from .quantization_layers import (  # noqa: F401
    BaseQuantizeParallelLinear,
    QuantizedColumnParallel,
    QuantizedExpertFusedColumnParallel,
    QuantizedExpertFusedRowParallel,
    QuantizedParallelLinearLayerStateDictAdaptor,
    QuantizedRowParallel,
    quantize_symmetric,
)
from .quantization_utils import (  # noqa: F401
    convert_qint8_to_int8_state_dict,
    quantize_pytorch_model_per_channel_symmetric,
    quantize_pytorch_model_per_tensor_symmetric,
)
from .quantize import convert  # noqa: F401
