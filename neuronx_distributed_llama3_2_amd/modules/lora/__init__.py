"""LoRA (reference: src/neuronx_distributed/modules/lora/)."""

from .config import LoraConfig
from .layer import LoraConv2d, LoraEmbedding, LoraLayer, LoraLinear
from .model import LoraModel
from .tp_layer import LoraGQAQKVParallelLinear, LoraParallelEmbedding, LoraParallelLinear

__all__ = ["LoraConfig", "LoraModel", "get_lora_model", "LoraLayer", "LoraLinear", "LoraEmbedding", "LoraConv2d",
           "LoraParallelLinear", "LoraGQAQKVParallelLinear", "LoraParallelEmbedding"]


def get_lora_model(model, lora_config: LoraConfig):
    if lora_config is None or not lora_config.enable_lora:
        return model
    from ...trainer.model import NxDModel

    if isinstance(model, NxDModel):
        model.module = LoraModel(model.module, lora_config)
        return model
    return LoraModel(model, lora_config)
