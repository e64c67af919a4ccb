from .modeling_mixtral import MixtralDecoderLayer, MixtralForCausalLM, MixtralModel, mixtral_config  # noqa: F401
