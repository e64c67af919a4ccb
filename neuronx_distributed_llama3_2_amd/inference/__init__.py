"""Inference stack: TP Llama and MoE (Mixtral, DBRX) with persistent KV cache, hipGraph-captured decode loop, on-device
sampling, bucketing, benchmark/report and runner (reference: examples/inference/, src/.../trace/)."""

from .bucketing import generate_buckets, select_bucket  # noqa: F401
from .config import InferenceConfig, NeuronInferenceConfig  # noqa: F401
from .generation import LlamaForCausalLMInference, load_hf_state_dict  # noqa: F401
from .modeling_llama import LlamaInferenceModel  # noqa: F401
from .model_base import DecoderInferenceMixin  # noqa: F401
from .modeling_moe import MoEInferenceModel  # noqa: F401
from .moe import DbrxForCausalLMInference, DbrxRunner, MixtralForCausalLMInference, MixtralRunner  # noqa: F401
