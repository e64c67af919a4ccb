"""Inference configuration (reference: examples/inference/modules/config.py:4-67 `NeuronInferenceConfig`,
examples/inference/llama3/neuron_modeling_llama.py `NeuronLlamaConfig`).

Same attribute names as the reference (tp_degree, batch_size, n_positions / max_length,
max_context_length, max_new_tokens, ctx/tkg batch sizes, continuous batching, on-device sampling,
bucketing, quantization, speculation, Medusa) plus the MI355X runtime knobs:

* `decode_graph_steps` — decode steps captured per hipGraph replay (the whole token loop runs on
  the device: sampling, next-token feed-back and position updates are inside the graph);
* `use_hip_graphs` — capture decode graphs at all (eager fallback for debugging).
* `prefill_graphs` — also capture the context-encoding forward per (batch, bucket).
"""

from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional

from .bucketing import generate_buckets


class InferenceConfig:
    def __init__(self, tp_degree: int = 1, batch_size: int = 1, seq_len: int = 128, padding_side: str = "right",
                 **kwargs):
        self.tp_degree = tp_degree
        self.batch_size = batch_size
        self.padding_side = padding_side
        self.n_active_tokens = seq_len
        self.n_positions = seq_len
        self.max_context_length = kwargs.pop("max_context_length", seq_len)
        self.max_new_tokens = seq_len - self.max_context_length or None
        self.max_length = seq_len
        self.ctx_batch_size = kwargs.pop("ctx_batch_size", batch_size)
        self.tkg_batch_size = kwargs.pop("tkg_batch_size", batch_size)
        self.max_batch_size = kwargs.pop("max_batch_size", batch_size)
        self.is_continuous_batching = kwargs.pop("is_continuous_batching", False)
        self.on_device_sampling = kwargs.pop("on_device_sampling", True)
        self.enable_bucketing = kwargs.pop("enable_bucketing", False)
        self.buckets: List[int] = kwargs.pop("buckets", None) or (
            generate_buckets(min(128, self.max_context_length), self.max_context_length) if self.enable_bucketing
            else [self.max_context_length])
        self.token_generation_buckets: List[int] = kwargs.pop("token_generation_buckets", None) or [seq_len]
        self.bucket_n_active_tokens = False
        self.quantized = kwargs.pop("quantized", False)
        self.quantized_checkpoints_path = kwargs.pop("quantized_checkpoints_path", None)
        self.quantization_type = kwargs.pop("quantization_type", "per_tensor_symmetric")
        self.trace_tokengen_model = kwargs.pop("trace_tokengen_model", True)
        self.speculation_length = kwargs.pop("speculation_length", 0)
        self.spec_rounds_per_graph = kwargs.pop("spec_rounds_per_graph", 4)
        self.spec_batch_size = batch_size
        self.is_medusa = kwargs.pop("is_medusa", False)
        self.medusa_speculation_length = kwargs.pop("medusa_speculation_length", 0)
        self.num_medusa_heads = kwargs.pop("num_medusa_heads", 0)
        self.medusa_tree = kwargs.pop("medusa_tree", None)
        self.do_sample = kwargs.pop("do_sample", False)
        self.top_k = kwargs.pop("top_k", 1)
        self.temperature = kwargs.pop("temperature", 1.0)
        self.num_beams = kwargs.pop("num_beams", 1)
        self.use_hip_graphs = kwargs.pop("use_hip_graphs", True)
        # bitwise-reproducible decode: no fp32-atomic fused attention + o_proj launch (model_base.py)
        self.deterministic = kwargs.pop("deterministic", False)
        # context encoding captured per (batch, bucket) hipGraph as well (needs use_hip_graphs)
        self.prefill_graphs = kwargs.pop("prefill_graphs", True)
        # GQA sharding (modules/gqa.py): "replicate-to-tp-degree" (default) | "convert-to-mha"
        self.gqa_sharding_strategy = kwargs.pop("gqa_sharding_strategy", None)
        # measured weight-layout pass at the context-encoding size (trace/weight_layout.py)
        self.weight_layout_optimization = kwargs.pop("weight_layout_optimization", False)
        self.decode_graph_steps = kwargs.pop("decode_graph_steps", 16)
        self.torch_dtype = kwargs.pop("torch_dtype", "bfloat16")
        self.generation_config: Dict[str, Any] = kwargs.pop("generation_config", None) or {"max_length": seq_len}
        self.extra = dict(kwargs)  # model-architecture fields (hidden_size, ...) when merged with an HF config
        for k, v in kwargs.items():
            setattr(self, k, v)

    # ------------------------------------------------------------------ (de)serialisation
    def to_dict(self) -> Dict[str, Any]:
        d = {k: v for k, v in self.__dict__.items() if k != "extra"}
        d["seq_len"] = self.max_length
        return d

    def save_pretrained(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "nxd_inference_config.json"), "w") as f:
            json.dump(self.to_dict(), f, indent=2, default=str)

    @classmethod
    def from_pretrained(cls, path: str) -> "InferenceConfig":
        with open(os.path.join(path, "nxd_inference_config.json")) as f:
            d = json.load(f)
        seq_len = d.pop("seq_len")
        base = {k: d.pop(k) for k in ("tp_degree", "batch_size", "padding_side") if k in d}
        for k in ("n_active_tokens", "n_positions", "max_new_tokens", "max_length", "spec_batch_size",
                  "bucket_n_active_tokens"):
            d.pop(k, None)
        return cls(seq_len=seq_len, **base, **d)


NeuronInferenceConfig = InferenceConfig


def model_config_from_dir(path: str):
    """HF `LlamaConfig` from a model directory's config.json (no network)."""
    from transformers import LlamaConfig

    with open(os.path.join(path, "config.json")) as f:
        d = json.load(f)
    return LlamaConfig(**{k: v for k, v in d.items() if k not in ("architectures", "transformers_version")})
