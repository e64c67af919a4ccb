"""Llama-3 / 3.1 / 3.2 inference model: tensor-parallel, persistent KV cache, fused CDNA4 kernels
(reference: examples/inference/llama3/neuron_modeling_llama.py:117-446).

The module IS the training `LlamaForCausalLM` (same parameter names, so training checkpoints and
converted HF weights load directly) with the shared inference forward of `model_base` and a dense
SwiGLU feed-forward: gate_up GEMM (or, at decode sizes, the skinny-GEMM kernel with SwiGLU fused
into its epilogue) -> down projection (+ TP all-reduce).
"""

from __future__ import annotations

import copy

import torch

from ..models.llama.modeling_llama import LlamaForCausalLM
from .model_base import DecoderInferenceMixin


class LlamaInferenceModel(DecoderInferenceMixin, LlamaForCausalLM):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        cfg = copy.copy(config)
        cfg.sequence_parallel_enabled = False
        LlamaForCausalLM.__init__(self, cfg, dtype=dtype, device=device)
        self._init_inference(config)

    def _fused_ffn_weights(self, layer):
        mlp = layer.mlp
        w_gu, w_d = mlp.gate_up_proj.weight, mlp.down_proj.weight
        if w_gu.dtype != torch.bfloat16 or w_d.dtype != torch.bfloat16 or \
                getattr(mlp.gate_up_proj, "bias", None) is not None or getattr(mlp.down_proj, "bias", None) is not None:
            return None
        return layer.post_attention_layernorm.weight, w_gu, w_d

    def _ffn(self, layer, h: torch.Tensor) -> torch.Tensor:
        mlp = layer.mlp
        a = self._proj(mlp.gate_up_proj, h, glu=True)   # SwiGLU fused into the decode GEMV
        return self._row(mlp.down_proj, a)
