"""Token sampling (reference: src/neuronx_distributed/utils/sampling.py:6-77).

Greedy (top_k == 1) runs the row-argmax kernel; top-k multinomial runs the fused radix-select
top-k + softmax + CDF kernel (csrc/inference.hip) with the reference's semantics: softmax over the
k largest logits, cumulative sum, and the sampled index is the number of CDF entries below one
uniform draw.  Both are graph-capturable (the uniform draws can be supplied from a pre-generated
buffer so a captured multi-step decode graph needs no RNG state).
"""

from __future__ import annotations

from typing import Optional

import torch

from .. import ops


class Sampler:
    def __init__(self, config=None, top_k: Optional[int] = None, temperature: float = 1.0, do_sample: Optional[bool] = None):
        self.on_device_sampling = bool(getattr(config, "on_device_sampling", True)) if config is not None else True
        self.is_medusa = bool(getattr(config, "is_medusa", False)) if config is not None else False
        if do_sample is None:
            do_sample = bool(getattr(config, "do_sample", False)) if config is not None else False
        num_beams = int(getattr(config, "num_beams", 1) or 1) if config is not None else 1
        if num_beams != 1:
            raise Exception("Selected sampling method is not supported.")
        k = top_k if top_k is not None else (getattr(config, "top_k", 1) if config is not None else 1)
        self.top_k = int(k) if (do_sample and k) else 1
        self.temperature = float(temperature if temperature is not None else getattr(config, "temperature", 1.0))
        self.sampling_method = self.multinomial

    def sample(self, token_logits: torch.Tensor, uniform: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.sampling_method(token_logits, uniform)

    def multinomial(self, token_logits: torch.Tensor, uniform: Optional[torch.Tensor] = None) -> torch.Tensor:
        """token_logits [B, V] -> token ids [B] (int64)."""
        if self.top_k == 1:
            return ops.argmax_rows(token_logits)
        if self.is_medusa:
            _, _, idx = ops.topk_sample(token_logits, self.top_k, self.temperature, uniform, return_topk=True)
            return idx
        return ops.topk_sample(token_logits, self.top_k, self.temperature, uniform)
