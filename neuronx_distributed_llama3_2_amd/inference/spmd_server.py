"""Resident single-controller generation over TP ranks (reference trace/spmd.py:82-187 +
trace/model_builder.py:380-451: one controller drives every rank's per-bucket compiled graphs,
weights and KV state stay on the devices).

Each rank is a worker process of trace/runtime.SpmdWorkerPool that owns its weight shard, its KV
cache and its captured prefill / decode hipGraphs for the life of the server.  `generate()` sends
the prompt token ids to every rank and gets the generated ids back from rank 0: the ranks run the
whole prefill + decode loop on their devices (collectives meet over RCCL, on-device sampling), so
the host traffic of a call is O(tokens) -- ids in, ids out, no activations or logits -- which
`last_host_bytes` reports.

    server = SpmdGenerationServer.from_compiled("traced_model/", tp_degree=2)   # LlamaForCausalLMInference.compile output
    out = server.generate(input_ids, max_new_tokens=64)
    server.close()
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from ..trace.runtime import SpmdWorkerPool

_DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}


def _build_compiled(rank: int, world: int, path: str, dtype: str, app: str):
    from . import LlamaForCausalLMInference

    cls = LlamaForCausalLMInference
    if app != "llama":
        from . import moe as _moe

        cls = getattr(_moe, app)
    return cls.load(path, dtype=_DTYPES[dtype])


def _build_from_full(rank: int, world: int, model_config: Dict[str, Any], full_sd_path: str,
                     inference_kwargs: Dict[str, Any], dtype: str):
    from transformers import LlamaConfig

    from . import InferenceConfig, LlamaForCausalLMInference

    cfg = LlamaConfig(**model_config)
    icfg = InferenceConfig(tp_degree=world, **inference_kwargs)
    m = LlamaForCausalLMInference(cfg, icfg, dtype=_DTYPES[dtype], init_weights=False)
    m._load_full(torch.load(full_sd_path, map_location="cpu", weights_only=True))
    return m


class SpmdGenerationServer:
    def __init__(self, pool: SpmdWorkerPool, config=None):
        self.pool = pool
        self.config = config      # InferenceConfig of the served model (runners read max_length etc.)

    @classmethod
    def from_compiled(cls, path: str, tp_degree: int, dtype: str = "bfloat16", app: str = "llama"):
        """Workers load the per-rank shards written by `compile()` (tp{r}_sharded_checkpoint.safetensors)."""
        from .config import InferenceConfig

        return cls(SpmdWorkerPool(tp_degree, _build_compiled, (path, dtype, app)), InferenceConfig.from_pretrained(path))

    @classmethod
    def from_full_state_dict(cls, model_config: Dict[str, Any], full_sd_path: str, tp_degree: int,
                             inference_kwargs: Optional[Dict[str, Any]] = None, dtype: str = "bfloat16"):
        """Workers shard a framework-named full state dict (torch.save file) themselves."""
        return cls(SpmdWorkerPool(tp_degree, _build_from_full,
                                  (model_config, full_sd_path, dict(inference_kwargs or {}), dtype)))

    def generate(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None, **kwargs) -> torch.Tensor:
        if kwargs.get("assistant_model") is not None:
            raise NotImplementedError("assisted decoding through the SPMD server: load the draft inside the workers")
        kwargs.pop("assistant_model", None)
        args = (input_ids.to(torch.int64).cpu(),) + ((attention_mask.cpu(),) if attention_mask is not None else ())
        return self.pool.call("generate", *args, **kwargs)

    @property
    def last_host_bytes(self) -> int:
        return self.pool.last_host_bytes

    def close(self) -> None:
        self.pool.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
