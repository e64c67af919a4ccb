"""Mixtral / DBRX inference applications and runners (reference: examples/inference/mixtral/
{neuron_modeling_mixtral.py:128-340, mixtral_runner.py}, examples/inference/dbrx/{neuron_modeling_dbrx.py,
dbrx_runner.py}, run_mixtral.py, run_dbrx.py).

Same lifecycle as the Llama application (from_pretrained -> compile -> load -> generate, hipGraph
token generation, on-device sampling, speculation), with the MoE device module
(inference/modeling_moe.py).  `capacity_factor` / `glu_mlp` are accepted for parity with the
reference's NeuronMixtralConfig / NeuronDbrxConfig: inference is always dropless (the reference's
capacity_factor=None default) and the experts are GLU.
"""

from __future__ import annotations

import json
import os

from ..models.mixtral.convert import dbrx_hf_to_nxd, dbrx_to_mixtral_config, mixtral_hf_to_nxd
from .config import InferenceConfig
from .generation import LlamaForCausalLMInference
from .modeling_moe import MoEInferenceModel
from .runner import InferenceRunner


def moe_config_from_dir(path: str):
    """config.json of a Mixtral or DBRX directory (or of a compiled MoE model) -> MixtralConfig."""
    from transformers import MixtralConfig

    with open(os.path.join(path, "config.json")) as f:
        d = json.load(f)
    d = {k: v for k, v in d.items() if k not in ("architectures", "transformers_version")}
    if d.get("model_type") == "dbrx":
        return dbrx_to_mixtral_config(d)
    d.pop("model_type", None)
    return MixtralConfig(**d)


class _MoEInferenceBase(LlamaForCausalLMInference):
    _model_cls = MoEInferenceModel

    @staticmethod
    def _config_from_dir(path: str):
        return moe_config_from_dir(path)

    def _quantize(self) -> None:
        raise NotImplementedError("int8 weight-only quantization is implemented for dense decoders only")


class MixtralForCausalLMInference(_MoEInferenceBase):
    @staticmethod
    def _hf_to_nxd(hf_sd, model_config):
        return mixtral_hf_to_nxd(hf_sd, model_config)


class DbrxForCausalLMInference(_MoEInferenceBase):
    @staticmethod
    def _hf_to_nxd(hf_sd, model_config):
        return dbrx_hf_to_nxd(hf_sd, model_config)


NeuronMixtralForCausalLM = MixtralForCausalLMInference
NeuronDbrxForCausalLM = DbrxForCausalLMInference


def _moe_inference_config(capacity_factor=None, glu_mlp=True, **kwargs) -> InferenceConfig:
    if not glu_mlp:
        raise NotImplementedError("Only GLU experts are supported (reference: neuron_modeling_mixtral.py:65)")
    cfg = InferenceConfig(**kwargs)
    cfg.capacity_factor = float(capacity_factor) if capacity_factor is not None else None
    cfg.glu_mlp = glu_mlp
    return cfg


class MixtralRunner(InferenceRunner):
    """reference: examples/inference/mixtral/mixtral_runner.py"""

    app_cls = MixtralForCausalLMInference

    def load_hf_model(self):
        from transformers import MixtralForCausalLM

        return MixtralForCausalLM.from_pretrained(self.model_path)

    def get_config_for_nxd(self, batch_size: int, tp_degree: int, max_prompt_length: int, sequence_length: int,
                           enable_bucketing: bool = False, **kwargs) -> InferenceConfig:
        return _moe_inference_config(tp_degree=tp_degree, batch_size=batch_size, seq_len=sequence_length,
                                     max_context_length=max_prompt_length, enable_bucketing=enable_bucketing, **kwargs)

    def get_model_config(self):
        return moe_config_from_dir(self.model_path)


class DbrxRunner(MixtralRunner):
    """reference: examples/inference/dbrx/dbrx_runner.py"""

    app_cls = DbrxForCausalLMInference

    def load_hf_model(self):
        from transformers import DbrxForCausalLM

        return DbrxForCausalLM.from_pretrained(self.model_path)
