"""Training API: `neuronx_distributed_config`, `initialize_parallel_model`, `initialize_parallel_optimizer`
(reference: src/neuronx_distributed/trainer/trainer.py:33-303; same config keys and defaults).

Model construction on MI355X: the model is built on the GPU directly (or on the meta device with
`model_init_config.meta_device_init` and materialised shard-by-shard with `param_init_fn`), wrapped
in NxDPPModel when pipeline parallel, optionally LoRA-ed / head-padded / activation-checkpointed.
Optimizers: with `zero_one_enabled` (or `use_master_weights`) the flat-buffer ZeRO-1 path
(fp32 master weights, fp32 grad accumulation, fused AdamW kernel); otherwise the user's optimizer
class on the parameters as-is.
"""

from __future__ import annotations

import os
from pprint import pformat
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state
from ..parallel_layers.pad import pad_model
from ..utils.activation_checkpoint import apply_activation_checkpointing
from ..utils.logger import get_logger
from ..utils.model_utils import get_model_sequential, init_on_device, is_hf_pretrained_model
from .model import NxDModel
from .optimizer import NxDOptimizer

logger = get_logger()


def _default(d: Dict[str, Any], key: str, value, warn: bool = True):
    if key not in d:
        if warn and parallel_state.is_global_rank_zero():
            logger.warning("%s is not set, automatically set it to %s.", key, value)
        d[key] = value


def neuronx_distributed_config(tensor_parallel_size: int = 1, pipeline_parallel_size: int = 1,
                               expert_parallel_size: int = 1, pipeline_config: Optional[dict] = None,
                               optimizer_config: Optional[dict] = None, activation_checkpoint_config=None,
                               pad_model: bool = False, sequence_parallel: bool = False,
                               model_init_config: Optional[dict] = None, lora_config=None,
                               mixed_precision_config: Optional[dict] = None) -> Dict[str, Any]:
    if optimizer_config is None:
        optimizer_config = {"zero_one_enabled": False, "grad_clipping": True, "max_grad_norm": 1.0}
    else:
        assert isinstance(optimizer_config, dict), "optimizer_config must be a dict."
        _default(optimizer_config, "zero_one_enabled", False)
        _default(optimizer_config, "grad_clipping", True)
        if optimizer_config["grad_clipping"]:
            _default(optimizer_config, "max_grad_norm", 1.0)
    if mixed_precision_config is None:
        mixed_precision_config = {"use_master_weights": optimizer_config["zero_one_enabled"],
                                  "use_fp32_grad_acc": optimizer_config["zero_one_enabled"],
                                  "use_master_weights_in_ckpt": False}
    else:
        assert isinstance(mixed_precision_config, dict), "mixed_precision_config must be a dict."
        _default(mixed_precision_config, "use_master_weights", optimizer_config["zero_one_enabled"])
        _default(mixed_precision_config, "use_fp32_grad_acc", optimizer_config["zero_one_enabled"])
        _default(mixed_precision_config, "use_master_weights_in_ckpt", False)
    if model_init_config is None:
        model_init_config = {"sequential_move_factor": 11, "meta_device_init": False, "param_init_fn": None}
    else:
        assert isinstance(model_init_config, dict), "model_init_config must be a dict."
        _default(model_init_config, "sequential_move_factor", 11)
        _default(model_init_config, "meta_device_init", False)
        if model_init_config["meta_device_init"] and "param_init_fn" not in model_init_config:
            raise ValueError("param_init_fn must be provided when meta_device_init is True")
    config = {
        "tensor_parallel_size": tensor_parallel_size,
        "pipeline_parallel_size": pipeline_parallel_size,
        "expert_parallel_size": expert_parallel_size,
        "pipeline_config": pipeline_config,
        "optimizer_config": optimizer_config,
        "activation_checkpoint_config": activation_checkpoint_config,
        "pad_model": pad_model,
        "sequence_parallel": sequence_parallel,
        "model_init_config": model_init_config,
        "lora_config": lora_config,
        "mixed_precision_config": mixed_precision_config,
    }
    if dist.is_initialized() and not parallel_state.model_parallel_is_initialized():
        parallel_state.initialize_model_parallel(tensor_model_parallel_size=tensor_parallel_size,
                                                 pipeline_model_parallel_size=pipeline_parallel_size,
                                                 expert_model_parallel_size=expert_parallel_size)
    if dist.is_initialized() and parallel_state.is_global_rank_zero():
        logger.info("NxD config: \n%s", pformat(config))
    return config


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def initialize_parallel_model(nxd_config: Dict[str, Any], model_fn, *model_args, **model_kwargs) -> NxDModel:
    if not parallel_state.model_parallel_is_initialized():
        parallel_state.initialize_model_parallel(nxd_config["tensor_parallel_size"], nxd_config["pipeline_parallel_size"],
                                                 nxd_config["expert_parallel_size"])
    init_cfg = nxd_config["model_init_config"]
    meta = init_cfg.get("meta_device_init", False)
    param_init_fn = init_cfg.get("param_init_fn", None)
    if meta:
        with init_on_device(torch.device("meta"), force_custom_init_on_device=True):
            model = model_fn(*model_args, **model_kwargs)
    else:
        model = model_fn(*model_args, **model_kwargs)
    base_model = model
    pp_enabled = nxd_config["pipeline_parallel_size"] > 1
    if pp_enabled:
        from ..pipeline.model import NxDPPModel

        pcfg = dict(nxd_config["pipeline_config"] or {})
        pcfg.update({"param_init_fn": param_init_fn, "use_model_wrapper": True})
        model = NxDPPModel(model, **pcfg)
    model = get_model_sequential(model, _device(), init_cfg.get("sequential_move_factor", 11), param_init_fn)
    lora_config = nxd_config.get("lora_config", None)
    if lora_config is not None and getattr(lora_config, "enable_lora", False):
        from ..modules.lora import LoraModel

        model = LoraModel(model, lora_config)
    if nxd_config["pad_model"]:
        assert is_hf_pretrained_model(base_model) or hasattr(base_model, "config"), "pad_model needs a model config"
        model = pad_model(model, parallel_state.get_tensor_model_parallel_size(), base_model.config.num_attention_heads)
    from ..parallel.grad_buffer import tag_shared_params

    tag_shared_params(model)
    nxd_model = NxDModel(model, nxd_config)
    ac = nxd_config["activation_checkpoint_config"]
    if ac is not None:
        if ac == "full":
            if pp_enabled:
                classes = (model.transformer_layer_cls,)
            elif hasattr(base_model, "_no_split_modules") and base_model._no_split_modules:
                names = set(base_model._no_split_modules)
                classes = tuple({type(m) for m in base_model.modules() if type(m).__name__ in names})
            else:
                from ..models.llama.modeling_llama import LlamaDecoderLayer

                classes = (LlamaDecoderLayer,)
        else:
            classes = tuple(ac) if isinstance(ac, (list, tuple)) else (ac,)
        assert classes and all(issubclass(c, torch.nn.Module) for c in classes)
        apply_activation_checkpointing(nxd_model, check_fn=lambda m: isinstance(m, classes))
    return nxd_model


def initialize_parallel_optimizer(nxd_config: Dict[str, Any], optimizer_class, parameters, **defaults) -> NxDOptimizer:
    optimizer = initialize_optimizer_from_class(nxd_config, optimizer_class, parameters, **defaults)
    return NxDOptimizer(optimizer, nxd_config)


def initialize_optimizer_from_class(nxd_config, optimizer_class, parameters, model=None, **defaults):
    ocfg = nxd_config["optimizer_config"]
    mp = nxd_config["mixed_precision_config"]
    if ocfg["zero_one_enabled"] or mp.get("use_master_weights", False):
        from ..optimizer.zero_redundancy_optimizer import NeuronEPZero1Optimizer, NeuronZero1Optimizer

        cls = NeuronEPZero1Optimizer if parallel_state.get_expert_model_parallel_size() > 1 else NeuronZero1Optimizer
        shared = None
        if model is not None:
            from ..parallel.grad_buffer import tag_shared_params

            shared = tag_shared_params(model)
        return cls(parameters, optimizer_class, grad_clipping=ocfg["grad_clipping"], shared_param_ids=shared,
                   max_norm=ocfg.get("max_grad_norm", 1.0),
                   save_master_weights=mp.get("use_master_weights_in_ckpt", False), **defaults)
    if mp.get("use_fp32_grad_acc", False) or mp.get("use_master_weights_in_ckpt", False):
        raise RuntimeError("Non Zero-1 optimizer does not support `use_fp32_grad_acc` of `use_master_weights_in_ckpt`.")
    return optimizer_class(parameters, **defaults)


def filter_to_local_parameter_group(optimizer, model):
    """Keep only parameters owned by this pipeline stage (post-partition hook)."""
    local = {id(p) for p in model.parameters()}
    for g in optimizer.param_groups:
        g["params"] = [p for p in g["params"] if id(p) in local]
