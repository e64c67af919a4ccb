"""LoraModel: adapter injection, trainability, merge/unmerge, adapter save/load
(reference: src/neuronx_distributed/modules/lora/model.py:75-694).

Checkpoint semantics follow the reference: `state_dict()` returns the adapter (plus biases /
`modules_to_save` per `bias`), the merged base model (`save_lora_base` + `merge_lora`) or everything
(`save_lora_base`), optionally with the LoRA config embedded ("lora_config" entry); in a
distributed run `nxd.save_checkpoint(model=...)` stores exactly that per rank.
"""

from __future__ import annotations

import json
import os
import re
from dataclasses import asdict
from typing import Any, Dict, Mapping, Optional, Tuple

import torch
from torch import nn

from ...parallel_layers import parallel_state as ps
from ...parallel_layers.layers import ColumnParallelLinear, ParallelEmbedding, RowParallelLinear
from ...utils.logger import get_logger
from ..qkv_linear import GQAQKVColumnParallelLinear
from .config import LoraConfig
from .layer import LoraConv2d, LoraEmbedding, LoraLayer, LoraLinear
from .tp_layer import LoraGQAQKVParallelLinear, LoraParallelEmbedding, LoraParallelLinear

logger = get_logger()

CONFIG_NAME = "adapter_config.json"
WEIGHTS_NAME = "adapter_model.pt"

# default adapter targets per architecture (fused projections of this framework's models)
TRANSFORMERS_MODELS_TO_LORA_TARGET_MODULES_MAPPING = {
    "llama": ["qkv_proj", "o_proj"],
    "mixtral": ["qkv_proj", "o_proj"],
    "mistral": ["qkv_proj", "o_proj"],
    "gpt_neox": ["query_key_value"],
    "bert": ["query", "value"],
}


class LoraModel(nn.Module):
    def __init__(self, module: nn.Module, config: LoraConfig) -> None:
        assert config is not None
        super().__init__()
        self.module = module
        self.lora_config = config
        self.modules_to_save = config.modules_to_save
        self.is_lora_merged = False
        self.is_config_saved = False
        self.is_lora_enabled = False
        self.is_checkpoint_loaded = False
        self.is_base_model_loaded = False
        self.lora_ckpt = None
        if config.load_lora_from_ckpt:
            self.load_checkpoint(config)
        else:
            self.inject_adapter()

    # ------------------------------------------------------------------ injection
    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def generate(self, *args, **kwargs):
        return self.module.generate(*args, **kwargs)

    def _set_target_modules(self) -> None:
        if self.lora_config.target_modules is not None:
            return
        mtype = getattr(getattr(self.module, "config", None), "model_type", None)
        if mtype not in TRANSFORMERS_MODELS_TO_LORA_TARGET_MODULES_MAPPING:
            raise ValueError("Please specify `target_modules` in the LoRA config")
        self.lora_config.target_modules = set(TRANSFORMERS_MODELS_TO_LORA_TARGET_MODULES_MAPPING[mtype])

    def _check_target_module_exists(self, key: str) -> bool:
        t = self.lora_config.target_modules
        if isinstance(t, str):
            return re.fullmatch(t, key) is not None
        return key in t or any(key.endswith("." + x) for x in t)

    def _get_submodules(self, key: str):
        parent = self.module.get_submodule(".".join(key.split(".")[:-1])) if "." in key else self.module
        return parent, self.module.get_submodule(key), key.split(".")[-1]

    def _create_new_module(self, target: nn.Module) -> LoraLayer:
        c = self.lora_config
        if isinstance(target, GQAQKVColumnParallelLinear):
            return LoraGQAQKVParallelLinear(target, c)
        if isinstance(target, (ColumnParallelLinear, RowParallelLinear)):
            return LoraParallelLinear(target, c)
        if isinstance(target, ParallelEmbedding):
            return LoraParallelEmbedding(target, c)
        if isinstance(target, nn.Embedding):
            return LoraEmbedding(target, c)
        if isinstance(target, nn.Conv2d):
            return LoraConv2d(target, c)
        if isinstance(target, nn.Linear):
            return LoraLinear(target, c)
        raise ValueError(f"Target module {type(target).__name__} is not supported by LoRA")

    def inject_adapter(self) -> None:
        self._set_target_modules()
        keys = [k for k, _ in self.module.named_modules()]
        found = False
        for key in keys:
            if not key or not self._check_target_module_exists(key):
                continue
            parent, target, name = self._get_submodules(key)
            if isinstance(target, LoraLayer):
                continue
            setattr(parent, name, self._create_new_module(target))
            found = True
        if not found:
            raise ValueError(f"Target modules {self.lora_config.target_modules} not found in the base model")
        self._mark_only_adapters_as_trainable()
        self.is_lora_enabled = True

    def _mark_only_adapters_as_trainable(self) -> None:
        bias = self.lora_config.bias
        for n, p in self.module.named_parameters():
            trainable = "lora_" in n
            if bias == "all" and n.endswith("bias"):
                trainable = True
            if self.modules_to_save and any(m in n for m in self.modules_to_save):
                trainable = True
            p.requires_grad_(trainable)
        if bias == "lora_only":
            for m in self.module.modules():
                if isinstance(m, LoraLayer) and getattr(m.base_layer, "bias", None) is not None:
                    m.base_layer.bias.requires_grad_(True)

    # ------------------------------------------------------------------ merge
    def _lora_layers(self):
        return [m for m in self.module.modules() if isinstance(m, LoraLayer)]

    def merge_lora(self) -> None:
        if not self.is_lora_merged:
            for m in self._lora_layers():
                m.merge()
            self.is_lora_merged = True

    def unmerge_lora(self) -> None:
        if self.is_lora_merged:
            for m in self._lora_layers():
                m.unmerge()
            self.is_lora_merged = False

    def get_base_model(self) -> nn.Module:
        return self.module

    @staticmethod
    def _restore_module_name(key: str) -> str:
        return key.replace(".base_layer", "")

    # ------------------------------------------------------------------ state dicts
    def module_state_dict(self) -> Dict[str, Any]:
        return self.module.state_dict()

    def _get_lora_adapter_state_dict(self, save_dir: Optional[str] = None) -> Dict[str, Any]:
        c = self.lora_config
        sd = self.module_state_dict()
        if c.save_lora_base and not c.merge_lora:
            out = dict(sd)
        elif c.save_lora_base and c.merge_lora:
            self.merge_lora()
            out = {self._restore_module_name(k): v.clone() for k, v in self.module_state_dict().items() if "lora_" not in k}
            self.unmerge_lora()
        else:
            if c.bias == "none":
                out = {k: v for k, v in sd.items() if "lora_" in k}
            elif c.bias == "all":
                out = {k: v for k, v in sd.items() if "lora_" in k or k.endswith("bias")}
            else:
                out = {}
                for k, v in sd.items():
                    if "lora_" in k:
                        out[k] = v
                        b = k.split("lora_")[0] + "base_layer.bias"
                        if b in sd:
                            out[b] = sd[b]
            if self.modules_to_save:
                for k, v in sd.items():
                    if any(m in k for m in self.modules_to_save):
                        out[k] = v
        if c.save_lora_config_adapter:
            out["lora_config"] = c.selected_fields_to_save()
        elif not self.is_config_saved and ps.is_global_rank_zero():
            self.save_config(save_dir)
        return out

    def state_dict(self, *args, **kwargs):
        return self._get_lora_adapter_state_dict()

    def update_state_dict_keys(self, state_dict: Dict[str, Any]) -> Dict[str, Any]:
        for mkey in self.module_state_dict().keys():
            if ".base_layer" in mkey:
                key = mkey.replace(".base_layer", "")
                if key in state_dict and mkey not in state_dict:
                    state_dict[mkey] = state_dict.pop(key)
        return state_dict

    def load_state_dict(self, state_dict: Mapping[str, Any] = None, strict: bool = True, assign: bool = False):
        """Step 1 base weights (un-adapted names are mapped onto `.base_layer`), step 2 adapters."""
        state_dict = dict(state_dict) if state_dict is not None else None
        res = None
        if state_dict is not None:
            cfg = state_dict.pop("lora_config", None)
            if self.is_lora_enabled:
                self.update_state_dict_keys(state_dict)
            res = self.module.load_state_dict(state_dict, strict=False)
            self.is_base_model_loaded = True
        if self.lora_config.load_lora_from_ckpt and self.lora_ckpt is not None:
            res = self.load_lora_adapter()
        return res

    # ------------------------------------------------------------------ single-device adapter IO
    def save_config(self, save_dir: Optional[str] = None) -> None:
        save_dir = save_dir or self.lora_config.lora_save_dir
        os.makedirs(save_dir, exist_ok=True)
        with open(os.path.join(save_dir, CONFIG_NAME), "w") as f:
            json.dump(self.lora_config.selected_fields_to_save(), f, indent=2, sort_keys=True)
        self.is_config_saved = True

    def save_lora(self, save_dir: Optional[str] = None, adapter_tag: Optional[str] = None) -> None:
        if ps.model_parallel_is_initialized() and ps.get_tensor_model_parallel_size() > 1:
            raise RuntimeError("Please use nxd.save_checkpoint() to save LoRA adapter with NxDModel.")
        save_dir = save_dir or self.lora_config.lora_save_dir
        out = save_dir if adapter_tag is None else os.path.join(save_dir, adapter_tag)
        os.makedirs(out, exist_ok=True)
        torch.save({k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in self.state_dict().items()},
                   os.path.join(out, WEIGHTS_NAME))

    def load_checkpoint(self, lora_config: LoraConfig) -> None:
        save_dir, tag = lora_config.lora_save_dir, lora_config.lora_load_tag
        path = os.path.join(save_dir if tag is None else os.path.join(save_dir, tag), WEIGHTS_NAME)
        if not os.path.isfile(path):
            raise FileNotFoundError(f"{path} is not found.")
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        if "lora_config" in ckpt:
            d = asdict(lora_config)
            d.update(ckpt.pop("lora_config"))
            self.lora_config = LoraConfig(**d)
        else:
            cfg_file = os.path.join(save_dir, CONFIG_NAME)
            if not os.path.isfile(cfg_file):
                raise FileNotFoundError(f"LoRA configuration file {cfg_file} is not found.")
            with open(cfg_file) as f:
                loaded = json.load(f)
            d = asdict(lora_config)
            d.update({k: loaded[k] for k in lora_config.get_selected_fields() if k in loaded})
            self.lora_config = LoraConfig(**d)
        self.lora_ckpt = ckpt
        self.is_checkpoint_loaded = True

    def load_lora_adapter(self):
        c = self.lora_config
        if not (c.save_lora_base and c.merge_lora) and not self.is_lora_enabled:
            self.inject_adapter()
        return self.module.load_state_dict(self.lora_ckpt, strict=False)

    def load_lora(self, save_dir: Optional[str] = None, adapter_tag: Optional[str] = None,
                  ckpt_path: Optional[str] = None, adapter_only: bool = True):
        if not self.is_checkpoint_loaded:
            cfg = LoraConfig(**{**asdict(self.lora_config), "lora_save_dir": save_dir or self.lora_config.lora_save_dir,
                                "lora_load_tag": adapter_tag})
            self.load_checkpoint(cfg)
        return self.load_lora_adapter()

    # ------------------------------------------------------------------ misc API
    def named_parameters(self, *args, **kwargs):
        return self.module.named_parameters(*args, **kwargs)

    @property
    def dtype(self):
        return next(self.module.parameters()).dtype

    @property
    def config(self):
        return getattr(self.module, "config", None)

    def __getattr__(self, name: str) -> Any:
        try:
            return super().__getattr__(name)
        except AttributeError:
            if name == "module":
                raise
            return getattr(self.module, name)

    def get_nb_trainable_parameters(self) -> Tuple[int, int]:
        trainable = sum(p.numel() for p in self.module.parameters() if p.requires_grad)
        total = sum(p.numel() for p in self.module.parameters())
        return trainable, total

    def print_trainable_parameters(self) -> None:
        t, a = self.get_nb_trainable_parameters()
        logger.info(f"trainable params: {t:,d} || all params: {a:,d} || trainable%: {100 * t / max(a, 1):.4f}")

    def print_model_info(self) -> None:
        if self.lora_config.lora_verbose:
            logger.info(str(self.module))
        self.print_trainable_parameters()
