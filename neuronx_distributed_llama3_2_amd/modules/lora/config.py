"""LoRA configuration (reference: src/neuronx_distributed/modules/lora/config.py:6-145; same fields)."""

from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import List, Literal, Optional, Union


@dataclass
class LoraConfig:
    enable_lora: bool = False
    lora_rank: int = 16
    target_modules: Optional[Union[List[str], str]] = None
    lora_alpha: int = 8
    lora_dropout: float = 0.0
    bias: Literal["none", "all", "lora_only"] = "none"
    use_rslora: bool = False
    init_lora_weights: Literal["default", "gaussian"] = "default"
    modules_to_save: Optional[List[str]] = None
    lora_verbose: bool = False
    load_lora_from_ckpt: bool = False
    lora_load_tag: Optional[str] = None
    lora_save_dir: Optional[str] = "lora_adapter"
    merge_lora: bool = False
    save_lora_base: bool = False
    save_lora_config_adapter: bool = True
    merge_sharded_lora: bool = False

    @staticmethod
    def get_selected_fields():
        return ["bias", "init_lora_weights", "lora_alpha", "lora_dropout", "lora_rank", "use_rslora", "target_modules",
                "modules_to_save", "save_lora_base", "merge_lora", "save_lora_config_adapter"]

    def selected_fields_to_save(self) -> dict:
        d = asdict(self)
        out = {k: v for k, v in d.items() if k in self.get_selected_fields()}
        if isinstance(out.get("target_modules"), set):
            out["target_modules"] = sorted(out["target_modules"])
        return out

    def __post_init__(self):
        if isinstance(self.target_modules, list):
            self.target_modules = set(self.target_modules)
        if self.bias not in ("none", "all", "lora_only"):
            raise ValueError(f"bias must be 'none', 'all' or 'lora_only', got {self.bias}")
