"""Legacy (v1) sharded save/load of `parallel_layers` (reference: src/neuronx_distributed/parallel_layers/checkpointing.py:35-269).

On-disk layout is unchanged:
  non-xser: <dir>/tp_rank_XX_pp_rank_XX[_dp_rank_XX]/checkpoint.pt
  xser:     <dir>/tp_rank_XX_pp_rank_XX[_dp_rank_XX]            (structure with tensor references)
            <dir>/tp_rank_XX_pp_rank_XX[_dp_rank_XX].tensors/tensor_<i>.pt
Barriers are plain `torch.distributed.barrier()` (no XLA rendezvous); `NXD_SKIP_RENDEZVOUS=1` skips them.
`load(..., sharded=False)` shards a full (unsharded) checkpoint on the fly using each parameter's
TP attributes and the modules' `preshard_hook`s.
"""

from __future__ import annotations

import gc
import os
from typing import Any, Callable, Dict, Optional

import torch
import torch.distributed as dist

from ..utils.logger import get_logger
from ..utils.serialization import xser_load, xser_save
from .layers import create_local_weight
from .parallel_state import (
    get_data_parallel_rank,
    get_pipeline_model_parallel_rank,
    get_tensor_model_parallel_rank,
    get_tensor_model_parallel_size,
)
from .utils import cast_all, move_all_tensor_to_cpu

logger = get_logger()

NXD_SKIP_RENDEZVOUS = "NXD_SKIP_RENDEZVOUS"


def _barrier():
    if os.environ.get(NXD_SKIP_RENDEZVOUS, "0") == "1":
        return
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def ensure_directory_exists(filename: str) -> None:
    os.makedirs(os.path.dirname(filename), exist_ok=True)


def _invoke_preshard_hook(module: torch.nn.Module, model_state_dict: Dict[str, Any], prefix: str = "") -> None:
    if module is None:
        return
    if hasattr(module, "preshard_hook"):
        module.preshard_hook(model_state_dict, prefix + "weight")
        return
    for name, child in module.named_children():
        _invoke_preshard_hook(child, model_state_dict, prefix + name + ".")


def get_sharded_model_dict(model: torch.nn.Module, model_state_dict: Dict[str, Any]) -> Dict[str, Any]:
    """Shard a full state dict to this TP rank using each parameter's partition attributes."""
    tp_size = get_tensor_model_parallel_size()
    model = getattr(model, "original_torch_module", model)
    _invoke_preshard_hook(model, model_state_dict)
    for name, param in model.state_dict(keep_vars=True).items():
        if getattr(param, "tensor_model_parallel", False) and name in model_state_dict:
            if param.partition_dim not in (0, 1):
                raise Exception(f"Partition value of 0,1 are supported, found {param.partition_dim}.")
            full = model_state_dict[name]
            per = full.shape[param.partition_dim] // tp_size
            model_state_dict[name] = create_local_weight(full, param.partition_dim, per,
                                                         getattr(param, "partition_stride", 1))
    return model_state_dict


def _path(output_dir: str, master_dp_only: bool) -> str:
    p = os.path.join(output_dir, "tp_rank_{:02d}_pp_rank_{:02d}".format(get_tensor_model_parallel_rank(),
                                                                        get_pipeline_model_parallel_rank()))
    if not master_dp_only:
        p += "_dp_rank_{:02d}".format(get_data_parallel_rank())
    return p


def save(checkpoint: dict, output_dir: str, save_serially: bool = True, save_xser: bool = False,
         down_cast_bf16: bool = False, master_dp_only: bool = True) -> None:
    logger.info("saving checkpoint to %s", output_dir)
    path = _path(output_dir, master_dp_only)
    if not save_xser:
        path = os.path.join(path, "checkpoint.pt")
    if down_cast_bf16:
        checkpoint = cast_all(checkpoint, from_dtype=torch.float32, to_dtype=torch.bfloat16)
    writer = get_data_parallel_rank() == 0 or not master_dp_only
    if writer:
        ensure_directory_exists(path)
        cpu = move_all_tensor_to_cpu(checkpoint)
        if save_xser:
            xser_save(cpu, path)
        else:
            torch.save(cpu, path)
        del cpu
        gc.collect()
    _barrier()


def load(chkpt_path: str, model: Optional[torch.nn.Module] = None, model_key: Optional[str] = "model",
         load_xser: bool = False, sharded: bool = True, strict: bool = True, master_dp_only: bool = True,
         weights_only: bool = True) -> Any:
    """Load this rank's shard (or shard a full checkpoint when `sharded=False`) into `model`."""
    if sharded:
        path = _path(chkpt_path, master_dp_only)
        if load_xser:
            ckpt = xser_load(path)
        else:
            ckpt = torch.load(os.path.join(path, "checkpoint.pt"), map_location="cpu", weights_only=weights_only)
    else:
        ckpt = torch.load(chkpt_path, map_location="cpu", weights_only=weights_only)
    if model is not None:
        sd = ckpt[model_key] if model_key is not None else ckpt
        if not sharded:
            sd = get_sharded_model_dict(model, sd)
        target = getattr(model, "original_torch_module", model)
        target.load_state_dict(sd, strict=strict)
    _barrier()
    return ckpt
