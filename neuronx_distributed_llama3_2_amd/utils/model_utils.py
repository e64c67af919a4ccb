"""Model construction utilities: meta-device (deferred) init, materialisation with a param_init_fn,
moving to the GPU while preserving TP/EP/SP parameter attributes and weight ties
(reference: src/neuronx_distributed/utils/model_utils.py:44-348).

MI355X note: the reference staggers host->device moves (`sequential_move_factor`) to avoid host
OOM on 32 NeuronCores per host; with one process per GPU and 288 GB of HBM each rank materialises
its own shard directly on its GPU, so the factor only bounds how many local ranks materialise
concurrently (barrier between waves).
"""

from __future__ import annotations

import contextlib
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

_PARALLEL_ATTRS = ("tensor_model_parallel", "partition_dim", "partition_stride", "num_partitions",
                   "sequence_parallel_enabled", "expert_model_parallel", "shared", "fused_qkv", "qkv_split")


def analyze_shared_parameters(module: nn.Module, prefix: str = "") -> List[List[str]]:
    """Groups of parameter names that refer to the same tensor (tied weights)."""
    by_id: Dict[int, List[str]] = defaultdict(list)
    for mname, m in module.named_modules(remove_duplicate=False):
        for pname, p in m.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            if full not in by_id[id(p)]:
                by_id[id(p)].append(prefix + full)
    return [names for names in by_id.values() if len(names) > 1]


def _get_by_name(module: nn.Module, name: str):
    *path, leaf = name.split(".")
    m = module
    for p in path:
        m = getattr(m, p)
    return m, leaf


def retie_shared_weights(module: nn.Module, shared_groups: List[List[str]]) -> None:
    for names in shared_groups:
        src_mod, src_leaf = _get_by_name(module, names[0])
        src = getattr(src_mod, src_leaf)
        for n in names[1:]:
            m, leaf = _get_by_name(module, n)
            setattr(m, leaf, src)


@contextlib.contextmanager
def preserve_shared_weights(module: nn.Module):
    groups = analyze_shared_parameters(module)
    try:
        yield
    finally:
        retie_shared_weights(module, groups)


def _collect_attrs(module: nn.Module):
    return {n: {a: getattr(p, a) for a in _PARALLEL_ATTRS if hasattr(p, a)} for n, p in module.named_parameters()}


def _restore_attrs(module: nn.Module, saved):
    for n, p in module.named_parameters():
        for a, v in saved.get(n, {}).items():
            setattr(p, a, v)


@contextlib.contextmanager
def preserve_parallel_attributes(module: nn.Module):
    saved = _collect_attrs(module)
    try:
        yield
    finally:
        _restore_attrs(module, saved)


def reinit_model(model: nn.Module, device, param_init_fn: Callable) -> None:
    """Materialise meta parameters on `device` and call `param_init_fn(module)` on each module."""
    with preserve_parallel_attributes(model), preserve_shared_weights(model):
        model.to_empty(device=device)
        for m in model.modules():
            param_init_fn(m)


def move_model_to_device(model: nn.Module, device) -> None:
    with preserve_parallel_attributes(model), preserve_shared_weights(model):
        model.to(device)


def maybe_materalize_model(model: nn.Module, device, param_init_fn: Optional[Callable] = None) -> None:
    if any(p.device.type == "meta" for p in model.parameters()):
        if param_init_fn is None:
            raise ValueError("model has meta parameters: a param_init_fn is required to materialise it")
        reinit_model(model, device, param_init_fn)


@contextlib.contextmanager
def init_on_device(device: torch.device, include_buffers: bool = False, force_custom_init_on_device: bool = False):
    """Create parameters (and optionally buffers) directly on `device` (e.g. meta) while the model
    is constructed; attributes set on the parameters by the constructors are kept."""
    old_register = nn.Module.register_parameter
    old_register_buffer = nn.Module.register_buffer

    def register_empty_parameter(module, name, param):
        old_register(module, name, param)
        if param is not None and param.device != device:
            attrs = {a: getattr(param, a) for a in _PARALLEL_ATTRS if hasattr(param, a)}
            cls = type(module._parameters[name])
            kwargs = module._parameters[name].__dict__
            new = cls(module._parameters[name].to(device), **({"requires_grad": param.requires_grad}
                                                              if cls is nn.Parameter else {}))
            for a, v in attrs.items():
                setattr(new, a, v)
            module._parameters[name] = new
            _ = kwargs

    def register_empty_buffer(module, name, buffer, persistent=True):
        old_register_buffer(module, name, buffer, persistent=persistent)
        if buffer is not None:
            module._buffers[name] = module._buffers[name].to(device)

    try:
        nn.Module.register_parameter = register_empty_parameter
        if include_buffers:
            nn.Module.register_buffer = register_empty_buffer
        yield
    finally:
        nn.Module.register_parameter = old_register
        nn.Module.register_buffer = old_register_buffer


def get_model_sequential(model: nn.Module, device, sequential_move_factor: int = 11,
                         param_init_fn: Optional[Callable] = None) -> nn.Module:
    """Materialise / move the model to `device`, at most `sequential_move_factor` local ranks at a time."""
    local_rank = 0
    local_world = 1
    if dist.is_initialized():
        from ..parallel_layers.utils import get_local_world_size

        local_world = get_local_world_size()
        local_rank = dist.get_rank() % local_world
    waves = max(1, (local_world + sequential_move_factor - 1) // sequential_move_factor)
    for wave in range(waves):
        if local_rank // sequential_move_factor == wave:
            if any(p.device.type == "meta" for p in model.parameters()):
                maybe_materalize_model(model, device, param_init_fn)
            else:
                move_model_to_device(model, device)
        if dist.is_initialized() and waves > 1:
            dist.barrier()
    return model


def is_hf_pretrained_model(model) -> bool:
    try:
        from transformers import PreTrainedModel

        return isinstance(model, PreTrainedModel)
    except Exception:  # pragma: no cover
        return False


def is_nxdt_pretrained_model(model) -> bool:
    return False


def get_delay_tracing(nxd_config) -> bool:
    return False


def check_delay_tracing(nxd_config) -> bool:
    return False
