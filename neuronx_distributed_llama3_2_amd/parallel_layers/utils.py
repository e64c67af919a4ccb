"""Tensor-parallel helpers: parameter attributes, divide/split, casting
(reference: src/neuronx_distributed/parallel_layers/utils.py:25-266)."""

from __future__ import annotations

from typing import Any, List, Sequence, Tuple

import torch

_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS = {
    "tensor_model_parallel": False,
    "partition_dim": -1,
    "partition_stride": 1,
}


class EmbeddingUtility:
    @staticmethod
    def range_from_per_partition_vocab_size(per_partition_vocab_size: int, rank: int, world_size: int) -> Tuple[int, int]:
        first = rank * per_partition_vocab_size
        return first, first + per_partition_vocab_size

    @staticmethod
    def range_from_global_vocab_size(global_vocab_size: int, rank: int, world_size: int) -> Tuple[int, int]:
        per = divide(global_vocab_size, world_size)
        return EmbeddingUtility.range_from_per_partition_vocab_size(per, rank, world_size)


def param_is_not_tensor_parallel_duplicate(param: torch.Tensor) -> bool:
    from .parallel_state import get_tensor_model_parallel_rank

    return (hasattr(param, "tensor_model_parallel") and param.tensor_model_parallel) or (
        get_tensor_model_parallel_rank() == 0)


def set_tensor_model_parallel_attributes(tensor: torch.Tensor, is_parallel: bool, dim: int, stride: int = 1,
                                         num_partitions: int = -1) -> None:
    for attr in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(tensor, attr) and attr != "tensor_model_parallel":
            pass
    setattr(tensor, "tensor_model_parallel", is_parallel)
    setattr(tensor, "partition_dim", dim)
    setattr(tensor, "partition_stride", stride)
    if num_partitions > 0:
        setattr(tensor, "num_partitions", num_partitions)


def set_defaults_if_not_set_tensor_model_parallel_attributes(tensor: torch.Tensor) -> None:
    for attr, value in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS.items():
        if not hasattr(tensor, attr):
            setattr(tensor, attr, value)


def copy_tensor_model_parallel_attributes(destination_tensor: torch.Tensor, source_tensor: torch.Tensor) -> None:
    for attr in list(_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS) + ["num_partitions", "sequence_parallel_enabled",
                                                             "expert_model_parallel", "shared"]:
        if hasattr(source_tensor, attr):
            setattr(destination_tensor, attr, getattr(source_tensor, attr))


def ensure_divisibility(numerator: int, denominator: int) -> None:
    assert numerator % denominator == 0, f"{numerator} is not divisible by {denominator}"


def divide(numerator: int, denominator: int) -> int:
    ensure_divisibility(numerator, denominator)
    return numerator // denominator


def split_tensor_along_dim(tensor: torch.Tensor, dim: int, num_partitions: int,
                           contiguous_split_chunks: bool = False) -> Sequence[torch.Tensor]:
    size = divide(tensor.size(dim), num_partitions)
    chunks = torch.split(tensor, size, dim=dim)
    if contiguous_split_chunks:
        return tuple(c.contiguous() for c in chunks)
    return chunks


def get_padding_length(numerator: int, denominator: int) -> int:
    return (denominator - numerator % denominator) % denominator


def split_tensor_along_last_dim(tensor: torch.Tensor, num_partitions: int, contiguous_split_chunks: bool = False):
    return split_tensor_along_dim(tensor, tensor.dim() - 1, num_partitions, contiguous_split_chunks)


def split_tensor_along_second_dim(tensor: torch.Tensor, num_partitions: int, contiguous_split_chunks: bool = False):
    return split_tensor_along_dim(tensor, 1, num_partitions, contiguous_split_chunks)


def cast_tensor(tensor: torch.Tensor, from_dtype=torch.float32, to_dtype=torch.bfloat16) -> Any:
    return tensor.to(dtype=to_dtype) if tensor.dtype == from_dtype else tensor


def cast_all(state: Any, from_dtype=torch.float32, to_dtype=torch.bfloat16) -> Any:
    if isinstance(state, torch.Tensor):
        return cast_tensor(state, from_dtype, to_dtype)
    if isinstance(state, dict):
        return {k: cast_all(v, from_dtype, to_dtype) for k, v in state.items()}
    if isinstance(state, (list, tuple)):
        return type(state)(cast_all(v, from_dtype, to_dtype) for v in state)
    return state


def cast_if_autocast_enabled(*args: Any) -> Any:
    if not torch.is_autocast_enabled():
        return args
    dt = torch.get_autocast_gpu_dtype() if hasattr(torch, "get_autocast_gpu_dtype") else torch.bfloat16
    return cast_all(args, torch.float32, dt)


def move_all_tensor_to_cpu(data: Any, convert: bool = True) -> Any:
    if isinstance(data, torch.Tensor):
        return data.detach().cpu() if convert else data
    if isinstance(data, dict):
        return {k: move_all_tensor_to_cpu(v, convert) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return type(data)(move_all_tensor_to_cpu(v, convert) for v in data)
    return data


def get_local_world_size() -> int:
    import os

    for k in ("LOCAL_WORLD_SIZE", "GPUS_PER_NODE"):
        if k in os.environ:
            return int(os.environ[k])
    if torch.cuda.is_available():
        return max(1, torch.cuda.device_count())
    return 1


def move_model_to_device(model: torch.nn.Module, device) -> None:
    from ..utils.model_utils import move_model_to_device as _mv

    _mv(model, device)


def verify_casted_dtype(value: Any) -> None:
    if isinstance(value, torch.Tensor):
        assert value.dtype != torch.float32 or not torch.is_autocast_enabled(), "unexpected fp32 tensor under autocast"


def indices_split_along_dim(full_size: int, num_partitions: int, rank: int, stride: int = 1) -> List[Tuple[int, int]]:
    """(start, end) index ranges of `rank`'s strided shard along a dim of size `full_size`."""
    per = divide(full_size, num_partitions * stride)
    return [((s * num_partitions + rank) * per, (s * num_partitions + rank + 1) * per) for s in range(stride)]
