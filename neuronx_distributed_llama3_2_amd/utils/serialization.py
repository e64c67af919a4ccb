"""Serialization helpers.

* xser (tensor-per-file) checkpoints, same layout as torch_xla's xser used by the reference
  (src/neuronx_distributed/parallel_layers/checkpointing.py:111-113, trainer/checkpoint.py:308-470):
  `<path>` holds the nested structure with every tensor replaced by a reference, and
  `<path>.tensors/tensor_<i>.pt` holds the tensors.  References are stored as plain
  `{"__nxd_tensor_ref__": i}` dicts so every file loads with `torch.load(weights_only=True)`.
* `SerializationManager`: strip tensors out of arbitrary nested Python objects (for pipeline
  stage IO) and rebuild them (reference: src/neuronx_distributed/utils/serialization.py:14-253).
"""

from __future__ import annotations

import dataclasses
import io
import os
import pickle
import zlib
from typing import Any, Dict, List, Tuple

import torch

_REF_KEY = "__nxd_tensor_ref__"


def _strip(obj, tensors: List[torch.Tensor]):
    if isinstance(obj, torch.Tensor):
        tensors.append(obj)
        return {_REF_KEY: len(tensors) - 1}
    if isinstance(obj, dict):
        return {k: _strip(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_strip(v, tensors) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_strip(v, tensors) for v in obj)
    return obj


def _rebuild(obj, loader):
    if isinstance(obj, dict):
        if len(obj) == 1 and _REF_KEY in obj:
            return loader(obj[_REF_KEY])
        return {k: _rebuild(v, loader) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_rebuild(v, loader) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_rebuild(v, loader) for v in obj)
    # torch_xla TensorReference-like objects (attribute `tid`)
    if hasattr(obj, "tid") and type(obj).__name__ == "TensorReference":
        return loader(obj.tid)
    return obj


def xser_save(data: Any, path: str, tensor_ids: List[int] = None) -> List[torch.Tensor]:
    tensors: List[torch.Tensor] = []
    ref = _strip(data, tensors)
    tdir = path + ".tensors"
    os.makedirs(tdir, exist_ok=True)
    for i, t in enumerate(tensors):
        if tensor_ids is None or i in tensor_ids:
            torch.save(t.detach().cpu().contiguous(), os.path.join(tdir, f"tensor_{i}.pt"))
    torch.save(ref, path)
    return tensors


def xser_load(path: str, map_location="cpu") -> Any:
    ref = torch.load(path, map_location=map_location, weights_only=True)
    tdir = path + ".tensors"

    def loader(i):
        return torch.load(os.path.join(tdir, f"tensor_{i}.pt"), map_location=map_location, weights_only=True)

    return _rebuild(ref, loader)


def compress_to_string(obj: Any) -> bytes:
    return zlib.compress(pickle.dumps(obj))


def uncompress_from_string(s: bytes) -> Any:
    return pickle.loads(zlib.decompress(s))  # only ever used on bytes this process produced


@dataclasses.dataclass
class TensorMeta:
    tensor_index: int
    dtype: torch.dtype
    shape: Tuple[int, ...]
    requires_grad: bool
    device: Any


class SerializationManager:
    """Separate tensors from a nested Python object: serialize(obj) -> (stub, tensors, metas);
    deserialize(stub, tensors) rebuilds the object."""

    def serialize(self, obj: Any):
        tensors: List[torch.Tensor] = []
        stub = _strip(obj, tensors)
        metas = [TensorMeta(i, t.dtype, tuple(t.shape), t.requires_grad, t.device) for i, t in enumerate(tensors)]
        return stub, tensors, metas

    def deserialize(self, stub: Any, tensors: List[torch.Tensor]) -> Any:
        return _rebuild(stub, lambda i: tensors[i])


def find_loss_from_output_and_spec(output_val, spec):
    """Locate the loss tensor in a model output by a boolean spec of the same structure
    (reference utils/serialization.py:36-70)."""
    if spec is True:
        if not isinstance(output_val, torch.Tensor):
            raise RuntimeError(f"loss spec points at a non-tensor: {type(output_val)}")
        return output_val
    if spec is False or spec is None:
        return None
    if isinstance(spec, (list, tuple)):
        for o, s in zip(output_val, spec):
            r = find_loss_from_output_and_spec(o, s)
            if r is not None:
                return r
        return None
    if isinstance(spec, dict):
        for k, s in spec.items():
            r = find_loss_from_output_and_spec(output_val[k], s)
            if r is not None:
                return r
        return None
    raise RuntimeError(f"unsupported loss spec {spec}")
