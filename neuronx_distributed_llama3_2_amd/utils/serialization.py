"""Serialization helpers.

* xser (tensor-per-file) checkpoints in torch_xla's xser format, as the reference writes them
  (src/neuronx_distributed/parallel_layers/checkpointing.py:111-113, trainer/checkpoint.py:308-470):
  `<path>` holds the nested structure with every tensor replaced by a
  `torch_xla.utils.serialization.TensorReference(tid)` record, `<path>.info.pt` maps tid ->
  {dtype, shape, expert_model_parallel}, and `<path>.tensors/tensor_<tid>.pt` holds the tensors.
  torch_xla is not needed: the record is written under that class path by a pickler override and
  read back with `torch.load(weights_only=True)` allow-listing only that one record type, so a
  reference checkpoint loads here and ours loads in the reference.  Files written by earlier
  versions of this package (`{"__nxd_tensor_ref__": i}` dict references) still load.
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
_XLA_MODULE = "torch_xla.utils.serialization"


class TensorReference:
    """Stand-in for torch_xla.utils.serialization.TensorReference (same pickled identity)."""

    def __init__(self, tid: int):
        self.tid = tid

    def __repr__(self) -> str:
        return f"TensorReference({self.tid})"


TensorReference.__module__ = _XLA_MODULE


class _XserPickler(pickle._Pickler):
    """Pure-Python pickler that writes TensorReference under torch_xla's class path without
    importing torch_xla (the C pickler would look the class up by that name and fail)."""

    def save_global(self, obj, name=None):
        if obj is TensorReference:
            self.write(pickle.GLOBAL + _XLA_MODULE.encode() + b"\n" + b"TensorReference\n")
            self.memoize(obj)
            return
        super().save_global(obj, name)


class _XserPickleModule:
    Pickler = _XserPickler
    Unpickler = pickle.Unpickler
    __name__ = "nxd_xser_pickle"


def _xser_torch_load(path, map_location):
    with torch.serialization.safe_globals([TensorReference]):
        return torch.load(path, map_location=map_location, weights_only=True)


def _strip_refs(obj, tensors: List[torch.Tensor]):
    if isinstance(obj, torch.Tensor):
        tensors.append(obj)
        return TensorReference(len(tensors) - 1)
    if isinstance(obj, dict):
        return type(obj)((k, _strip_refs(v, tensors)) for k, v in obj.items()) if type(obj) is not dict \
            else {k: _strip_refs(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_strip_refs(v, tensors) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_strip_refs(v, tensors) for v in obj)
    return obj


def assign_tensors_to_bins(tensors: List[torch.Tensor], bin_count: int) -> List[List[int]]:
    """Greedy largest-remaining-first balancing of tensor bytes over `bin_count` writers (the
    reference's DP-deduplicated xser save, trainer/checkpoint.py:393-428)."""
    bins: List[List[int]] = [[] for _ in range(bin_count)]
    sizes = [0] * bin_count
    order = sorted(range(len(tensors)), key=lambda i: tensors[i].numel() * tensors[i].element_size(), reverse=True)
    for i in order:
        b = sizes.index(min(sizes))
        bins[b].append(i)
        sizes[b] += tensors[i].numel() * tensors[i].element_size()
    return bins


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


def xser_tensors(data: Any) -> List[torch.Tensor]:
    """The tensors of `data` in xser tid order."""
    tensors: List[torch.Tensor] = []
    _strip_refs(data, tensors)
    return tensors


def xser_save(data: Any, path: str, tensor_ids=None, write_ref: bool = True) -> List[torch.Tensor]:
    """Write `data` in xser format.  tensor_ids: the tids this writer stores (None: all) -- DP
    replicas split one shard's tensor files between them; write_ref: this writer also stores the
    reference structure and `.info.pt`."""
    tensors: List[torch.Tensor] = []
    ref = _strip_refs(data, tensors)
    tdir = path + ".tensors"
    os.makedirs(tdir, exist_ok=True)
    ids = set(range(len(tensors))) if tensor_ids is None else set(tensor_ids)
    for i, t in enumerate(tensors):
        if i in ids:
            torch.save(t.detach().cpu().contiguous(), os.path.join(tdir, f"tensor_{i}.pt"))
    if write_ref:
        info = {i: {"dtype": t.dtype, "shape": t.shape,
                    "expert_model_parallel": bool(getattr(t, "expert_model_parallel", False))}
                for i, t in enumerate(tensors)}
        torch.save(ref, path, pickle_module=_XserPickleModule)
        torch.save(info, path + ".info.pt")
    return tensors


def xser_load_info(path: str):
    """tid -> {dtype, shape, expert_model_parallel} (None for checkpoints without `.info.pt`)."""
    p = path + ".info.pt"
    return torch.load(p, map_location="cpu", weights_only=True) if os.path.exists(p) else None


def xser_load(path: str, map_location="cpu", tensor_loader=None) -> Any:
    """Load an xser checkpoint (ours or a reference one).  tensor_loader(tid, file) overrides how a
    tensor is obtained (the checkpoint loader reads 1/N of them and broadcasts the rest)."""
    ref = _xser_torch_load(path, map_location)
    tdir = path + ".tensors"

    def loader(i):
        f = os.path.join(tdir, f"tensor_{i}.pt")
        if tensor_loader is not None:
            return tensor_loader(i, f)
        return torch.load(f, map_location=map_location, weights_only=True)

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
