"""`parallel_model_trace` / `parallel_model_save` / `parallel_model_load` and the weight-sharding
helpers of the legacy inference trace API (reference: src/neuronx_distributed/trace/trace.py:52-736).

`func()` returns the model (or `(model, input_output_aliases)`) built from the framework's
parallel layers, which shard themselves for the current TP rank.  Tracing = moving the shard to
this rank's GPU and capturing one hipGraph per example-input bucket (trace/spmd.py).  Modes:

* in-process SPMD: tp_degree == 1, or torch.distributed already initialised with one process per
  rank (torchrun) — every rank calls parallel_model_trace and gets its own shard;
* single controller: tp_degree > 1 from a plain process — one worker per GPU is spawned
  (trace/runtime.py); `func` and `checkpoint_loader_callable` must then be picklable.

Saved format (`parallel_model_save`): `tp_XX.safetensors` per rank (weights AND states) +
`nxd_trace.json` (TP degree, bucket input shapes / dtypes, the importable `module:qualname` of
`func`).  Only safetensors/JSON are read back — nothing executable comes from the artifact.
"""

from __future__ import annotations

import importlib
import json
import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state as ps
from ..parallel_layers.sharding import _attrs, shard_state_dict, shard_tensor
from .runtime import SpmdWorkerPool, worker_device
from .spmd import SPMDBucketModel

_META = "nxd_trace.json"
_DT = {str(d): d for d in (torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.int8,
                           torch.bool, torch.uint8)}


class ParallelModel(torch.nn.Module):
    pass


def _buckets(example_inputs) -> List[tuple]:
    """One example (tensor or tuple of tensors) or a list of per-bucket examples."""
    if isinstance(example_inputs, torch.Tensor):
        return [(example_inputs,)]
    if isinstance(example_inputs, list) and example_inputs and isinstance(example_inputs[0], (tuple, list)):
        return [tuple(e) for e in example_inputs]
    return [tuple(example_inputs)]


def _func_path(func) -> Optional[str]:
    mod, qn = getattr(func, "__module__", None), getattr(func, "__qualname__", None)
    if mod and qn and "<locals>" not in qn and "<lambda>" not in qn:
        return f"{mod}:{qn}"
    return None


def _resolve(path: str):
    mod, qn = path.split(":")
    obj = importlib.import_module(mod)
    for part in qn.split("."):
        obj = getattr(obj, part)
    return obj


def _build_model(func):
    out = func()
    if isinstance(out, tuple):
        return out[0], (out[1] if len(out) > 1 else None)
    return out, None


class _LocalTraced:
    """This rank's traced shard: model on its device + the per-bucket graphs."""

    def __init__(self, func, buckets, checkpoint_loader_callable=None, weights_file=None, use_graph=True):
        rank = ps.get_tensor_model_parallel_rank()
        tp = ps.get_tensor_model_parallel_size()
        self.device = worker_device(rank, tp) if torch.cuda.is_available() else torch.device("cpu")
        if self.device.type == "cuda" and dist.is_initialized() and dist.get_backend() != "nccl":
            self.device = torch.device("cuda", torch.cuda.current_device())
        model, self.aliases = _build_model(func)
        if checkpoint_loader_callable is not None:
            full = checkpoint_loader_callable()
            model.load_state_dict(shard_state_dict(model, full, tp, rank, strict=False), strict=False)
        if weights_file is not None:
            from safetensors.torch import load_file

            model.load_state_dict(load_file(weights_file), strict=False)
        self.model = model.to(self.device).eval()
        self.func = func
        self.buckets = [tuple(t.to(self.device) for t in b) for b in buckets]
        with torch.no_grad():
            self.bucket_model = SPMDBucketModel(self.model, self.buckets, use_graph=use_graph)
            self.bucket_model.build()

    @torch.no_grad()
    def __call__(self, *inputs):
        return self.bucket_model(*[t.to(self.device) for t in inputs])

    def save(self, save_dir: str) -> None:
        from safetensors.torch import save_file

        os.makedirs(save_dir, exist_ok=True)
        rank = ps.get_tensor_model_parallel_rank()
        sd = {}
        for k, v in list(self.model.state_dict().items()):
            sd[k] = v.detach().contiguous().cpu()
        # tied parameters appear once (safetensors refuses shared storage)
        seen, uniq = {}, {}
        for k, v in sd.items():
            key = (v.data_ptr(), tuple(v.shape)) if v.numel() else None
            if key is not None and key in seen:
                continue
            if key is not None:
                seen[key] = k
            uniq[k] = v
        save_file(uniq, os.path.join(save_dir, f"tp_{rank:02d}.safetensors"))
        if rank == 0:
            meta = {"tp_degree": ps.get_tensor_model_parallel_size(), "func": _func_path(self.func),
                    "buckets": [[[list(t.shape), str(t.dtype)] for t in b] for b in self.buckets]}
            with open(os.path.join(save_dir, _META), "w") as f:
                json.dump(meta, f, indent=2)


def _pool_build(rank, world, func, buckets, loader, weights_dir):
    wf = os.path.join(weights_dir, f"tp_{rank:02d}.safetensors") if weights_dir else None
    return _LocalTraced(func, buckets, loader, wf)


class TensorParallelNeuronModel(ParallelModel):
    """Handle returned by parallel_model_trace: calls go to this rank's graphs (SPMD) or to the
    worker pool (single controller)."""

    def __init__(self, local: Optional[_LocalTraced] = None, pool: Optional[SpmdWorkerPool] = None, tp_degree: int = 1):
        super().__init__()
        self.local, self.pool, self.tp_degree = local, pool, tp_degree

    def forward(self, *tensors):
        if self.local is not None:
            return self.local(*tensors)
        return self.pool(*tensors)

    def save(self, save_dir: str) -> None:
        if self.local is not None:
            self.local.save(save_dir)
            if dist.is_initialized() and dist.get_world_size() > 1:
                dist.barrier()
        else:
            self.pool.call("save", save_dir)

    def close(self) -> None:
        if self.pool is not None:
            self.pool.close()
            self.pool = None


TensorParallelModel = TensorParallelNeuronModel


def _spmd_context(tp_degree: int) -> bool:
    """True when this process is one rank of an SPMD launch (or TP=1 in-process)."""
    if dist.is_initialized():
        if not ps.model_parallel_is_initialized():
            ps.initialize_model_parallel(tensor_model_parallel_size=tp_degree)
        assert ps.get_tensor_model_parallel_size() == tp_degree, "tp_degree != initialised TP size"
        return True
    if tp_degree == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 1000))
        dist.init_process_group("gloo", rank=0, world_size=1)
        ps.initialize_model_parallel(tensor_model_parallel_size=1)
        return True
    return False


def parallel_model_trace(func: Union[Callable, torch.nn.Module], example_inputs: Any, states=None,
                         compiler_workdir: Optional[str] = None, compiler_args=None, inline_weights_to_neff: bool = True,
                         bucket_config=None, tp_degree: int = 1, max_parallel_compilations: Optional[int] = None,
                         spmd_mode: bool = False, checkpoint_loader_callable: Optional[Callable] = None,
                         force_custom_init_on_device: bool = False, serialization_path: Optional[str] = None,
                         use_graph: bool = True) -> TensorParallelNeuronModel:
    """Trace (graph-capture) a TP model for every example-input bucket.  Compiler-specific
    arguments of the reference (compiler_workdir/args, inline_weights_to_neff, max_parallel_
    compilations) are accepted and ignored: there is no compiler step on MI355X."""
    buckets = _buckets(example_inputs)
    if isinstance(func, torch.nn.Module):
        mod = func
        func = lambda: mod  # noqa: E731  (in-process only)
    if _spmd_context(tp_degree):
        local = _LocalTraced(func, buckets, checkpoint_loader_callable, use_graph=use_graph)
        model = TensorParallelNeuronModel(local=local, tp_degree=tp_degree)
    else:
        pool = SpmdWorkerPool(tp_degree, _pool_build, (func, [tuple(t.cpu() for t in b) for b in buckets],
                                                       checkpoint_loader_callable, None))
        model = TensorParallelNeuronModel(pool=pool, tp_degree=tp_degree)
    if serialization_path:
        model.save(serialization_path)
    return model


def parallel_model_save(model: TensorParallelNeuronModel, save_dir: str) -> None:
    model.save(save_dir)


def parallel_model_load(model_dir: str, func: Optional[Callable] = None) -> TensorParallelNeuronModel:
    """Rebuild a saved traced model: the model code comes from `func` (or the recorded importable
    path), weights/states from the per-rank safetensors, graphs are re-captured."""
    with open(os.path.join(model_dir, _META)) as f:
        meta = json.load(f)
    tp = int(meta["tp_degree"])
    if func is None:
        assert meta.get("func"), "saved model has no importable func; pass func="
        func = _resolve(meta["func"])
    buckets = [tuple(torch.zeros(s, dtype=_DT[d]) for s, d in b) for b in meta["buckets"]]
    if _spmd_context(tp):
        rank = ps.get_tensor_model_parallel_rank()
        local = _LocalTraced(func, buckets, weights_file=os.path.join(model_dir, f"tp_{rank:02d}.safetensors"))
        return TensorParallelNeuronModel(local=local, tp_degree=tp)
    pool = SpmdWorkerPool(tp, _pool_build, (func, buckets, None, model_dir))
    return TensorParallelNeuronModel(pool=pool, tp_degree=tp)


# ---------------------------------------------------------------------------- weight sharding helpers
def get_sharded_checkpoint(checkpoint: Dict[str, torch.Tensor], model: torch.nn.Module, rank: int,
                           tp_degree: int) -> Dict[str, torch.Tensor]:
    """Replace the full tensors in `checkpoint` by `rank`'s shards (in place; also returned)."""
    local = shard_state_dict(model, checkpoint, tp_degree, rank, strict=False)
    checkpoint.update(local)
    return checkpoint


def create_local_weight(rank: int, world_size: int, full_weight: torch.Tensor, partition_dim: int,
                        per_partition_size: int, stride: int, out_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    w = shard_tensor(full_weight, {"tp": True, "dim": partition_dim, "stride": stride, "qkv": None}, world_size, rank)
    assert w.shape[partition_dim] == per_partition_size, (w.shape, per_partition_size)
    if out_weight is not None:
        out_weight.data.copy_(w)
        return out_weight
    return w


def create_local_weight_qkv(rank: int, world_size: int, full_weight: torch.Tensor, partition_dim: int, q_len: int,
                            kv_len: int, out_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused [q; k; v] weight (rows): each of q / k / v split separately over the TP ranks."""
    assert partition_dim == 0
    w = shard_tensor(full_weight, {"tp": True, "dim": 0, "stride": 1, "qkv": (q_len, kv_len, 1)}, world_size, rank)
    if out_weight is not None:
        out_weight.data.copy_(w)
        return out_weight
    return w


def shard_children(module: torch.nn.Module, checkpoint: Dict[str, torch.Tensor], prefix: str, dtype, rank: int,
                   tp_degree: int) -> None:
    """Shard (in place) every checkpoint entry under `prefix` that belongs to a TP parameter of
    `module`, casting floating tensors to `dtype`."""
    for name, p in module.named_parameters():
        key = prefix + name
        if key in checkpoint:
            t = shard_tensor(checkpoint[key], _attrs(p), tp_degree, rank)
            checkpoint[key] = t.to(dtype) if (dtype is not None and t.is_floating_point()) else t
