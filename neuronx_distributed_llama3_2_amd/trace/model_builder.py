"""ModelBuilder: several bucketed models (e.g. context encoding and token generation) that share
one set of TP-sharded weights, traced into an NxDModel (reference: src/neuronx_distributed/trace/
model_builder.py:37-586).

    builder = ModelBuilder(router=None, tp_degree=2, checkpoint_loader=load_full_state_dict)
    builder.add("context_encoding", BaseModelInstance(build_cte, {}), [(ids_128,), (ids_512,)])
    builder.add("token_generation", BaseModelInstance(build_tkg, {}), [(ids_1,)])
    nxd = builder.trace()          # NxDModelExecutor: nxd(ids) routes on the input shape
    builder.shard_checkpoint(dir)  # tp{r}_sharded_checkpoint.safetensors for every rank

"trace" = load this rank's shard, capture one hipGraph per bucket; there are no HLOs / NEFFs.
Modules returned by different instances may be the SAME object (shared weights, loaded once).
Weight-layout optimisation of the reference (priority model HLO stubs) has no counterpart: the
hipBLASLt solutions are picked per GEMM shape by the tuner (csrc/gemm.cpp).
"""

from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state as ps
from ..parallel_layers.sharding import shard_state_dict
from .runtime import SpmdWorkerPool, worker_device
from .spmd import NxDModel, NxDModelExecutor, SPMDBucketModel, StateInitializer
from .trace import _buckets, _spmd_context


class BaseModelInstance:
    def __init__(self, module_cls: Callable, input_output_aliases=None):
        self.module_cls = module_cls
        self.module = None
        self.input_output_aliases = [input_output_aliases]

    def load_module(self):
        self.module = self.module_cls()

    def get(self, bucket_rank, **kwargs):
        return self.module, self.input_output_aliases[0]


class ModelContainer:
    def __init__(self, model_instance: BaseModelInstance, example_inputs, compiler_args=None, bucket_config=None,
                 priority_model_idx=None):
        self.model_instance = model_instance
        self.example_inputs = _buckets(example_inputs)
        self.compiler_args = compiler_args
        self.bucket_config = bucket_config
        self.priority_model_idx = priority_model_idx


def _bucket_tokens(example) -> int:
    """GEMM row count of a bucket: B*S of its first input (ids [B, S], or [B, S, H] activations)."""
    t = example[0]
    if t.dim() >= 3 or t.is_floating_point():
        shape = t.shape[:-1]
    else:
        shape = t.shape
    n = 1
    for d in shape:
        n *= int(d)
    return max(n, 1)


def _build_nxd(rank, world, collection, checkpoint_loader, router, states, use_graph=True):
    dev = worker_device(rank, world) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda" and dist.is_initialized() and dist.get_backend() != "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    models: Dict[str, SPMDBucketModel] = {}
    unique = {}
    for key, mc in collection.items():
        if mc.model_instance.module is None:
            mc.model_instance.load_module()
        mod, _ = mc.model_instance.get(0)
        unique[id(mod)] = mod
        models[key] = SPMDBucketModel(mod, [tuple(t.to(dev) for t in b) for b in mc.example_inputs], use_graph)
    if checkpoint_loader is not None:
        full = checkpoint_loader()
        for mod in unique.values():
            mod.load_state_dict(shard_state_dict(mod, full, world, rank, strict=False), strict=False)
    for mod in unique.values():
        mod.to(dev).eval()
    for mc in collection.values():
        if mc.priority_model_idx is not None:
            # weight layout chosen at the priority bucket's shapes, shared by every bucket
            # (reference trace/model_builder.py:457-586)
            from .weight_layout import optimize_weight_layout

            mod, _ = mc.model_instance.get(0)
            optimize_weight_layout(mod, _bucket_tokens(mc.example_inputs[mc.priority_model_idx]))
    state_init = StateInitializer(*states, tp_degree=world, device=dev) if states else None
    nxd = NxDModel(models, tp_degree=world, router=router, state_initializer=state_init)
    with torch.no_grad():
        nxd.initialize_with_saved_weights()
    return _NoGradExecutor(nxd)


class _NoGradExecutor(NxDModelExecutor):
    @torch.no_grad()
    def forward(self, *inputs):
        return self.nxd_model([t.to(self._dev()) for t in inputs])

    def _dev(self):
        m = next(iter(self.nxd_model.models.values())).module
        p = next(m.parameters(), None)
        return p.device if p is not None else torch.device("cpu")


class _PoolExecutor(torch.nn.Module):
    def __init__(self, pool: SpmdWorkerPool):
        super().__init__()
        self.pool = pool

    def forward(self, *inputs):
        return self.pool(*inputs)

    def close(self):
        self.pool.close()


class ModelBuilder:
    def __init__(self, router: Optional[Callable], tp_degree: int, checkpoint_loader: Optional[Callable],
                 compiler_workdir: Optional[str] = None, master_proc_env_vars: Optional[Dict[str, str]] = None):
        self.router = router
        self.tp_degree = tp_degree
        self.checkpoint_loader = checkpoint_loader
        self.compiler_workdir = compiler_workdir or "/tmp/nxd_model/"
        self.master_proc_env_vars = master_proc_env_vars
        self.model_collection: Dict[str, ModelContainer] = {}
        self.states = None

    def add(self, key: str, model_instance: BaseModelInstance, example_inputs, compiler_args=None,
            bucket_config=None, priority_model_idx: Optional[int] = None) -> "ModelBuilder":
        self.model_collection[key] = ModelContainer(model_instance, example_inputs, compiler_args, bucket_config,
                                                    priority_model_idx)
        return self

    def add_states(self, shapes: Dict[str, Sequence[int]], dtypes: Dict[str, torch.dtype]) -> "ModelBuilder":
        """Optional state tensors (zero-initialised per rank at initialisation)."""
        self.states = (shapes, dtypes)
        return self

    def trace(self, tp_degree: Optional[int] = None, initialize_model_weights: bool = True):
        if tp_degree is not None:
            self.tp_degree = tp_degree
        if self.master_proc_env_vars:
            os.environ.update(self.master_proc_env_vars)
        loader = self.checkpoint_loader if initialize_model_weights else None
        if _spmd_context(self.tp_degree):
            return _build_nxd(ps.get_tensor_model_parallel_rank(), self.tp_degree, self.model_collection, loader,
                              self.router, self.states)
        pool = SpmdWorkerPool(self.tp_degree, _build_nxd, (self.model_collection, loader, self.router, self.states))
        return _PoolExecutor(pool)

    def shard_checkpoint(self, serialize_path: str) -> None:
        """Write `tp{rank}_sharded_checkpoint.safetensors` for every rank from the full checkpoint
        (parameter partition attributes of the first model decide the layout)."""
        from safetensors.torch import save_file

        assert self.checkpoint_loader is not None, "shard_checkpoint needs a checkpoint_loader"
        os.makedirs(serialize_path, exist_ok=True)
        mc = next(iter(self.model_collection.values()))
        if mc.model_instance.module is None:
            mc.model_instance.load_module()
        model, _ = mc.model_instance.get(0)
        full = self.checkpoint_loader()
        for rank in range(self.tp_degree):
            local = shard_state_dict(model, full, self.tp_degree, rank, strict=False)
            save_file({k: v.contiguous() for k, v in local.items()},
                      os.path.join(serialize_path, f"tp{rank}_sharded_checkpoint.safetensors"))
