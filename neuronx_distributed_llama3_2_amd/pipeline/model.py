"""NxDPPModel: pipeline-parallel wrapper — trace, partition, and a 1F1B / interleaved runtime over
RCCL point-to-point (reference: src/neuronx_distributed/pipeline/model.py:54-1641; same
constructor keywords and run_train / run_eval / local_* API).

Runtime (MI355X-first, no XLA graph breaks, no mark_step):
* the model is traced with torch.fx (decoder layers / TP layers are leaves) and split before the
  chosen transformer layers (`pipeline_cuts`, or evenly with `auto_partition`); with
  `virtual_pipeline_size` V each rank owns V chunks (virtual stages chunk*PP + rank);
* non-local stage submodules are dropped right after partitioning, so each rank only ever
  materialises / moves / optimises its own parameters;
* compute tasks run in the order of the schedule generators (pipeline/scheduler.py); every group
  of sends/receives between two compute tasks goes out as one `batch_isend_irecv`, activations and
  their gradients are real RCCL p2p transfers of exactly the tensors a boundary needs
  (pass-through values are forwarded hop by hop and their gradients accumulated on the way back);
* tensor shapes for each boundary are discovered once per input shape by a metadata pass over the
  gloo pipeline group;
* the last micro-batch's backward arms the backward-overlapped DP gradient buckets
  (parallel/grad_buffer.py); shared parameters across stages (tied embeddings) get their
  gradients all-reduced between the owning stages; sent outputs can be deallocated
  (`deallocate_pipeline_outputs`) to cut activation memory.
"""

from __future__ import annotations

import math
from collections import defaultdict
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.fx as fx
from torch import nn

from ..parallel.grad_buffer import arm_grad_sync
from ..parallel_layers import parallel_state as ps
from ..utils.logger import get_logger
from .comm import P2PGroup, recv_python_object, send_python_object
from .partition import (
    analyze_pipeline_module,
    analyze_shared_weights_across_stages,
    create_partitions,
    partition_traced_model,
)
from .scheduler import (
    BackwardPostprocessTask,
    BackwardPreprocessTask,
    BackwardStepTask,
    ForwardPostprocessTask,
    ForwardPreprocessTask,
    ForwardStepTask,
    InferenceSchedule,
    ReduceGradsTask,
    Train1F1BSchedule,
    TrainInterleavedSchedule,
)
from .timeline import PPTimeline
from .trace import trace_model

logger = get_logger()


def _record_saved(saved: set):
    def pack(t):
        if isinstance(t, torch.Tensor) and t.device.type != "meta":
            saved.add(t.untyped_storage().data_ptr())
        return t

    return pack


def _identity(t):
    return t


class NxDPPModel(nn.Module):
    def __init__(self, module: nn.Module, transformer_layer_cls=None, num_microbatches: int = 1,
                 virtual_pipeline_size: int = 1, output_loss_value_spec=None, return_mb_loss: bool = False,
                 broadcast_and_average_loss: bool = False, pipeline_cuts: Optional[List[str]] = None,
                 input_names: Optional[List[str]] = None, leaf_module_cls: Optional[List[Any]] = None,
                 autowrap_functions=None, autowrap_modules=None, autowrap_obj_methods=None, tracer_cls=None,
                 param_init_fn=None, trace_file_path=None, use_zero1_optimizer: bool = False,
                 use_optimizer_wrapper: bool = False, use_model_wrapper: bool = False, return_loss_on_cpu: bool = True,
                 deallocate_pipeline_outputs: bool = False, auto_partition: bool = False,
                 fuse_microbatches: bool = False, _debug_mode: bool = False, _debug_pp_size: int = 1,
                 _debug_pp_rank: int = 0, _delay_tracing: bool = False, _all_reduce_send_recv: bool = False,
                 _fused_send_recv: bool = False, _fused_fwd_bwd: bool = False, _use_gloo_for_metadata_comm: bool = False,
                 _turn_off_odd_even_scheduler: bool = False, **unused):
        super().__init__()
        # not a registered child: moving / materialising this wrapper touches only the local stages
        self.__dict__["original_torch_module"] = module
        self.transformer_layer_cls = transformer_layer_cls
        self.num_microbatches = num_microbatches
        self.virtual_pipeline_size = virtual_pipeline_size
        self.output_loss_value_spec = output_loss_value_spec
        self.return_mb_loss = return_mb_loss
        self.broadcast_and_average_loss = broadcast_and_average_loss
        self.return_loss_on_cpu = return_loss_on_cpu
        self.deallocate_pipeline_outputs = deallocate_pipeline_outputs
        # fuse_microbatches (reference :230-233): there the whole step becomes one XLA graph.  Here
        # the step never blocks the host between micro-batches anyway (async p2p, device losses);
        # the flag keeps the reference's contract that the loss stays on the device.
        self.fuse_microbatches = fuse_microbatches
        if fuse_microbatches and return_loss_on_cpu:
            logger.warning("return_loss_on_cpu will be set to False when fuse_microbatches is set to True.")
            self.return_loss_on_cpu = False
        self.stats: Dict[str, int] = {}
        self.param_init_fn = param_init_fn
        self.input_names = input_names
        if _debug_mode:
            self.pp_size, self.pp_rank = _debug_pp_size, _debug_pp_rank
        else:
            self.pp_size = ps.get_pipeline_model_parallel_size()
            self.pp_rank = ps.get_pipeline_model_parallel_rank()
        self._debug = _debug_mode
        self.num_stages = self.pp_size * virtual_pipeline_size
        # ---- trace + partition
        leaves = list(leaf_module_cls or [])
        if transformer_layer_cls is not None:
            leaves.append(transformer_layer_cls)
        gm = trace_model(module, input_names, leaf_modules=leaves, autowrap_functions=autowrap_functions or (),
                         autowrap_modules=autowrap_modules or (), tracer_cls=tracer_cls)
        layer_names = [n.target for n in gm.graph.nodes
                       if n.op == "call_module" and transformer_layer_cls is not None
                       and isinstance(gm.get_submodule(n.target), transformer_layer_cls)]
        if pipeline_cuts is None:
            if not auto_partition and self.num_stages > 1:
                raise ValueError("provide pipeline_cuts or set auto_partition=True")
            starts = create_partitions(self.num_stages, len(layer_names))
            pipeline_cuts = [layer_names[i] for i in starts]
        else:
            # reference cuts name the LAST layer of a stage; we cut before the following layer
            pipeline_cuts = [layer_names[layer_names.index(c) + 1] if c in layer_names else c for c in pipeline_cuts]
        if len(pipeline_cuts) != self.num_stages - 1:
            raise ValueError(f"{len(pipeline_cuts)} cuts for {self.num_stages} stages")
        self.pipeline_cuts = pipeline_cuts
        split = partition_traced_model(gm, pipeline_cuts)
        self.ios = analyze_pipeline_module(split, self.num_stages)
        self.shared_weights = analyze_shared_weights_across_stages(split, self.num_stages)
        self._wiring = split.graph
        self._out_node = [n for n in split.graph.nodes if n.op == "output"][0]
        self.local_stage_ids = [c * self.pp_size + self.pp_rank for c in range(virtual_pipeline_size)]
        self.local_stage_modules = nn.ModuleList([getattr(split, f"submod_{s}") for s in self.local_stage_ids])
        self._local_index = {s: i for i, s in enumerate(self.local_stage_ids)}
        self._build_name_map(module)
        self._release_nonlocal(split)
        self._shared_groups = None
        self._meta: Dict[int, List[Tuple[str, torch.Size, torch.dtype, bool]]] = {}
        self._meta_key = None
        self.fused_send_recv, self.fused_fwd_bwd = _fused_send_recv, _fused_fwd_bwd
        self.use_odd_even = (num_microbatches == self.pp_size) and not _turn_off_odd_even_scheduler and \
            virtual_pipeline_size > 1
        if not _debug_mode and dist.is_initialized() and self.pp_size > 1:
            ps.initialize_pp_gloo_groups()
            self._build_shared_groups()
        self.timeline = PPTimeline(trace_file_path if not _debug_mode else None, self.pp_rank)
        from ..trainer import hooks

        hooks.execute_all_hooks(self)
        del gm, split

    def _release_nonlocal(self, split: fx.GraphModule) -> None:
        """Swap parameters/buffers only used by other ranks' stages for meta tensors (frees host or
        device memory of a model that was built whole)."""
        keep = {id(t) for m in self.local_stage_modules for t in list(m.parameters()) + list(m.buffers())}
        for s in range(self.num_stages):
            if s in self._local_index:
                continue
            for mod in getattr(split, f"submod_{s}").modules():
                for k, p in list(mod._parameters.items()):
                    if p is not None and id(p) not in keep and p.device.type != "meta":
                        mod._parameters[k] = nn.Parameter(torch.empty_like(p, device="meta"), p.requires_grad)
                for k, b in list(mod._buffers.items()):
                    if b is not None and id(b) not in keep and b.device.type != "meta":
                        mod._buffers[k] = torch.empty_like(b, device="meta")

    # ------------------------------------------------------------------ module API
    def _build_name_map(self, module: nn.Module) -> None:
        """split_module renames submodule paths ("model.layers.3" -> "model_layers_3"): map every
        local stage's tensor names back to the original model's qualified names (by identity)."""
        aliases: Dict[int, List[str]] = defaultdict(list)
        for n, t in list(module.named_parameters(remove_duplicate=False)) + list(module.named_buffers(remove_duplicate=False)):
            aliases[id(t)].append(n)
        self._orig = []
        for m in self.local_stage_modules:
            mp = {}
            for n, t in list(m.named_parameters(remove_duplicate=False)) + list(m.named_buffers(remove_duplicate=False)):
                cands = aliases.get(id(t), [n])
                flat = n.replace(".", "_")
                mp[n] = next((c for c in cands if c.replace(".", "_") == flat), cands[0])
            self._orig.append(mp)

    def local_named_parameters(self, *args, **kwargs):
        for i, m in enumerate(self.local_stage_modules):
            for n, p in m.named_parameters(*args, **kwargs):
                yield self._orig[i].get(n, n), p

    def local_parameters(self):
        for _, p in self.local_named_parameters():
            yield p

    def local_named_buffers(self, *args, **kwargs):
        for i, m in enumerate(self.local_stage_modules):
            for n, b in m.named_buffers(*args, **kwargs):
                yield self._orig[i].get(n, n), b

    def local_named_children(self):
        for i, m in enumerate(self.local_stage_modules):
            yield f"stage{self.local_stage_ids[i]}", m

    def local_named_modules(self, *args, **kwargs):
        for i, m in enumerate(self.local_stage_modules):
            for n, mm in m.named_modules(*args, **kwargs):
                yield f"stage{self.local_stage_ids[i]}" + (f".{n}" if n else ""), mm

    def local_state_dict(self, *args, **kwargs):
        """State dict of the local stages keyed by the ORIGINAL model's names."""
        out = {}
        for i, m in enumerate(self.local_stage_modules):
            for k, v in m.state_dict(*args, **kwargs).items():
                out[self._orig[i].get(k, k)] = v
        return out

    def load_state_dict(self, state_dict, strict: bool = True):
        missing, used = [], set()
        for i, m in enumerate(self.local_stage_modules):
            sub = {}
            for k in m.state_dict():
                ok = self._orig[i].get(k, k)
                if ok in state_dict:
                    sub[k] = state_dict[ok]
                    used.add(ok)
                else:
                    missing.append(ok)
            m.load_state_dict(sub, strict=False)
        if strict and missing:
            raise RuntimeError(f"missing keys for the local pipeline stages: {missing[:8]}")
        return missing, sorted(set(state_dict) - used)

    def parameters(self, recurse: bool = True):
        return self.local_parameters()

    def named_parameters(self, *args, **kwargs):
        return self.local_named_parameters(*args, **kwargs)

    def forward(self, *args, **kwargs):
        raise RuntimeError("NxDPPModel: use run_train(**batch) / run_eval(**batch)")

    # ------------------------------------------------------------------ helpers
    def _owner(self, stage: int) -> int:
        return ps.get_pipeline_model_parallel_global_ranks()[stage % self.pp_size]

    def _split_batch(self, kwargs) -> List[Dict[str, Any]]:
        mbs = [dict() for _ in range(self.num_microbatches)]
        for k, v in kwargs.items():
            if isinstance(v, torch.Tensor):
                assert v.shape[0] % self.num_microbatches == 0, f"batch of {k} not divisible by num_microbatches"
                for i, c in enumerate(v.chunk(self.num_microbatches, dim=0)):
                    mbs[i][k] = c
            else:
                for i in range(self.num_microbatches):
                    mbs[i][k] = v
        return mbs

    def _stage_args(self, stage: int, env: Dict[str, Any], batch: Dict[str, Any]):
        io = self.ios[stage]
        args = []
        for name in io.inputs:
            if name in env:
                args.append(env[name])
            elif name in batch:
                args.append(batch[name])
            else:
                args.append(None)
        return args

    def _run_stage(self, stage: int, env: Dict[str, Any], batch: Dict[str, Any]):
        mod = self.local_stage_modules[self._local_index[stage]]
        out = mod(*self._stage_args(stage, env, batch))
        io = self.ios[stage]
        sub_node = f"submod_{stage}"
        env[sub_node] = out
        for name in io.outputs:
            if name != sub_node:
                # getitem_k of a multi-output submodule: find its index in the wiring graph
                idx = self._getitem_index(name)
                env[name] = out[idx]
        return out

    def _getitem_index(self, name: str) -> int:
        if not hasattr(self, "_gi_cache"):
            self._gi_cache = {}
            for n in self._wiring.nodes:
                if n.op == "call_function" and getattr(n.target, "__name__", "") == "getitem":
                    self._gi_cache[n.name] = n.args[1]
        return self._gi_cache[name]

    def _final_output(self, env):
        def build(a):
            if isinstance(a, fx.Node):
                return env.get(a.name)
            if isinstance(a, (list, tuple)):
                return type(a)(build(x) for x in a)
            if isinstance(a, dict):
                return {k: build(v) for k, v in a.items()}
            return a

        return build(self._out_node.args[0])

    def _loss_from_output(self, out):
        if self.output_loss_value_spec is not None and not isinstance(out, dict):
            from ..utils.serialization import find_loss_from_output_and_spec

            return find_loss_from_output_and_spec(out, self.output_loss_value_spec)
        if isinstance(out, dict):
            return out["loss"]
        if isinstance(out, (list, tuple)):
            return out[0]
        return out

    # ------------------------------------------------------------------ metadata (shape) pass
    def _infer_meta(self, batch0: Dict[str, Any]) -> None:
        key = tuple((k, tuple(v.shape)) for k, v in sorted(batch0.items()) if isinstance(v, torch.Tensor))
        if key == self._meta_key:
            return
        self._meta = {}
        with torch.no_grad():
            for s in range(self.num_stages):
                owner = self._owner(s)
                me = dist.get_rank()
                if owner == me:
                    env = {}
                    if s > 0:
                        metas = recv_python_object(self._owner(s - 1)) if self._owner(s - 1) != me else self._meta[s - 1]
                        self._meta[s - 1] = metas
                        dev = self._device()
                        for name, shape, dtype, _ in metas:
                            env[name] = torch.zeros(shape, dtype=dtype, device=dev)
                    self._run_stage(s, env, batch0)
                    io = self.ios[s]
                    metas = []
                    for name in io.send:
                        t = env[name]
                        metas.append((name, tuple(t.shape), t.dtype, bool(t.is_floating_point())))
                    self._meta[s] = metas
                    if s + 1 < self.num_stages and self._owner(s + 1) != me:
                        send_python_object(metas, self._owner(s + 1))
        self._meta_key = key

    def _device(self):
        p = next(self.local_stage_modules.parameters(), None)
        if p is not None:
            return p.device
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    # ------------------------------------------------------------------ execution
    def _schedule(self, train: bool):
        if not train:
            return InferenceSchedule(self.num_microbatches, self.pp_size, self.pp_rank) if self.virtual_pipeline_size == 1 \
                else None
        if self.virtual_pipeline_size == 1:
            return Train1F1BSchedule(self.num_microbatches, self.pp_size, self.pp_rank)
        return TrainInterleavedSchedule(self.num_microbatches, self.virtual_pipeline_size, self.pp_size, self.pp_rank,
                                        self.fused_send_recv, self.fused_fwd_bwd, self.use_odd_even)

    def _execute(self, batch: Dict[str, Any], train: bool):
        mbs = self._split_batch(batch)
        if self.num_stages > 1:
            self._infer_meta(mbs[0])
        dev = self._device()
        PP = self.pp_size
        envs: Dict[Tuple[int, int], Dict[str, Any]] = defaultdict(dict)   # (mb, stage) -> values
        recv_leaves: Dict[Tuple[int, int], Dict[str, torch.Tensor]] = {}
        grads_in: Dict[Tuple[int, int], Dict[str, torch.Tensor]] = {}
        losses: List[Optional[torch.Tensor]] = [None] * self.num_microbatches
        last_stage = self.num_stages - 1
        group = P2PGroup()
        if train:
            tasks = [t for step in self._schedule(True).steps() for t in step]
        elif self.virtual_pipeline_size == 1:
            tasks = [t for step in InferenceSchedule(self.num_microbatches, PP, self.pp_rank).steps() for t in step]
        else:
            # interleaved forward-only: the interleaved schedule's all-warmup ordering (micro-batches
            # advance in groups of PP per chunk, so neighbours' send/recv groups pair up)
            sched = TrainInterleavedSchedule(self.num_microbatches, self.virtual_pipeline_size, PP, self.pp_rank)
            sched.num_warmup_steps = sched.num_microbatches_steps
            sched.num_steady_state_steps = 0
            sched.num_remaining_steps = 0
            fwd = (ForwardPreprocessTask, ForwardStepTask, ForwardPostprocessTask)
            tasks = [t for step in sched.steps() for t in step if isinstance(t, fwd)]
        n_bwd = sum(1 for t in tasks if isinstance(t, BackwardStepTask))
        bwd_done = 0
        outputs = [None] * self.num_microbatches
        scale = 1.0 / self.num_microbatches

        def stage_of(task):
            return task.model_chunk * PP + self.pp_rank

        dealloc = train and self.deallocate_pipeline_outputs
        saved_storages: Dict[Tuple[int, int], set] = {}
        self.stats = {"held_output_bytes": 0, "held_output_bytes_peak": 0, "deallocated_outputs": 0}

        for task in tasks:
            if isinstance(task, (ForwardStepTask, BackwardStepTask)):
                group.issue()          # exchanges go out; nobody waits for a send
            elif isinstance(task, ReduceGradsTask):
                group.flush()
            if isinstance(task, ForwardPreprocessTask):
                s = stage_of(task)
                if s == 0:
                    continue
                buf = {}
                for name, shape, dtype, rg in self._meta[s - 1]:
                    t = torch.empty(shape, dtype=dtype, device=dev)
                    group.recv(t, self._owner(s - 1))
                    buf[name] = t
                recv_leaves[(task.mb, s)] = buf
            elif isinstance(task, ForwardStepTask):
                s = stage_of(task)
                label = f"mb_{task.mb}_stage{s}_ForwardStep"
                self.timeline.mark_event_start(label)
                env = envs[(task.mb, s)]
                leaves_in = recv_leaves.get((task.mb, s), {})
                group.wait_for(leaves_in.values())   # only this task's inputs are waited for
                for name, t in leaves_in.items():
                    if train and t.is_floating_point():
                        t.requires_grad_(True)
                    env[name] = t
                with torch.set_grad_enabled(train):
                    if dealloc and s != last_stage:
                        saved = saved_storages[(task.mb, s)] = set()
                        with torch.autograd.graph.saved_tensors_hooks(_record_saved(saved), _identity):
                            self._run_stage(s, env, mbs[task.mb])
                    else:
                        self._run_stage(s, env, mbs[task.mb])
                if s == last_stage:
                    out = self._final_output(env)
                    loss = self._loss_from_output(out)
                    losses[task.mb] = loss
                    outputs[task.mb] = out if self.return_mb_loss or not train else None
                self.timeline.mark_event_end(label)
            elif isinstance(task, ForwardPostprocessTask):
                s = stage_of(task)
                if s == last_stage:
                    continue
                env = envs[(task.mb, s)]
                for name, _, _, _ in self._meta[s]:
                    group.send(env[name].detach(), self._owner(s + 1))
                if train:
                    self._account_outputs(env, recv_leaves.get((task.mb, s), {}), s,
                                          saved_storages.pop((task.mb, s), None) if dealloc else None)
            elif isinstance(task, BackwardPreprocessTask):
                s = stage_of(task)
                if s == last_stage:
                    continue
                gbuf = {}
                for name, shape, dtype, rg in self._meta[s]:
                    if rg:
                        g = torch.empty(shape, dtype=dtype, device=dev)
                        group.recv(g, self._owner(s + 1))
                        gbuf[name] = g
                grads_in[(task.mb, s)] = gbuf
            elif isinstance(task, BackwardStepTask):
                s = stage_of(task)
                label = f"mb_{task.mb}_stage{s}_BackwardStep"
                self.timeline.mark_event_start(label)
                bwd_done += 1
                if bwd_done == n_bwd:
                    arm_grad_sync(True)  # last backward of the step: overlap DP bucket reduction
                env = envs[(task.mb, s)]
                leaves = recv_leaves.get((task.mb, s), {})
                if s == last_stage:
                    losses_mb = losses[task.mb]
                    (losses_mb * scale).backward()
                else:
                    gin = grads_in.pop((task.mb, s), {})
                    group.wait_for(gin.values())
                    outs, grads = [], []
                    for name, g in gin.items():
                        t = env[name]
                        if name in leaves and t is leaves[name]:
                            # pass-through value: its gradient continues to the previous stage
                            t.grad = g if t.grad is None else t.grad + g
                        elif t.requires_grad:
                            outs.append(t)
                            grads.append(g)
                    if outs:
                        if any(getattr(t, "_nxd_dealloc_shape", None) is not None for t in outs):
                            # deallocated outputs: the C++ engine checks grads against the grad_fn's
                            # recorded input metadata, not the (now 1-element) tensor
                            torch.autograd.Variable._execution_engine.run_backward(
                                tuple(outs), tuple(grads), False, False, tuple(), True, True)
                        else:
                            torch.autograd.backward(outs, grads)
                    self._release_outputs(env, s)
                envs.pop((task.mb, s), None)
                self.timeline.mark_event_end(label)
            elif isinstance(task, BackwardPostprocessTask):
                s = stage_of(task)
                if s == 0:
                    continue
                leaves = recv_leaves.pop((task.mb, s), {})
                for name, shape, dtype, rg in self._meta[s - 1]:
                    if rg:
                        t = leaves[name]
                        g = t.grad if t.grad is not None else torch.zeros(shape, dtype=dtype, device=dev)
                        group.send(g, self._owner(s - 1))
            elif isinstance(task, ReduceGradsTask):
                self._reduce_shared_grads()
        group.flush()
        return losses, outputs

    def _account_outputs(self, env, leaves, s, saved) -> None:
        """After a stage's outputs were handed to the p2p runtime: track the activation bytes the
        stage keeps for backward and, with `deallocate_pipeline_outputs`, pseudo-free every output
        whose values backward does not need (reference pipeline/model.py:921-939): its storage is
        swapped for one element and only the autograd node is kept.  Unlike the reference, an
        output is freed only if no autograd node saved it (recorded by a saved-tensor hook during
        the stage forward), so it is safe for any stage boundary, e.g. a fused residual-add whose
        sum the norm backward re-reads."""
        held = 0
        for name, _, _, _ in self._meta[s]:
            t = env[name]
            if not isinstance(t, torch.Tensor) or (name in leaves and t is leaves[name]):
                continue
            base = t._base
            free = (saved is not None and t.requires_grad and t.numel() > 1
                    and t.untyped_storage().data_ptr() not in saved
                    # a whole-tensor alias (e.g. an identity TP mapping at TP=1) frees its base too
                    and (base is None or (base.numel() == t.numel() and base._base is None)))
            if free:
                t._nxd_dealloc_shape = t.shape
                if base is not None:
                    base.data = torch.empty((1,), dtype=base.dtype, device=base.device)
                t.data = torch.empty((1,), dtype=t.dtype, device=t.device)
                self.stats["deallocated_outputs"] += 1
            else:
                held += t.untyped_storage().nbytes()
        env["__held_bytes__"] = held
        self.stats["held_output_bytes"] += held
        self.stats["held_output_bytes_peak"] = max(self.stats["held_output_bytes_peak"],
                                                   self.stats["held_output_bytes"])

    def _release_outputs(self, env, s) -> None:
        self.stats["held_output_bytes"] -= env.pop("__held_bytes__", 0)

    def _build_shared_groups(self):
        """One group per cross-stage shared parameter set, created collectively over every PP mesh
        row (dist.new_group must be entered by all ranks with the same arguments)."""
        self._shared_groups = []
        me = dist.get_rank()
        for grp in self.shared_weights:
            positions = sorted({s % self.pp_size for s, _ in grp})
            mine, mine_ranks = None, []
            for row in ps.get_pipeline_model_parallel_group(as_list=True):
                ranks = [row[p] for p in positions]
                pg = dist.new_group(ranks) if len(ranks) > 1 else None
                if me in ranks:
                    mine, mine_ranks = pg, ranks
            self._shared_groups.append((grp, mine, mine_ranks))
            for s, name in grp:
                if s in self._local_index:
                    self.local_stage_modules[self._local_index[s]].get_parameter(name)._nxd_pp_shared = True

    def _reduce_shared_grads(self):
        if not self.shared_weights or self.pp_size == 1 or self._shared_groups is None:
            return
        for grp, pg, ranks in self._shared_groups:
            if pg is None or dist.get_rank() not in ranks:
                continue
            for s, name in grp:
                if s in self._local_index:
                    p = self.local_stage_modules[self._local_index[s]].get_parameter(name)
                    g = getattr(p, "main_grad", None)
                    g = p.grad if g is None else g
                    if g is not None:
                        dist.all_reduce(g, group=pg)
                    break

    def _finish_loss(self, losses):
        have = [l for l in losses if l is not None]
        if have:
            loss = torch.stack([l.detach().float() for l in have]).mean()
        else:
            loss = torch.zeros((), dtype=torch.float32, device=self._device())
        if self.broadcast_and_average_loss and self.pp_size > 1:
            # only the last stage holds the loss: sum over the PP group (zeros elsewhere)
            buf = loss.reshape(1).clone() if have else torch.zeros(1, dtype=torch.float32, device=self._device())
            dist.all_reduce(buf, group=ps.get_pipeline_model_parallel_group())
            dp = ps.get_data_parallel_size()
            if dp > 1:
                dist.all_reduce(buf, group=ps.get_data_parallel_group())
                buf /= dp
            loss = buf[0]
        if self.return_loss_on_cpu:
            loss = loss.cpu()
        return loss

    def run_train(self, **kwargs):
        self.local_stage_modules.train()
        losses, outputs = self._execute(kwargs, train=True)
        loss = self._finish_loss(losses)
        self.timeline.mark_step_end()
        if self.return_mb_loss:
            return [l.detach() if l is not None else None for l in losses]
        return loss

    @torch.no_grad()
    def run_eval(self, **kwargs):
        self.local_stage_modules.eval()
        losses, outputs = self._execute(kwargs, train=False)
        if self.return_mb_loss:
            return [l.detach() if l is not None else None for l in losses]
        return self._finish_loss(losses)
