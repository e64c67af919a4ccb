"""Training checkpoints: save_checkpoint / load_checkpoint / has_checkpoint / finalize_checkpoint
(reference: src/neuronx_distributed/trainer/checkpoint.py:50-853; on-disk layout unchanged):

    <dir>/<tag>/checkpoint                                      (begun marker)
    <dir>/<tag>/model/dp_rank_00[_ep_rank_XX]_tp_rank_XX_pp_rank_XX.pt   (+ .tensors/ with xser)
    <dir>/<tag>/optim/dp_rank_XX[_ep_rank_XX]_tp_rank_XX_pp_rank_XX.pt   (one per DP rank under ZeRO-1)
    <dir>/<tag>/scheduler.pt, user_content.pt
    <dir>/<tag>/done                                            (completion marker)

Every rank writes its own shard in parallel (no XLA rendezvous staggering); with `async_save` the
device->host copy happens synchronously (so training may mutate the weights right away) and the
file writes run on a background thread, overlapped with the following steps; `num_kept_ckpts`
garbage-collects the oldest completed tags and interrupted deletions.  Loads map to the current
GPU and use `weights_only=True`.
"""

from __future__ import annotations

import atexit
import concurrent.futures as cf
import os
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel_layers.parallel_state import (
    get_data_parallel_group,
    get_data_parallel_rank,
    get_expert_data_parallel_group,
    get_expert_data_parallel_rank,
    get_expert_model_parallel_rank,
    get_expert_model_parallel_size,
    get_pipeline_model_parallel_rank,
    get_tensor_model_parallel_rank,
    model_parallel_is_initialized,
)
from ..parallel_layers.utils import move_all_tensor_to_cpu
from ..utils.logger import get_logger
from ..utils.resilience import fault_point
from ..utils.serialization import assign_tensors_to_bins, xser_load, xser_load_info, xser_save, xser_tensors
from .checkpoint_storage import BaseCheckpointStorage, FilesysCheckpointStorage, create_checkpoint_storage

logger = get_logger()


def _ranks():
    if model_parallel_is_initialized():
        return (get_data_parallel_rank(), get_expert_model_parallel_rank(), get_tensor_model_parallel_rank(),
                get_pipeline_model_parallel_rank())
    return 0, 0, 0, 0


def _get_path(prefix: str, tp: bool = True, pp: bool = True, dp: bool = False, ep: bool = False) -> str:
    dpr, epr, tpr, ppr = _ranks()
    path = "dp_rank_{:02d}".format(dpr if dp else 0)
    if ep:
        path += "_ep_rank_{:02d}".format(epr)
    path += "_tp_rank_{:02d}".format(tpr if tp else 0)
    path += "_pp_rank_{:02d}".format(ppr if pp else 0)
    return f"{prefix}/{path}.pt"


def _barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _global_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _determine_remove_tags(checkpoint_dir: BaseCheckpointStorage, num_kept: Optional[int],
                           current: Optional[str] = None) -> List[str]:
    """Tags to delete: every tag without its `done` marker other than the one being written
    (interrupted saves and interrupted deletions — the reference only catches the latter,
    trainer/checkpoint.py:62-89) plus the oldest completed tags beyond `num_kept`."""
    tags = checkpoint_dir.list_checkpoint_tags()
    corrupted, completed = [], []
    for tag in tags:
        if checkpoint_dir.file_exists(os.path.join(tag, "done")):
            completed.append(tag)
        elif tag != current:
            corrupted.append(tag)
    remove = corrupted
    if num_kept is not None and num_kept != -1 and len(completed) > num_kept:
        remove += completed[: len(completed) - num_kept]
    return remove


def _snapshot(data: Any) -> Any:
    """Host copy that training can no longer mutate: device tensors are copied to the host, host
    tensors are cloned (`.cpu()` of a host tensor aliases it, and the async writer thread would
    otherwise serialise a state the next optimizer steps are already changing)."""
    if isinstance(data, torch.Tensor):
        t = data.detach()
        return t.clone() if t.device.type == "cpu" else t.cpu()
    if isinstance(data, dict):
        return {k: _snapshot(v) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return type(data)(_snapshot(v) for v in data)
    return data


def _snapshot_owned(data: Any, owned: set, counter: List[int]) -> Any:
    """Like _snapshot, but tensors whose xser tid (traversal index) is not in `owned` become meta
    placeholders of the same shape / dtype / EP flag (another replica writes their files)."""
    if isinstance(data, torch.Tensor):
        tid = counter[0]
        counter[0] += 1
        if tid in owned:
            out = _snapshot(data)
        else:
            out = torch.empty(data.shape, dtype=data.dtype, device="meta")
        if getattr(data, "expert_model_parallel", False):
            out.expert_model_parallel = True
        return out
    if isinstance(data, dict):
        return {k: _snapshot_owned(v, owned, counter) for k, v in data.items()}
    if isinstance(data, list):
        return [_snapshot_owned(v, owned, counter) for v in data]
    if isinstance(data, tuple):
        return tuple(_snapshot_owned(v, owned, counter) for v in data)
    return data


def _model_replica_group():
    """(group, size, rank) of the ranks holding identical copies of this rank's model shard: the
    expert-data-parallel group under EP, else the DP group."""
    if not (model_parallel_is_initialized() and dist.is_available() and dist.is_initialized()):
        return None, 1, 0
    g = get_expert_data_parallel_group() if get_expert_model_parallel_size() > 1 else get_data_parallel_group()
    return g, dist.get_world_size(group=g), dist.get_rank(group=g)


def _tag_expert_tensors(model, sd: Dict[str, Any]) -> None:
    """Mark expert-parallel entries of a model state dict (recorded in xser `.info.pt`)."""
    target = getattr(model, "module", model)
    if not hasattr(target, "named_parameters"):
        return
    for n, p in target.named_parameters():
        if getattr(p, "expert_model_parallel", False) and isinstance(sd.get(n), torch.Tensor):
            sd[n].expert_model_parallel = True


class CheckpointIOState:
    """Tracks the in-flight (possibly asynchronous) checkpoint and its save tasks."""

    def __init__(self, async_save: bool = False):
        self.async_save = async_save
        self.executor: Optional[cf.ThreadPoolExecutor] = cf.ThreadPoolExecutor(max_workers=1) if async_save else None
        self.pending: Optional[cf.Future] = None
        self.tasks: List[Tuple[Any, str, bool]] = []
        self.storage: Optional[BaseCheckpointStorage] = None
        self.tag: Optional[str] = None

    def wait_save(self) -> None:
        if self.pending is not None:
            fut, self.pending = self.pending, None
            fut.result()  # re-raises a failed async save (once; its tag never gets `done`)

    def begin(self, storage: BaseCheckpointStorage, tag: str) -> None:
        self.wait_save()
        _barrier()
        self.storage, self.tag = storage, str(tag)
        if _global_rank() == 0:
            storage.create_dir(self.tag, exist_ok=True)
            storage.save_text("1", os.path.join(self.tag, "checkpoint"))
        _barrier()
        self.tasks = []

    def add_save_task(self, obj: Any, filename: str, xser: bool = False, xser_ids=None, xser_ref: bool = True) -> None:
        if xser_ids is not None:
            # this rank stores only its bin of the shard's tensor files: copy just those to the host
            snap = _snapshot_owned(obj, set(xser_ids), [0])
        else:
            snap = _snapshot(obj) if self.async_save else move_all_tensor_to_cpu(obj)
        self.tasks.append((snap, filename, (xser, xser_ids, xser_ref)))

    def _run(self, tasks, storage):
        for obj, fn, (xser, ids, ref) in tasks:
            if xser and isinstance(storage, FilesysCheckpointStorage):
                path = os.path.join(storage.dirname(), fn)
                os.makedirs(os.path.dirname(path), exist_ok=True)
                xser_save(obj, path, tensor_ids=ids, write_ref=ref)
            else:
                storage.save_object(obj, fn)
            fault_point("ckpt_after_shard_write")

    def _finish(self, storage, tag, num_kept):
        _barrier()
        if _global_rank() == 0:
            fault_point("ckpt_before_done")
            storage.save_text("1", os.path.join(tag, "done"))
            for t in _determine_remove_tags(storage, num_kept, current=tag):
                if t != tag:
                    storage.remove_dir(t)

    def end(self, num_kept: Optional[int]) -> None:
        tasks, storage, tag = self.tasks, self.storage, self.tag
        self.tasks = []
        if self.async_save:
            def job():
                self._run(tasks, storage)
                return True

            fut = self.executor.submit(job)
            # completion marker after every rank's writes: done at the next begin()/finalize
            self.pending = fut
            self._deferred = (storage, tag, num_kept)
        else:
            self._run(tasks, storage)
            self._finish(storage, tag, num_kept)

    def finalize(self) -> None:
        if self.pending is not None:
            self.wait_save()
            storage, tag, num_kept = self._deferred
            self._finish(storage, tag, num_kept)


g_iostate: Optional[CheckpointIOState] = None


def _iostate(async_save: bool) -> CheckpointIOState:
    global g_iostate
    if g_iostate is None or g_iostate.async_save != async_save:
        if g_iostate is not None:
            g_iostate.finalize()
        g_iostate = CheckpointIOState(async_save)
        atexit.register(g_iostate.finalize)
    else:
        g_iostate.finalize()
    return g_iostate


def has_checkpoint(checkpoint_dir_str: str) -> bool:
    storage = create_checkpoint_storage(checkpoint_dir_str)
    try:
        storage.get_latest_tag()
        return True
    except RuntimeError:
        return False


def _model_state(model) -> Dict[str, Any]:
    if hasattr(model, "local_state_dict"):
        return model.local_state_dict()
    return model.state_dict()


def _is_zero1(optimizer) -> bool:
    inner = getattr(optimizer, "optimizer", optimizer)
    return bool(getattr(inner, "zero1", False)) or hasattr(inner, "inner")


def save_checkpoint(checkpoint_dir_str: str, tag: str, model=None, optimizer=None, scheduler=None,
                    user_content=None, num_workers: int = 8, use_xser: bool = False,
                    num_kept_ckpts: Optional[int] = None, async_save: bool = False, zero1_optimizer: bool = False,
                    use_zero1_dcp: bool = False) -> None:
    storage = create_checkpoint_storage(checkpoint_dir_str)
    st = _iostate(async_save)
    st.begin(storage, tag)
    dpr, _, _, _ = _ranks()
    ep = model_parallel_is_initialized() and get_expert_model_parallel_size() > 1
    if model is not None:
        # one writer per distinct model shard: DP rank 0, or with EP the expert-data-parallel rank 0
        # of every EP rank (EDP replicas hold identical shards and would race on one path;
        # reference trainer/checkpoint.py:496)
        group, gsize, grank = _model_replica_group()
        fn = os.path.join(str(tag), _get_path("model", ep=ep))
        if use_xser and gsize > 1 and isinstance(storage, FilesysCheckpointStorage):
            # DP-deduplicated xser save (reference trainer/checkpoint.py:430-470): the replicas split
            # the shard's tensor files by size; replica 0 also writes the structure and .info.pt.
            # Filesystem only: object stores get one complete object from the single writer below
            # (replicas writing partial objects to one key would overwrite each other).
            sd = _model_state(model)
            _tag_expert_tensors(model, sd)
            bins = assign_tensors_to_bins(xser_tensors(sd), gsize)
            st.add_save_task(sd, fn, xser=True, xser_ids=bins[grank], xser_ref=(grank == 0))
        elif (get_expert_data_parallel_rank() == 0) if ep else (dpr == 0):
            sd = _model_state(model)
            _tag_expert_tensors(model, sd)
            st.add_save_task(sd, fn, xser=use_xser)
    if optimizer is not None:
        zero = zero1_optimizer or _is_zero1(optimizer)
        if zero or dpr == 0:
            st.add_save_task(optimizer.state_dict(), os.path.join(str(tag), _get_path("optim", dp=zero, ep=ep)),
                             xser=use_xser)
    if _global_rank() == 0:
        if scheduler is not None:
            st.add_save_task(scheduler.state_dict(), os.path.join(str(tag), "scheduler.pt"))
        if user_content is not None:
            st.add_save_task(user_content, os.path.join(str(tag), "user_content.pt"))
    st.end(num_kept_ckpts)


def finalize_checkpoint() -> None:
    if g_iostate is not None:
        g_iostate.finalize()


def _load_obj(storage: BaseCheckpointStorage, filename: str, xser: bool, map_location, replicas: bool = False):
    if xser and isinstance(storage, FilesysCheckpointStorage):
        path = os.path.join(storage.dirname(), filename)
        group, gsize, grank = _model_replica_group() if replicas else (None, 1, 0)
        info = xser_load_info(path) if gsize > 1 else None
        if info is None:
            return xser_load(path, map_location=map_location)
        # replicas read 1/N of the tensor files each and broadcast them to the others (reference
        # _xser_load_data round-robin + broadcast, trainer/checkpoint.py:308-380)
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
            else torch.device("cpu")

        def tensor_loader(tid, f):
            owner = tid % gsize
            if owner == grank:
                t = torch.load(f, map_location=dev, weights_only=True).contiguous()
            else:
                t = torch.empty(tuple(info[tid]["shape"]), dtype=info[tid]["dtype"], device=dev)
            dist.broadcast(t, src=dist.get_global_rank(group, owner), group=group)
            return t   # stays on the broadcast device; load_state_dict copies into the parameters

        return xser_load(path, map_location=map_location, tensor_loader=tensor_loader)
    return storage.load_object(filename, map_location=map_location, weights_only=True)


def load_checkpoint(path: str, tag: Optional[str] = None, model=None, optimizer=None, scheduler=None,
                    num_workers: int = 8, strict: bool = True, weights_only: bool = True):
    """Load into model / optimizer / scheduler; returns the saved user content (or None)."""
    finalize_checkpoint()
    storage = create_checkpoint_storage(path)
    if tag is None:
        tag = storage.get_latest_tag()
    tag = str(tag)
    if not storage.dir_exists(tag):
        raise RuntimeError(f"checkpoint tag {tag} not found under {path}")
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    ep = model_parallel_is_initialized() and get_expert_model_parallel_size() > 1
    if model is not None:
        fn = os.path.join(tag, _get_path("model", ep=ep))
        xser = storage.dir_exists(fn + ".tensors")
        sd = _load_obj(storage, fn, xser, "cpu", replicas=True)
        target = getattr(model, "module", model)
        if hasattr(model, "load_state_dict"):
            model.load_state_dict(sd, strict=strict)
        else:
            target.load_state_dict(sd, strict=strict)
    if optimizer is not None:
        zero = _is_zero1(optimizer)
        fn = os.path.join(tag, _get_path("optim", dp=zero, ep=ep))
        xser = storage.dir_exists(fn + ".tensors")
        osd = _load_obj(storage, fn, xser, dev)
        optimizer.load_state_dict(osd)
    if scheduler is not None and storage.file_exists(os.path.join(tag, "scheduler.pt")):
        scheduler.load_state_dict(storage.load_object(os.path.join(tag, "scheduler.pt"), map_location="cpu",
                                                      weights_only=weights_only))
    user = None
    if storage.file_exists(os.path.join(tag, "user_content.pt")):
        user = storage.load_object(os.path.join(tag, "user_content.pt"), map_location="cpu", weights_only=weights_only)
    _barrier()
    return user
