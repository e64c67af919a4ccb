"""Process-group topology: the rank mesh -> TP / DP / PP / EP / expert-DP groups.

Same public API and rank layout as the reference (src/neuronx_distributed/parallel_layers/parallel_state.py:60-766):

* non-expert regions: ranks laid out row-major as [PP, DP, TP]  (TP contiguous);
* expert regions:     [PP, DP_exp, EP, TP] with DP = DP_exp * EP, so switching regions keeps
  every rank's PP and TP coordinates.

MI355X-first differences: groups are plain `torch.distributed` groups on the NCCL backend (= RCCL
over xGMI on ROCm) — no XLA replica-group meshes, no dummy all-reduce + mark_step warm-up, no
trn1 TP=4 special layout.  With TP contiguous, a TP group of <= 8 ranks is always one node, i.e.
one fully-connected xGMI island (7 point-to-point links per GPU), which is where the per-layer
sequence-parallel traffic goes.  Pipeline neighbours talk through real point-to-point send/recv
on the PP group (`get_pipeline_model_parallel_{next,prev}_rank`), so the reference's even/odd
parity 2-rank groups are not needed; `get_next_rank_group`/`get_prev_rank_group` remain for API
compatibility and return 2-rank groups built on demand.  A gloo PP group carries CPU metadata.
"""

from __future__ import annotations

import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from ..utils.logger import get_logger

logger = get_logger()

_TP_GROUP = None
_TP_MESH: Optional[List[List[int]]] = None
_DP_GROUP = None
_DP_MESH: Optional[List[List[int]]] = None
_PP_GROUP = None
_PP_MESH: Optional[List[List[int]]] = None
_EP_GROUP = None
_EP_MESH: Optional[List[List[int]]] = None
_EDP_GROUP = None
_EDP_MESH: Optional[List[List[int]]] = None
_PP_GLOO_GROUP = None
_WORLD_GLOO_GROUP = None
_PP_GLOBAL_RANKS: Optional[List[int]] = None
_NEXT_GROUP = None
_PREV_GROUP = None
_INITIALIZED = False

# overrides (used to shard checkpoints / trace without a process group, reference :49-53)
_MPU_TP_SIZE: Optional[int] = None
_MPU_TP_RANK: Optional[int] = None
_MPU_EP_SIZE: Optional[int] = None
_MPU_EP_RANK: Optional[int] = None
_MPU_PP_SIZE: Optional[int] = None
_MPU_PP_RANK: Optional[int] = None
_MPU_DP_SIZE: Optional[int] = None
_MPU_DP_RANK: Optional[int] = None


def _build_meshes(world_size: int, tp: int, pp: int, ep: int):
    if world_size % (tp * pp) != 0:
        raise RuntimeError(f"world_size ({world_size}) is not divisible by tp ({tp}) x pp ({pp})")
    dp = world_size // (tp * pp)
    if dp % ep != 0:
        raise RuntimeError(f"data parallel size ({dp}) must be divisible by expert parallel size ({ep})")
    edp = dp // ep
    ranks = torch.arange(world_size)
    nonexp = ranks.reshape(pp, dp, tp)
    exp = ranks.reshape(pp, edp, ep, tp)
    tp_mesh = nonexp.reshape(-1, tp).tolist()
    dp_mesh = nonexp.permute(0, 2, 1).reshape(-1, dp).tolist()
    pp_mesh = nonexp.permute(1, 2, 0).reshape(-1, pp).tolist()
    ep_mesh = exp.permute(0, 1, 3, 2).reshape(-1, ep).tolist()
    edp_mesh = exp.permute(0, 2, 3, 1).reshape(-1, edp).tolist()
    return dp, edp, tp_mesh, dp_mesh, pp_mesh, ep_mesh, edp_mesh


def _comm_options(high_priority: bool):
    """RCCL group options: the groups whose collectives overlap GEMMs (TP/SP, EP all-to-all) get a
    high-priority HIP stream, so the RCCL kernels are dispatched ahead of queued compute work
    (NXD_COMM_HIGH_PRIORITY=0 turns it off)."""
    if not high_priority or os.environ.get("NXD_COMM_HIGH_PRIORITY", "1") != "1":
        return None
    if dist.get_backend() != "nccl" or not hasattr(dist, "ProcessGroupNCCL"):
        return None
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def _assign(mesh: List[List[int]], rank: int, backend=None, high_priority: bool = False):
    """Create one group per mesh row (collectively on every rank) and return the one containing `rank`."""
    mine = None
    opts = _comm_options(high_priority) if backend is None else None
    for ranks in mesh:
        g = dist.new_group(ranks, backend=backend, pg_options=opts) if opts is not None else \
            dist.new_group(ranks, backend=backend)
        if rank in ranks:
            mine = g
    return mine


def initialize_model_parallel(tensor_model_parallel_size: int = 1, pipeline_model_parallel_size: int = 1,
                              expert_model_parallel_size: int = 1) -> None:
    """Build every group; must be called on all ranks after `torch.distributed.init_process_group`."""
    global _TP_GROUP, _TP_MESH, _DP_GROUP, _DP_MESH, _PP_GROUP, _PP_MESH, _EP_GROUP, _EP_MESH, _EDP_GROUP, _EDP_MESH
    global _PP_GLOBAL_RANKS, _INITIALIZED, _WORLD_GLOO_GROUP
    assert dist.is_initialized(), "torch.distributed must be initialised first"
    world = dist.get_world_size()
    rank = dist.get_rank()
    tp, pp, ep = tensor_model_parallel_size, pipeline_model_parallel_size, expert_model_parallel_size
    dp, edp, tp_mesh, dp_mesh, pp_mesh, ep_mesh, edp_mesh = _build_meshes(world, tp, pp, ep)
    logger.info("> initializing tensor model parallel with size %d", tp)
    logger.info("> initializing pipeline model parallel with size %d", pp)
    logger.info("> initializing data parallel with size %d", dp)
    if ep > 1:
        logger.info("> initializing expert model parallel with size %d (expert data parallel %d)", ep, edp)
    _TP_MESH, _DP_MESH, _PP_MESH, _EP_MESH, _EDP_MESH = tp_mesh, dp_mesh, pp_mesh, ep_mesh, edp_mesh
    from ..ops.gemm import set_overlap_safe
    from ..parallel.rccl_env import log_comm_config

    log_comm_config()
    # NXD_GEMM_NO_STREAMK=1: skip stream-K solutions of the heuristic list for runs whose GEMMs
    # overlap other kernels -- collectives, or the other SP part's kernels (opt-in; csrc/gemm.cpp)
    set_overlap_safe(os.environ.get("NXD_GEMM_NO_STREAMK", "0") == "1")
    _TP_GROUP = _assign(tp_mesh, rank, high_priority=True)
    _DP_GROUP = _assign(dp_mesh, rank)
    _PP_GROUP = _assign(pp_mesh, rank)
    _EP_GROUP = _assign(ep_mesh, rank, high_priority=True)
    _EDP_GROUP = _assign(edp_mesh, rank)
    for ranks in pp_mesh:
        if rank in ranks:
            _PP_GLOBAL_RANKS = list(ranks)
    if dist.get_backend() not in ("gloo", "fake"):   # ("fake": single-process rank emulation, tools/emulate_tp_rank.py)
        _WORLD_GLOO_GROUP = dist.new_group(list(range(world)), backend="gloo")
    else:
        _WORLD_GLOO_GROUP = dist.group.WORLD
    _INITIALIZED = True


def model_parallel_is_initialized() -> bool:
    return _INITIALIZED


def _mesh_or_group(group, mesh, as_list):
    if as_list:
        return mesh
    return group


def get_tensor_model_parallel_group(as_list: bool = False):
    assert _TP_GROUP is not None or as_list, "intra_layer_model parallel group is not initialized"
    return _mesh_or_group(_TP_GROUP, _TP_MESH, as_list)


def get_data_parallel_group(as_list: bool = False):
    assert _DP_GROUP is not None or as_list, "data parallel group is not initialized"
    return _mesh_or_group(_DP_GROUP, _DP_MESH, as_list)


def get_pipeline_model_parallel_group(as_list: bool = False):
    assert _PP_GROUP is not None or as_list, "pipeline_model parallel group is not initialized"
    return _mesh_or_group(_PP_GROUP, _PP_MESH, as_list)


def get_expert_model_parallel_group(as_list: bool = False):
    assert _EP_GROUP is not None or as_list, "expert model parallel group is not initialized"
    return _mesh_or_group(_EP_GROUP, _EP_MESH, as_list)


def get_expert_data_parallel_group(as_list: bool = False):
    assert _EDP_GROUP is not None or as_list, "expert data parallel group is not initialized"
    return _mesh_or_group(_EDP_GROUP, _EDP_MESH, as_list)


def _size(group) -> int:
    return dist.get_world_size(group=group) if group is not None else 1


def _rank(group) -> int:
    return dist.get_rank(group=group) if group is not None else 0


def set_tensor_model_parallel_size(world_size: Optional[int]) -> None:
    global _MPU_TP_SIZE
    _MPU_TP_SIZE = world_size


def set_tensor_model_parallel_rank(rank: Optional[int]) -> None:
    global _MPU_TP_RANK
    _MPU_TP_RANK = rank


def get_tensor_model_parallel_size() -> int:
    if _MPU_TP_SIZE is not None:
        return _MPU_TP_SIZE
    return _size(_TP_GROUP) if _INITIALIZED else 1


def get_tensor_model_parallel_rank() -> int:
    if _MPU_TP_RANK is not None:
        return _MPU_TP_RANK
    return _rank(_TP_GROUP) if _INITIALIZED else 0


def get_tensor_model_parallel_src_rank() -> int:
    """Global rank of TP-rank 0 of this rank's TP group."""
    g = dist.get_rank() if dist.is_initialized() else 0
    return (g // get_tensor_model_parallel_size()) * get_tensor_model_parallel_size()


def set_expert_model_parallel_size(world_size: Optional[int]) -> None:
    global _MPU_EP_SIZE
    _MPU_EP_SIZE = world_size


def set_expert_model_parallel_rank(rank: Optional[int]) -> None:
    global _MPU_EP_RANK
    _MPU_EP_RANK = rank


def get_expert_model_parallel_size() -> int:
    if _MPU_EP_SIZE is not None:
        return _MPU_EP_SIZE
    return _size(_EP_GROUP) if _INITIALIZED else 1


def get_expert_model_parallel_rank() -> int:
    if _MPU_EP_RANK is not None:
        return _MPU_EP_RANK
    return _rank(_EP_GROUP) if _INITIALIZED else 0


def set_data_parallel_size(world_size: Optional[int]) -> None:
    global _MPU_DP_SIZE
    _MPU_DP_SIZE = world_size


def set_data_parallel_rank(rank: Optional[int]) -> None:
    global _MPU_DP_RANK
    _MPU_DP_RANK = rank


def get_data_parallel_size() -> int:
    if _MPU_DP_SIZE is not None:
        return _MPU_DP_SIZE
    return _size(_DP_GROUP) if _INITIALIZED else 1


def get_data_parallel_rank() -> int:
    if _MPU_DP_RANK is not None:
        return _MPU_DP_RANK
    return _rank(_DP_GROUP) if _INITIALIZED else 0


def get_data_parallel_src_rank() -> int:
    assert _DP_MESH is not None
    g = dist.get_rank()
    for ranks in _DP_MESH:
        if g in ranks:
            return ranks[0]
    return 0


def get_expert_data_parallel_size() -> int:
    return _size(_EDP_GROUP) if _INITIALIZED else 1


def get_expert_data_parallel_rank() -> int:
    return _rank(_EDP_GROUP) if _INITIALIZED else 0


def set_pipeline_model_parallel_size(world_size: Optional[int]) -> None:
    global _MPU_PP_SIZE
    _MPU_PP_SIZE = world_size


def set_pipeline_model_parallel_rank(rank: Optional[int]) -> None:
    global _MPU_PP_RANK
    _MPU_PP_RANK = rank


def get_pipeline_model_parallel_size() -> int:
    if _MPU_PP_SIZE is not None:
        return _MPU_PP_SIZE
    return _size(_PP_GROUP) if _INITIALIZED else 1


def get_pipeline_model_parallel_rank() -> int:
    if _MPU_PP_RANK is not None:
        return _MPU_PP_RANK
    return _rank(_PP_GROUP) if _INITIALIZED else 0


def get_pipeline_model_parallel_next_rank() -> int:
    """Global rank of the next pipeline stage (wraps around)."""
    assert _PP_GLOBAL_RANKS is not None, "pipeline parallel group not initialised"
    r = get_pipeline_model_parallel_rank()
    return _PP_GLOBAL_RANKS[(r + 1) % len(_PP_GLOBAL_RANKS)]


def get_pipeline_model_parallel_prev_rank() -> int:
    assert _PP_GLOBAL_RANKS is not None, "pipeline parallel group not initialised"
    r = get_pipeline_model_parallel_rank()
    return _PP_GLOBAL_RANKS[(r - 1) % len(_PP_GLOBAL_RANKS)]


def get_pipeline_model_parallel_global_ranks() -> List[int]:
    assert _PP_GLOBAL_RANKS is not None
    return list(_PP_GLOBAL_RANKS)


def _pair_groups():
    """2-rank (stage, stage+1) groups, created collectively on first use (API compatibility)."""
    global _NEXT_GROUP, _PREV_GROUP
    if _NEXT_GROUP is not None or _PP_MESH is None:
        return
    rank = dist.get_rank()
    pp = len(_PP_MESH[0])
    for s in range(pp):
        for ranks in _PP_MESH:
            pair = sorted({ranks[s], ranks[(s + 1) % pp]})
            g = dist.new_group(pair)
            if rank == ranks[s]:
                _NEXT_GROUP = g
            if rank == ranks[(s + 1) % pp]:
                _PREV_GROUP = g


def get_next_rank_group(as_list: bool = False):
    _pair_groups()
    return _NEXT_GROUP


def get_prev_rank_group(as_list: bool = False):
    _pair_groups()
    return _PREV_GROUP


def get_pipeline_model_parallel_sr_group(parity: bool):
    """Reference API (parallel_state.py:580-591); with real p2p the PP group itself is used."""
    return get_pipeline_model_parallel_group()


def initialize_pp_gloo_groups() -> None:
    global _PP_GLOO_GROUP
    if _PP_GLOO_GROUP is not None:
        return
    assert _PP_MESH is not None
    rank = dist.get_rank()
    for ranks in _PP_MESH:
        g = dist.new_group(ranks, backend="gloo")
        if rank in ranks:
            _PP_GLOO_GROUP = g


def get_pp_gloo_group():
    assert _PP_GLOO_GROUP is not None, "call initialize_pp_gloo_groups() first"
    return _PP_GLOO_GROUP


def get_world_gloo_group():
    return _WORLD_GLOO_GROUP


def is_global_rank_zero() -> bool:
    return not dist.is_initialized() or dist.get_rank() == 0


def create_pg_with_ranks(ranks: List[int]):
    """Collectively create a group containing `ranks` (every rank must call with the same list)."""
    return dist.new_group(sorted(ranks))


def is_tcp_store_available() -> bool:
    return "MASTER_ADDR" in os.environ and "MASTER_PORT" in os.environ


def get_tcp_store():
    from torch.distributed import TCPStore

    host, port = os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]) + 1
    return TCPStore(host, port, dist.get_world_size(), dist.get_rank() == 0, use_libuv=False)


def gather_python_object(obj: Any, group=None) -> List[Any]:
    """All-gather an arbitrary picklable object over a (CPU-capable) group."""
    g = group if group is not None else _WORLD_GLOO_GROUP
    out = [None] * dist.get_world_size(group=g)
    dist.all_gather_object(out, obj, group=g)
    return out


def destroy_model_parallel() -> None:
    global _TP_GROUP, _TP_MESH, _DP_GROUP, _DP_MESH, _PP_GROUP, _PP_MESH, _EP_GROUP, _EP_MESH, _EDP_GROUP, _EDP_MESH
    global _PP_GLOO_GROUP, _PP_GLOBAL_RANKS, _NEXT_GROUP, _PREV_GROUP, _INITIALIZED, _WORLD_GLOO_GROUP
    global _MPU_TP_SIZE, _MPU_TP_RANK, _MPU_EP_SIZE, _MPU_EP_RANK, _MPU_PP_SIZE, _MPU_PP_RANK, _MPU_DP_SIZE, _MPU_DP_RANK
    _TP_GROUP = _DP_GROUP = _PP_GROUP = _EP_GROUP = _EDP_GROUP = _PP_GLOO_GROUP = None
    _TP_MESH = _DP_MESH = _PP_MESH = _EP_MESH = _EDP_MESH = None
    _PP_GLOBAL_RANKS = None
    _NEXT_GROUP = _PREV_GROUP = None
    _WORLD_GLOO_GROUP = None
    _MPU_TP_SIZE = _MPU_TP_RANK = _MPU_EP_SIZE = _MPU_EP_RANK = None
    _MPU_PP_SIZE = _MPU_PP_RANK = _MPU_DP_SIZE = _MPU_DP_RANK = None
    _INITIALIZED = False


def rmsg(msg: str) -> str:
    """Prefix a message with this rank's coordinates (reference parallel_state.py:740)."""
    try:
        g = dist.get_rank() if dist.is_initialized() else 0
        return (f"[rank_{g}_pp{get_pipeline_model_parallel_rank()}_tp{get_tensor_model_parallel_rank()}"
                f"_dp{get_data_parallel_rank()}] {msg}")
    except Exception:  # pragma: no cover
        return msg


def rmsg_ep(msg: str) -> str:
    try:
        g = dist.get_rank() if dist.is_initialized() else 0
        return (f"[rank_{g}_pp{get_pipeline_model_parallel_rank()}_tp{get_tensor_model_parallel_rank()}"
                f"_ep{get_expert_model_parallel_rank()}_edp{get_expert_data_parallel_rank()}] {msg}")
    except Exception:  # pragma: no cover
        return msg
