"""Lightning strategy for NxD parallelism on MI355X (reference: lightning/strategy.py
NeuronXLAStrategy): one process per GPU, RCCL process group, NxD TP/PP/EP mesh, DP-rank data
sharding, no DDP wrapper (the framework's flat-buffer optimizer reduces DP gradients overlapped
with backward), sharded checkpoints via NeuronCheckpointIO, reductions over the DP group."""

from typing import Any, Dict, Optional

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state as ps
from ._compat import DDPStrategy, require_lightning
from .checkpoint_io import NeuronCheckpointIO

require_lightning()


class NeuronXLAStrategy(DDPStrategy):
    def __init__(self, nxd_config: Optional[Dict[str, Any]] = None, tensor_parallel_size: int = 1,
                 pipeline_parallel_size: int = 1, expert_parallel_size: int = 1, debug: bool = False,
                 sync_module_states: bool = False, checkpoint_io: Optional[NeuronCheckpointIO] = None,
                 save_load_xser: bool = True, process_group_backend: str = "nccl", **kwargs):
        super().__init__(process_group_backend=process_group_backend, checkpoint_io=checkpoint_io or
                         NeuronCheckpointIO(save_load_xser=save_load_xser), **kwargs)
        self.nxd_config = nxd_config
        if nxd_config is not None:
            tensor_parallel_size = nxd_config["tensor_parallel_size"]
            pipeline_parallel_size = nxd_config["pipeline_parallel_size"]
            expert_parallel_size = nxd_config.get("expert_parallel_size", 1)
        self.tensor_parallel_size = tensor_parallel_size
        self.pipeline_parallel_size = pipeline_parallel_size
        self.expert_parallel_size = expert_parallel_size
        self.debug = debug

    def _configure_launcher(self) -> None:
        from .launcher import _NeuronXLALauncher

        self._launcher = _NeuronXLALauncher(self)

    def setup_distributed(self) -> None:
        super().setup_distributed()
        if not ps.model_parallel_is_initialized():
            ps.initialize_model_parallel(self.tensor_parallel_size, self.pipeline_parallel_size,
                                         self.expert_parallel_size)

    @property
    def distributed_sampler_kwargs(self) -> Dict[str, int]:
        return {"num_replicas": ps.get_data_parallel_size(), "rank": ps.get_data_parallel_rank()}

    def configure_ddp(self) -> None:   # no DDP wrapper: DP reduction lives in the NxD optimizer
        pass

    def _setup_model(self, model):
        return model

    def reduce(self, tensor, group: Optional[Any] = None, reduce_op: Optional[str] = "mean"):
        if not isinstance(tensor, torch.Tensor) or not dist.is_initialized():
            return tensor
        g = group if group is not None else ps.get_data_parallel_group()
        dist.all_reduce(tensor, group=g)
        if reduce_op in ("mean", "avg") or reduce_op is None:
            tensor = tensor / dist.get_world_size(group=g)
        return tensor

    def broadcast(self, obj, src: int = 0):
        out = [obj]
        dist.broadcast_object_list(out, src=src)
        return out[0]

    @property
    def is_global_zero(self) -> bool:
        return dist.get_rank() == 0 if dist.is_initialized() else True

    def save_checkpoint(self, checkpoint: Dict[str, Any], filepath, storage_options: Optional[Any] = None) -> None:
        # every rank writes its own shard (TP/PP/DP-sharded model + ZeRO-1 optimizer state)
        self.checkpoint_io.save_checkpoint(checkpoint, filepath, storage_options=storage_options)
        self.barrier("save_checkpoint")

    def load_checkpoint(self, checkpoint_path) -> Dict[str, Any]:
        return self.checkpoint_io.load_checkpoint(checkpoint_path)

    def remove_checkpoint(self, filepath) -> None:
        if self.is_global_zero:
            self.checkpoint_io.remove_checkpoint(filepath)


NxDStrategy = NeuronXLAStrategy
