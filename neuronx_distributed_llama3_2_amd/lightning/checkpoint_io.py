"""Checkpoint IO through the NxD sharded format (reference: lightning/checkpoint_io.py): every rank
writes / reads its own `{dp,tp,pp}` shard of the Lightning checkpoint dict; optional xser
(tensor-per-file) serialisation."""

import os
from typing import Any, Dict, Optional

import torch

from ..parallel_layers import parallel_state as ps
from ._compat import CheckpointIO, require_lightning

require_lightning()


def _shard_name() -> str:
    return (f"dp_rank_{ps.get_data_parallel_rank():02d}_tp_rank_{ps.get_tensor_model_parallel_rank():02d}"
            f"_pp_rank_{ps.get_pipeline_model_parallel_rank():02d}.pt")


class NeuronCheckpointIO(CheckpointIO):
    def __init__(self, save_load_xser: bool = True, weights_only: bool = True, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.save_load_xser = save_load_xser
        self.weights_only = weights_only

    def save_checkpoint(self, checkpoint: Dict[str, Any], path, storage_options: Optional[Any] = None) -> None:
        from ..parallel_layers.utils import move_all_tensor_to_cpu
        from ..utils.serialization import xser_save

        os.makedirs(path, exist_ok=True)
        f = os.path.join(path, _shard_name())
        cpu = move_all_tensor_to_cpu(checkpoint)
        if self.save_load_xser:
            xser_save(cpu, f)
        else:
            torch.save(cpu, f)

    def load_checkpoint(self, path, map_location: Optional[Any] = None) -> Dict[str, Any]:
        from ..utils.serialization import xser_load

        f = os.path.join(path, _shard_name())
        if self.save_load_xser and os.path.exists(f + ".tensors"):
            return xser_load(f)
        return torch.load(f, map_location=map_location or "cpu", weights_only=self.weights_only)

    def remove_checkpoint(self, path) -> None:
        import shutil

        shutil.rmtree(path, ignore_errors=True)
