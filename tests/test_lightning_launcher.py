"""Lightning launcher core (reference lightning/launcher.py `_NeuronXLALauncher`): spawns the rank
processes itself, or runs in place under torchrun; rank 0's result comes back; failures surface."""

import os

import pytest
import torch

from neuronx_distributed_llama3_2_amd.lightning import NeuronLauncher


def _job(scale):
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    dist.init_process_group("gloo")
    ps.initialize_model_parallel(tensor_model_parallel_size=2)
    t = torch.tensor([float(dist.get_rank() + 1)])
    dist.all_reduce(t)
    out = (int(os.environ["LOCAL_RANK"]), int(os.environ["WORLD_SIZE"]), float(t) * scale,
           ps.get_tensor_model_parallel_size())
    ps.destroy_model_parallel()
    dist.destroy_process_group()
    return out


def _fail():
    if int(os.environ["RANK"]) == 1:
        raise ValueError("boom on rank 1")
    return 0


def test_launcher_spawns_ranks_and_returns_rank0(monkeypatch):
    for k in ("LOCAL_RANK", "WORLD_SIZE", "RANK"):
        monkeypatch.delenv(k, raising=False)
    res = NeuronLauncher(2).launch(_job, 10.0)
    assert res == (0, 2, 30.0, 2)


def test_launcher_reports_rank_failure(monkeypatch):
    for k in ("LOCAL_RANK", "WORLD_SIZE", "RANK"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(RuntimeError, match="boom on rank 1"):
        NeuronLauncher(2).launch(_fail)


def test_launcher_runs_in_place_under_torchrun(monkeypatch):
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    launcher = NeuronLauncher(4)
    assert launcher.creates_processes_externally
    assert launcher.launch(lambda x: x + 1, 41) == 42
