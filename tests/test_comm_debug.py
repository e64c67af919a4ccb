"""Stream-ordering debug mode of the collective layer (parallel/comm.py): leaked async
handles are reported with their op and call site; a full TP2 x DP2 ZeRO-1 training run (SP
pipelined all-gather / reduce-scatter, bucketed backward-overlapped DP reduce-scatter, parameter
all-gather) completes with the checker armed, i.e. every launched collective is waited on."""

import os
import tempfile

import torch

from tests.dist_utils import run_distributed


def _leak(rank, world):
    from neuronx_distributed_llama3_2_amd.parallel import comm

    comm.set_comm_debug(True)
    t = torch.ones(8)
    h = comm.all_reduce(t, async_op=True)
    out = torch.empty(16)
    h2 = comm.all_gather_into_tensor(out, torch.full((8,), float(rank)), async_op=True)
    try:
        comm.assert_no_pending_collectives("probe")
        raise RuntimeError("leak not detected")
    except AssertionError as e:
        msg = str(e)
        assert "2 async collective(s)" in msg and "all_reduce(8,)" in msg and "all_gather(16,)" in msg, msg
    h.wait()
    h2.wait()
    comm.assert_no_pending_collectives("after wait")
    assert torch.all(t == world) and torch.equal(out, torch.arange(2.0).repeat_interleave(8))
    comm.set_comm_debug(False)


def test_leaked_handle_detected():
    run_distributed(_leak, 2)


def test_zero1_training_clean_under_debug(monkeypatch):
    from tests.test_trainer import _train

    monkeypatch.setenv("NXD_COMM_DEBUG", "1")
    d = tempfile.mkdtemp()
    run_distributed(_train, 4, 2, True, 2, os.path.join(d, "a.pt"))
    losses = torch.load(os.path.join(d, "a.pt"))
    assert len(losses) == 2 and all(l == l for l in losses)
