"""Native RCCL layer (csrc/comm.cpp) on the one-GPU box: communicator from a torch-broadcast unique
id, coalesced group launches, bucketed all-reduce through the staging buffer, stream ordering.
(Multi-rank RCCL needs one GPU per rank: exercised by the driver's multi-GPU node only.)"""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _comm():
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel.native_comm import NativeCommunicator

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29661")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    return NativeCommunicator()


def test_native_comm_single_rank_semantics():
    c = _comm()
    try:
        ts = [torch.randn(n, device="cuda") for n in (1, 7, 1000, 4096 + 3)]
        ref = [t.clone() for t in ts]
        c.all_reduce(ts)
        for a, b in zip(ts, ref):
            assert torch.equal(a, b)
        # bucketed: 300 tensors of mixed sizes, one collective; values unchanged on one rank, and the
        # pack / unpack must not bleed between neighbours (16-B slot alignment)
        many = [torch.full((i % 37 + 1,), float(i), device="cuda", dtype=torch.bfloat16) for i in range(300)]
        w = c.bucketed_all_reduce(many, async_op=True)
        w.wait()
        for i, t in enumerate(many):
            assert torch.all(t == float(i)), i
        x = torch.randn(256, device="cuda")
        out = torch.empty(256, device="cuda")
        c.all_gather([out], [x])
        assert torch.equal(out, x)
        y = torch.empty(256, device="cuda")
        c.reduce_scatter([y], [x], op="max")
        assert torch.equal(y, x)
        z = torch.empty(256, device="cuda")
        c.all_to_all(z, x)
        assert torch.equal(z, x)
        r = torch.empty(256, device="cuda")
        c.batch_p2p([x], [0], [r], [0])
        assert torch.equal(r, x)
        # ordering: a producer on the default stream, the collective on the comm stream
        big = torch.zeros(1 << 22, device="cuda")
        big.add_(3.0)
        c.all_reduce([big], op="sum")
        assert float(big[-1]) == 3.0
    finally:
        c.close()


def test_comm_layer_routes_gpu_tensors_to_native_rccl():
    """NXD_NATIVE_COMM on: the framework's comm primitives (used by the DP grad buckets and the SP
    norm-gradient all-reduce) run on the native communicator for RCCL-group GPU tensors."""
    _comm()
    from neuronx_distributed_llama3_2_amd.parallel import comm

    comm.set_native_comm(True)
    try:
        x = torch.randn(1024, device="cuda")
        ref = x.clone()
        w = comm.all_reduce(x, async_op=True)
        w.wait()
        assert torch.equal(x, ref)
        out = torch.empty(1024, device="cuda")
        comm.reduce_scatter_tensor(out, x, async_op=True).wait()
        assert torch.equal(out, ref)
        g = torch.empty(1024, device="cuda")
        comm.all_gather_into_tensor(g, out)
        torch.cuda.synchronize()
        assert torch.equal(g, ref)
        assert len(comm._native_comms) == 1      # one communicator for the world group
    finally:
        comm.set_native_comm(False)
