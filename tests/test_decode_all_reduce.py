"""The TP decode all-reduce's process-group fallback (parallel/peer_allreduce.py ProcessGroupAllReduce)
on 2 gloo ranks: the same three operations and rounding as the one-shot peer kernel (GPU test:
tests/test_peer_allreduce_gpu.py)."""
import torch
import torch.distributed as dist

from neuronx_distributed_llama3_2_amd.parallel.peer_allreduce import ProcessGroupAllReduce, make_decode_all_reduce

from dist_utils import run_distributed


def _worker(rank, world):
    ar = make_decode_all_reduce(None, 4096, torch.device("cpu"))
    assert isinstance(ar, ProcessGroupAllReduce)
    parts = [torch.randn(64, generator=torch.Generator().manual_seed(10 + r)) for r in range(world)]
    want = parts[0] + parts[1]
    inp, out = parts[rank].clone(), torch.empty(64)
    ar.sum_(inp, out, zero_in=True)
    assert torch.equal(out, want) and not inp.any()
    res0 = torch.randn(64, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    xadd = torch.randn(64, generator=torch.Generator().manual_seed(4))
    res = res0.clone()
    ar.fold_residual_(parts[rank].clone(), res, xadd)
    y = (res0.float() + xadd.to(torch.bfloat16).float()).to(torch.bfloat16)
    assert torch.equal(res, (y.float() + want.to(torch.bfloat16).float()).to(torch.bfloat16))
    res = res0.clone()
    ar.set_residual_(parts[rank].clone(), res)
    assert torch.equal(res, want.to(torch.bfloat16))


def test_process_group_decode_all_reduce():
    run_distributed(_worker, 2)
