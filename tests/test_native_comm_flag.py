"""NXD_NATIVE_COMM: the comm layer's native-RCCL switch.  On CPU / gloo the switch must leave every
collective on the torch path (the same calls the flag-on GPU path makes), so the framework code
that routes through it -- DP bucket reduce-scatter / all-gather, the coalesced SP norm-gradient
all-reduce -- is exercised here with the flag on; on one GPU the native path itself runs
(tests/test_native_comm_gpu.py)."""

import os
import tempfile

import torch
import torch.distributed as dist

from dist_utils import run_distributed


def _w_prims(rank, world):
    from neuronx_distributed_llama3_2_amd.parallel import comm

    comm.set_native_comm(True)
    ts = [torch.full((n,), float(rank + 1)) for n in (3, 1, 17)]
    comm.all_reduce_coalesced(ts)
    for t in ts:
        assert torch.all(t == sum(range(1, world + 1)))
    x = torch.arange(4 * world, dtype=torch.float32) + rank
    out = torch.empty(4)
    comm.reduce_scatter_tensor(out, x)
    assert torch.equal(out, sum(torch.arange(4 * world, dtype=torch.float32) + r for r in range(world))[4 * rank:4 * rank + 4])
    g = torch.empty(4 * world)
    comm.all_gather_into_tensor(g, out)
    assert g.shape[0] == 4 * world


def test_native_flag_falls_back_on_gloo():
    run_distributed(_w_prims, 2)


def _w_train(rank, world, native, out):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel import comm
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    comm.set_native_comm(native)
    ps.initialize_model_parallel(2)          # TP=2 (+SP) x DP=2 ZeRO-1 on 4 ranks
    cfg = llama_config("tiny", sequence_parallel_enabled=True)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.float32, device=torch.device("cpu"))
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=2e-3, zero1=True, grad_clipping=True,
                                  shared_param_ids=find_shared_params(model))
    ids = torch.randint(0, cfg.vocab_size, (4, 64), generator=torch.Generator().manual_seed(5))
    local = ids.chunk(ps.get_data_parallel_size())[ps.get_data_parallel_rank()]
    losses = []
    for _ in range(3):
        loss = model(local, labels=local).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
        lo = loss.detach().clone()
        dist.all_reduce(lo)
        losses.append(float(lo))
    if rank == 0:
        torch.save(losses, out)


def test_training_with_native_flag_matches_default():
    d = tempfile.mkdtemp()
    run_distributed(_w_train, 4, False, os.path.join(d, "a.pt"))
    run_distributed(_w_train, 4, True, os.path.join(d, "b.pt"))
    assert torch.load(os.path.join(d, "a.pt")) == torch.load(os.path.join(d, "b.pt"))
