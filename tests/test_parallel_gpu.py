"""Tensor + sequence parallel training step with the GPU kernels: two ranks share the single MI355X
of the test box (gloo collectives on staged GPU tensors; the RCCL path is the same code with the
nccl backend).  Checks TP=2 (+SP, chunk-pipelined collectives) against TP=1 on the same GPU."""

import os
import tempfile

import pytest
import torch

from dist_utils import run_distributed

pytestmark = pytest.mark.gpu


def _w_step(rank, world, sp, out):
    torch.cuda.set_device(0)
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.initialize_model_parallel(world)
    cfg = llama_config("tiny", hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                       vocab_size=1024, sequence_parallel_enabled=sp)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda"))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device="cuda")
    loss = model(ids, labels=ids).loss
    loss.backward()
    sq = torch.zeros((), device="cuda", dtype=torch.float32)
    for p in model.parameters():
        g = p.grad.float()
        if not getattr(p, "tensor_model_parallel", False):
            if sp:  # partial sums over TP
                g = g.clone()
                torch.distributed.all_reduce(g)
            g = g / world ** 0.5  # counted once across the TP ranks after the all-reduce below
        sq += (g * g).sum()
    torch.distributed.all_reduce(sq)
    if rank == 0:
        torch.save({"loss": float(loss), "gn": float(sq.sqrt())}, out)


@pytest.mark.parametrize("sp", [False, True])
def test_tp2_on_one_gpu_matches_tp1(sp):
    d = tempfile.mkdtemp()
    run_distributed(_w_step, 1, False, os.path.join(d, "a.pt"))
    run_distributed(_w_step, 2, sp, os.path.join(d, "b.pt"))
    a, b = torch.load(os.path.join(d, "a.pt")), torch.load(os.path.join(d, "b.pt"))
    assert abs(a["loss"] - b["loss"]) < 2e-2 * abs(a["loss"]), (a, b)
    assert abs(a["gn"] - b["gn"]) < 5e-2 * a["gn"], (a, b)
