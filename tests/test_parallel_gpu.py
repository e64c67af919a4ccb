"""Tensor + sequence parallel TRAINING with the GPU kernels, checked against TP=1 on the same GPU.

N ranks share the single MI355X of the test box (gloo collectives on staged GPU tensors; the RCCL
path is the same code with the nccl backend).  Each run trains 4 fused-AdamW steps on one fixed
batch (the loss falls fast, so a wrongly sharded gradient shows as a diverging loss curve) and
records the per-step loss and global gradient norm.  Cases mirror the headline layout
(reference test/integration/parallel_layers/test_layers.py:44-101 sweeps TP against a
single-device reference, :746-777):
  * `tiny8` (16 q / 8 kv heads of 64): TP=8 keeps ONE kv head per rank as Llama-3-8B at TP=8,
    TP=4 two; sequence parallel with the chunk-pipelined all-gather / reduce-scatter;
  * `tiny` (4 q / 2 kv heads): TP=2 +- SP, and TP=4 with the kv heads replicated on 2 ranks
    (kv_size_multiplier 2: q head groups reshuffled as the reference converter does, replicated
    K/V rows counted once in the clip norm -- exactly the unsharded model).
"""

import os
import tempfile

import pytest
import torch

from dist_utils import run_distributed

pytestmark = pytest.mark.gpu

STEPS = 4


def _w_train(rank, world, preset, sp, out, streams=1):
    torch.cuda.set_device(0)
    from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split

    # streams=2: the two-stream SP half micro-batch interleaving (NXD_SP_STREAMS=2, opt-in)
    stream_split.set_enabled(streams >= 2, streams)
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.initialize_model_parallel(world)
    cfg = llama_config(preset, sequence_parallel_enabled=sp, max_position_embeddings=512)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda"))
    model.train()
    decay = [p for p in model.parameters() if p.dim() > 1]
    no_decay = [p for p in model.parameters() if p.dim() <= 1]
    opt = FlatMixedPrecisionAdamW([{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}],
                                  lr=1e-3, betas=(0.9, 0.95), eps=1e-8, grad_clipping=True, max_grad_norm=1.0,
                                  shared_param_ids=find_shared_params(model))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 512), device="cuda")
    losses, norms = [], []
    for _ in range(STEPS):
        loss = model(ids, labels=ids).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
        norms.append(float(opt.grad_norm))
    if rank == 0:
        torch.save({"loss": losses, "gn": norms}, out)


def _train(world, preset, sp, streams=1):
    d = tempfile.mkdtemp()
    run_distributed(_w_train, world, preset, sp, os.path.join(d, "r.pt"), streams)
    return torch.load(os.path.join(d, "r.pt"))


_BASE = {}


def _baseline(preset):
    if preset not in _BASE:
        _BASE[preset] = _train(1, preset, False)
    return _BASE[preset]


@pytest.mark.parametrize("preset,tp,sp", [("tiny", 2, False), ("tiny", 2, True), ("tiny", 4, True), ("tiny8", 2, True),
                                          ("tiny8", 4, True), ("tiny8", 8, True), ("tiny8", 8, False)])
def test_tp_training_on_one_gpu_matches_tp1(preset, tp, sp):
    a, b = _baseline(preset), _train(tp, preset, sp)
    assert a["loss"][-1] < a["loss"][0] - 0.3, a          # the fixed batch is being learned
    for i in range(STEPS):
        assert abs(a["loss"][i] - b["loss"][i]) < 1.5e-2 * abs(a["loss"][i]), (i, a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 5e-2 * a["gn"][i], (i, a, b)


def test_tp8_sp_two_stream_halves_match_tp1():
    # the opt-in two-stream SP halves (NXD_SP_STREAMS=2) at the headline head layout
    a, b = _baseline("tiny8"), _train(8, "tiny8", True, streams=2)
    for i in range(STEPS):
        assert abs(a["loss"][i] - b["loss"][i]) < 1.5e-2 * abs(a["loss"][i]), (i, a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 5e-2 * a["gn"][i], (i, a, b)
