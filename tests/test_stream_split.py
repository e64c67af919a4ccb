"""Two-stream interleaving of half micro-batches under TP + SP (parallel_layers/stream_split.py):
same losses and gradient norms as the one-pass step, same collective order on every rank
(gloo ranks here: a mismatched order would deadlock or mix tensors)."""

import os
import tempfile

import torch

from dist_utils import run_distributed


def _w(rank, world, streams, out, preset="tiny8", stagger=0):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split

    stream_split.set_enabled(streams >= 2, streams)
    stream_split.set_stagger(stagger)
    ps.initialize_model_parallel(world)
    cfg = llama_config(preset, sequence_parallel_enabled=True, max_position_embeddings=128, num_hidden_layers=2)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.float32, device=torch.device("cpu"))
    model.train()
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=1e-3, grad_clipping=True, max_grad_norm=1.0,
                                  shared_param_ids=find_shared_params(model))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (4, 128))
    calls = []
    orig = LlamaForCausalLM._forward_interleaved

    def spy(self, *a, **k):
        calls.append(1)
        return orig(self, *a, **k)

    LlamaForCausalLM._forward_interleaved = spy
    losses, norms = [], []
    for _ in range(3):
        loss = model(ids, labels=ids).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
        norms.append(float(opt.grad_norm))
    LlamaForCausalLM._forward_interleaved = orig
    if rank == 0:
        torch.save({"loss": losses, "gn": norms, "interleaved": len(calls)}, out)


def _run(world, streams, preset="tiny8", stagger=0):
    d = tempfile.mkdtemp()
    run_distributed(_w, world, streams, os.path.join(d, "r.pt"), preset, stagger)
    return torch.load(os.path.join(d, "r.pt"))


def test_interleaved_halves_match_one_pass_tp2():
    a, b = _run(2, 1), _run(2, 2)
    assert a["interleaved"] == 0 and b["interleaved"] == 3
    for i in range(3):
        assert abs(a["loss"][i] - b["loss"][i]) < 1e-4 * abs(a["loss"][i]), (a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 1e-3 * a["gn"][i], (a, b)


def test_interleaved_halves_match_one_pass_tp4_replicated_kv():
    # tiny: 2 kv heads at TP=4 -> kv heads replicated on 2 ranks (KV-group all-reduce in backward)
    a, b = _run(4, 1, "tiny"), _run(4, 2, "tiny")
    assert b["interleaved"] == 3
    for i in range(3):
        assert abs(a["loss"][i] - b["loss"][i]) < 1e-4 * abs(a["loss"][i]), (a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 1e-3 * a["gn"][i], (a, b)


def test_four_parts_match_one_pass_tp2():
    # NXD_SP_STREAMS=4: the micro-batch of 4 as four parts on four streams
    a, b = _run(2, 1), _run(2, 4)
    assert b["interleaved"] == 3
    for i in range(3):
        assert abs(a["loss"][i] - b["loss"][i]) < 1e-4 * abs(a["loss"][i]), (a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 1e-3 * a["gn"][i], (a, b)


def test_staggered_halves_match_one_pass_tp2():
    # NXD_SP_STAGGER=2: the second half starts two collective steps (half a layer) behind
    a, b = _run(2, 1), _run(2, 2, stagger=2)
    assert b["interleaved"] == 3
    for i in range(3):
        assert abs(a["loss"][i] - b["loss"][i]) < 1e-4 * abs(a["loss"][i]), (a, b)
        assert abs(a["gn"][i] - b["gn"][i]) < 1e-3 * a["gn"][i], (a, b)
