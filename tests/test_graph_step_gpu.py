"""Whole training step (fwd + bwd + clipped AdamW) captured in one hipGraph == the eager step."""

import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup():
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29651")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    if not ps.model_parallel_is_initialized():
        ps.initialize_model_parallel(1)


def _model():
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW

    torch.manual_seed(0)
    cfg = llama_config("tiny", num_hidden_layers=2, hidden_size=512, intermediate_size=1024, num_attention_heads=8,
                       num_key_value_heads=2, vocab_size=4096)
    m = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda", 0))
    opt = FlatMixedPrecisionAdamW(m.parameters(), lr=1e-3, grad_clipping=True, max_grad_norm=1.0)
    return cfg, m, opt


def _loss(model, ids):
    return model(ids, labels=ids).loss / 2


def test_graphed_train_step_matches_eager():
    from neuronx_distributed_llama3_2_amd.utils.graph_step import GraphedTrainStep

    _setup()
    cfg, me, oe = _model()
    _, mg, og = _model()
    g = torch.Generator(device="cpu").manual_seed(1)
    two = [[torch.randint(0, cfg.vocab_size, (2, 256), generator=g).cuda() for _ in range(2)] for _ in range(2)]
    batches = [two[i % 2] for i in range(6)]   # learnable: the loss must fall
    step = GraphedTrainStep(mg, og, _loss, [(b,) for b in batches[0]])
    for p_e, p_g in zip(me.parameters(), mg.parameters()):   # warm-up left the state untouched
        assert torch.equal(p_e, p_g)
    le, lg = [], []
    for bs in batches:
        tot = 0.0
        for b in bs:
            loss = _loss(me, b)
            loss.backward()
            tot += float(loss)
        oe.step()
        oe.zero_grad()
        le.append(tot)
        lg.append(float(step(*[(b,) for b in bs])))
    assert le[-1] < le[0]
    for a, b in zip(le, lg):
        assert abs(a - b) < 2e-2 * abs(a), (le, lg)
    # replay speed (launch-bound tiny model): report, do not assert
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step(*[(b,) for b in batches[0]])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(10):
        for b in batches[0]:
            _loss(me, b).backward()
        oe.step()
        oe.zero_grad()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graphed step {1e3 * (t1 - t0) / 10:.2f} ms vs eager {1e3 * (t2 - t1) / 10:.2f} ms")
