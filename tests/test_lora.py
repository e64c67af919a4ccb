"""LoRA: plain-layer adapters, merge/unmerge, adapter save/load, TP=2 (+SP) parity with TP=1
(reference tests: test/unit_test/modules/lora/test_lora_layer.py, test_lora_model.py)."""

import os
import tempfile

import pytest
import torch
from torch import nn

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps


def test_plain_layers_merge_roundtrip():
    from neuronx_distributed_llama3_2_amd.modules.lora import LoraConfig, LoraConv2d, LoraEmbedding, LoraLinear

    torch.manual_seed(0)
    cfg = LoraConfig(enable_lora=True, lora_rank=4, lora_alpha=8, target_modules=["x"])
    cases = [(LoraLinear(nn.Linear(16, 8), cfg), torch.randn(3, 16)),
             (LoraEmbedding(nn.Embedding(20, 8), cfg), torch.randint(0, 20, (3, 5))),
             (LoraConv2d(nn.Conv2d(4, 6, 3, padding=1), cfg), torch.randn(2, 4, 7, 7))]
    for layer, x in cases:
        base = layer.base_layer(x)
        torch.testing.assert_close(layer(x), base)  # B (or A for embeddings) starts at zero
        for n, p in layer.named_parameters():
            if "lora_" in n:
                p.data.normal_(0, 0.1)
        y = layer(x)
        assert not torch.allclose(y, base)
        layer.merge()
        torch.testing.assert_close(layer(x), y, atol=1e-5, rtol=1e-5)
        layer.unmerge()
        torch.testing.assert_close(layer.base_layer(x), base, atol=1e-5, rtol=1e-5)


def _tiny(tp_sp=False):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config

    cfg = llama_config("tiny", sequence_parallel_enabled=tp_sp)
    torch.manual_seed(0)
    return cfg, LlamaForCausalLM(cfg, dtype=torch.float32)


def _lora_cfg(**kw):
    from neuronx_distributed_llama3_2_amd.modules.lora import LoraConfig

    d = dict(enable_lora=True, lora_rank=4, lora_alpha=16,
             target_modules=["qkv_proj", "o_proj", "gate_up_proj", "down_proj"])
    d.update(kw)
    return LoraConfig(**d)


def _full_adapters(model, seed=3):
    """Deterministic FULL adapter tensors keyed by name (TP-degree independent)."""
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import _attrs

    g = torch.Generator().manual_seed(seed)
    tp = ps.get_tensor_model_parallel_size()
    out = {}
    for n, p in model.named_parameters():
        if "lora_" not in n:
            continue
        a = _attrs(p)
        shape = list(p.shape)
        if a["tp"]:
            if a["qkv"] is not None:
                q, kv, mult = a["qkv"]
                shape[0] = q + 2 * kv
            else:
                shape[a["dim"]] *= tp
        out[n] = torch.randn(shape, generator=g) * 0.1
    return out


def _load_adapters(model, full):
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import _attrs, shard_tensor

    tp, r = ps.get_tensor_model_parallel_size(), ps.get_tensor_model_parallel_rank()
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n in full:
                p.copy_(shard_tensor(full[n], _attrs(p), tp, r))


def _w_lora_tp(rank, world, sp, out):
    from neuronx_distributed_llama3_2_amd.modules.lora import LoraModel

    ps.initialize_model_parallel(world)
    cfg, base = _tiny(sp)
    model = LoraModel(base, _lora_cfg())
    assert all(("lora_" in n) == p.requires_grad for n, p in model.named_parameters())
    _load_adapters(model.module, _full_adapters(model.module))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 32))
    loss = model(ids, labels=ids).loss
    loss.backward()
    # adapter grad norm (TP-aware: replicated factors counted once, SP partials summed)
    sq = torch.zeros(())
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad
        if not getattr(p, "tensor_model_parallel", False):
            if getattr(p, "sequence_parallel_enabled", False) and world > 1:
                g = g.clone()
                torch.distributed.all_reduce(g)
            g = g / world ** 0.5
        sq += (g.float() ** 2).sum()
    torch.distributed.all_reduce(sq)
    with torch.no_grad():
        before = model(ids, labels=ids).loss
        model.merge_lora()
        merged = model(ids, labels=ids).loss
        model.unmerge_lora()
    sd = model.state_dict()
    assert "lora_config" in sd and all("lora_" in k for k in sd if k != "lora_config")
    if rank == 0:
        torch.save({"loss": float(loss), "gn": float(sq.sqrt()), "before": float(before), "merged": float(merged)}, out)


@pytest.mark.parametrize("sp", [False, True])
def test_lora_tp2_matches_tp1(sp):
    d = tempfile.mkdtemp()
    run_distributed(_w_lora_tp, 1, False, os.path.join(d, "a.pt"))
    run_distributed(_w_lora_tp, 2, sp, os.path.join(d, "b.pt"))
    a, b = torch.load(os.path.join(d, "a.pt")), torch.load(os.path.join(d, "b.pt"))
    assert abs(a["loss"] - b["loss"]) < 1e-4, (a, b)
    assert abs(a["gn"] - b["gn"]) < 1e-3 * a["gn"], (a, b)
    for r in (a, b):
        assert abs(r["before"] - r["merged"]) < 1e-4, r


def test_lora_save_load_single_device():
    from neuronx_distributed_llama3_2_amd.modules.lora import LoraModel
    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29641")
        dist.init_process_group("gloo", rank=0, world_size=1)
    if not ps.model_parallel_is_initialized():
        ps.initialize_model_parallel(1)
    cfg, base = _tiny()
    m = LoraModel(base, _lora_cfg())
    _load_adapters(m.module, _full_adapters(m.module, seed=9))
    d = tempfile.mkdtemp()
    m.save_lora(d, "tag1")
    ids = torch.randint(0, cfg.vocab_size, (1, 16))
    with torch.no_grad():
        ref = m(ids, labels=ids).loss
    _, base2 = _tiny()
    m2 = LoraModel(base2, _lora_cfg(load_lora_from_ckpt=True, lora_save_dir=d, lora_load_tag="tag1"))
    m2.load_state_dict(None)
    with torch.no_grad():
        got = m2(ids, labels=ids).loss
    torch.testing.assert_close(got, ref)
