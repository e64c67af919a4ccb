"""MoE inference (Mixtral, DBRX) on CPU: HF parity of prefill logits and greedy generation,
the three expert dispatch paths agree, legacy / fused HF checkpoint layouts convert identically,
TP=2 == TP=1, compile/load round trip (reference: examples/inference/{mixtral,dbrx}; accuracy
check against HF CPU outputs as in examples/inference/runner.py `check_accuracy`)."""

import os
import tempfile

import torch

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps


def _mixtral_cfg(**kw):
    from transformers import MixtralConfig

    d = dict(hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
             vocab_size=256, max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=1e6, num_local_experts=4,
             num_experts_per_tok=2, tie_word_embeddings=False, bos_token_id=1, eos_token_id=2)
    d.update(kw)
    return MixtralConfig(**d)


def _dbrx_hf(seed=0):
    from transformers import DbrxConfig, DbrxForCausalLM

    c = DbrxConfig(d_model=64, n_heads=4, n_layers=2, max_seq_len=256, vocab_size=256,
                   attn_config=dict(kv_n_heads=2, clip_qkv=0.5, rope_theta=10000.0),
                   ffn_config=dict(ffn_hidden_size=96, moe_num_experts=4, moe_top_k=2))
    torch.manual_seed(seed)
    m = DbrxForCausalLM(c).eval()
    with torch.no_grad():   # HF init leaves the expert weights ~0; make the experts matter
        for n, p in m.named_parameters():
            if "experts" in n or "norm" in n:
                p.normal_(0.0, 0.2) if "experts" in n else p.uniform_(0.5, 1.5)
    return c, m


def _mixtral_hf(cfg, seed=0):
    from transformers import MixtralForCausalLM

    torch.manual_seed(seed)
    m = MixtralForCausalLM(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "experts" in n:
                p.normal_(0.0, 0.1)
    return m


def _app(cls, cfg, full_sd, tp=1, batch=2, max_len=64, **kw):
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig

    icfg = InferenceConfig(tp_degree=tp, batch_size=batch, seq_len=max_len, max_context_length=32, **kw)
    m = cls(cfg, icfg, dtype=torch.float32, init_weights=False)
    m._load_full(full_sd)
    return m


def test_mixtral_hf_parity_and_greedy():
    from neuronx_distributed_llama3_2_amd.inference import MixtralForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.mixtral.convert import mixtral_hf_to_nxd

    cfg = _mixtral_cfg()
    hf = _mixtral_hf(cfg)
    m = _app(MixtralForCausalLMInference, cfg, mixtral_hf_to_nxd(hf.state_dict(), cfg))
    torch.manual_seed(3)
    ids = torch.randint(3, cfg.vocab_size, (2, 12))
    mask = torch.ones_like(ids)
    mask[1, 9:] = 0
    with torch.no_grad():
        ref = hf(ids).logits
    logits = m._context_encode(ids, mask)
    torch.testing.assert_close(logits[0], ref[0, 11], atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(logits[1], ref[1, 8], atol=2e-4, rtol=2e-4)
    out = m.generate(ids[:1], max_new_tokens=10, eos_token_id=-1)
    with torch.no_grad():
        hf_out = hf.generate(ids[:1], max_new_tokens=10, do_sample=False, eos_token_id=None, pad_token_id=0)
    assert torch.equal(out, hf_out), (out, hf_out)


def test_dbrx_hf_parity_and_greedy():
    from neuronx_distributed_llama3_2_amd.inference import DbrxForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.mixtral.convert import dbrx_hf_to_nxd, dbrx_to_mixtral_config

    c, hf = _dbrx_hf()
    cfg = dbrx_to_mixtral_config(c)
    assert cfg.norm_type == "layernorm" and cfg.clip_qkv == 0.5
    m = _app(DbrxForCausalLMInference, cfg, dbrx_hf_to_nxd(hf.state_dict(), cfg))
    ids = torch.randint(3, 256, (1, 11))
    with torch.no_grad():
        ref = hf(ids).logits
    torch.testing.assert_close(m._context_encode(ids)[0], ref[0, -1], atol=3e-4, rtol=3e-4)
    out = m.generate(ids, max_new_tokens=8, eos_token_id=-1)
    with torch.no_grad():
        hf_out = hf.generate(ids, max_new_tokens=8, do_sample=False, eos_token_id=None, pad_token_id=0)
    assert torch.equal(out, hf_out), (out, hf_out)


def test_moe_dispatch_paths_agree_and_legacy_layout():
    """selective loading (T*k <= E), dense all-experts and sorted grouped GEMMs give the same
    block output; hub (per-expert w1/w2/w3) and transformers-5 fused layouts convert identically."""
    from neuronx_distributed_llama3_2_amd.inference import MixtralForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.mixtral.convert import mixtral_hf_to_nxd, mixtral_nxd_to_hf

    cfg = _mixtral_cfg(num_local_experts=8)
    hf = _mixtral_hf(cfg, seed=1)
    full = mixtral_hf_to_nxd(hf.state_dict(), cfg)
    legacy = mixtral_nxd_to_hf(full, cfg)
    assert "model.layers.0.block_sparse_moe.experts.3.w2.weight" in legacy
    again = mixtral_hf_to_nxd(legacy, cfg)
    assert set(again) == set(full) and all(torch.equal(again[k], full[k]) for k in full)
    m = _app(MixtralForCausalLMInference, cfg, full).model
    layer = m.model.layers[0]
    w_gu, w_d = m._expert_weights(layer)
    assert w_gu.shape == (8, 64, 192) and w_gu.stride(1) == 1   # output-major storage, logical shape kept
    x = torch.randn(3, 64)
    top_w, top_i = m._route(layer, x)
    a = m._selective(x, top_w, top_i, w_gu, w_d)
    b = m._all_experts(x, top_w, top_i, w_gu, w_d)
    c = m._grouped(x, top_w, top_i, w_gu, w_d)
    torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(b, c, atol=1e-5, rtol=1e-5)


def _w_moe_tp(rank, world, out_path, ckpt_dir):
    from neuronx_distributed_llama3_2_amd.inference import MixtralForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.mixtral.convert import mixtral_hf_to_nxd

    cfg = _mixtral_cfg()
    hf = _mixtral_hf(cfg, seed=2)
    ps.initialize_model_parallel(tensor_model_parallel_size=world)
    m = _app(MixtralForCausalLMInference, cfg, mixtral_hf_to_nxd(hf.state_dict(), cfg), tp=world,
             decode_graph_steps=3)
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 9))
    out = m.generate(ids, max_new_tokens=8, eos_token_id=-1)
    m.compile(ckpt_dir)
    m2 = MixtralForCausalLMInference.load(ckpt_dir, dtype=torch.float32)
    again = m2.generate(ids, max_new_tokens=8, eos_token_id=-1)
    if rank == 0:
        torch.save({"greedy": out, "reload": again}, out_path)


def test_mixtral_tp2_matches_tp1_and_reload():
    d = tempfile.mkdtemp()
    run_distributed(_w_moe_tp, 1, os.path.join(d, "tp1.pt"), os.path.join(d, "c1"))
    run_distributed(_w_moe_tp, 2, os.path.join(d, "tp2.pt"), os.path.join(d, "c2"))
    a, b = torch.load(os.path.join(d, "tp1.pt")), torch.load(os.path.join(d, "tp2.pt"))
    assert torch.equal(a["greedy"], b["greedy"])
    assert torch.equal(a["greedy"], a["reload"]) and torch.equal(b["greedy"], b["reload"])


def test_mixtral_runner_from_hf_dir():
    """Runner flow on an HF directory on disk: trace (shard + write) -> load -> check_accuracy."""
    from neuronx_distributed_llama3_2_amd.inference import MixtralRunner

    cfg = _mixtral_cfg()
    hf = _mixtral_hf(cfg, seed=4)
    src, traced = tempfile.mkdtemp(), tempfile.mkdtemp()
    hf.save_pretrained(src)
    r = MixtralRunner(model_path=src)
    r.trace(traced, tp_degree=1, batch_size=1, max_prompt_length=16, sequence_length=32, capacity_factor=None)
    model = r.load_neuron_model(traced)
    assert model.config.capacity_factor is None
    prompts = [[5, 9, 13, 17, 21, 25]]
    assert r.check_accuracy(model, prompts, max_length=20)
