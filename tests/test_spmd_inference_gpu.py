"""TP=2 serving on the GPU kernels (the fork's notebook config: Llama-3.2-1B, tp_degree=2; reference
examples/inference/llama3_2_inference.ipynb cell 8, trace/spmd.py:82-187), rehearsed on the one
MI355X of the test box: SpmdGenerationServer with 2 resident worker ranks sharing cuda:0 over gloo
(host-staged collectives, so decode runs eagerly), against a TP=1 server on the same GPU (RCCL
world of 1, hipGraph decode through the fused kernels).

bf16 TP=2 and TP=1 round their partial sums differently (the row-parallel all-reduce adds two bf16
partials), so a random-init model can flip a greedy argmax where its top-2 logits nearly tie.  The
check: greedy tokens identical for all 64 new tokens -- or, at the first differing position,
teacher-forced prefill logits of both servers agree (relative L2 and max errors <= 3.5e-2, ~10 %
above the largest of 18 measured samples, profiles/r6_tp2_prefill_parity_distribution.jsonl) and, in each row that flips, TP=1's margin between its token and TP=2's token is within
the two servers' logit differences at those two tokens (a genuine near-tie).  The
"peaked" model (untied lm_head = a row permutation of the embedding: next token = pi(current) by a
wide margin) must match exactly."""

import os
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(kind):
    from transformers import LlamaConfig

    if kind == "tiny":
        d = dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, vocab_size=2048, tie_word_embeddings=True)
    else:   # Llama-3.2-1B geometry
        d = dict(hidden_size=2048, intermediate_size=8192, num_hidden_layers=16, num_attention_heads=32,
                 num_key_value_heads=8, vocab_size=128256, tie_word_embeddings=kind != "peaked")
    d.update(max_position_embeddings=2048, rms_norm_eps=1e-5, rope_theta=500000.0, bos_token_id=1, eos_token_id=2,
             rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                           "original_max_position_embeddings": 8192})
    return LlamaConfig(**d)


def _random_full_state(cfg, kind, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    nq, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    D = H // nq

    def rnd(*shape, std=0.02):
        return (torch.randn(*shape, generator=g, device="cuda") * std).to(torch.bfloat16).cpu()

    emb_std = 1.0 if kind == "peaked" else 0.05
    sd = {"model.embed_tokens.weight": rnd(V, H, std=emb_std), "model.norm.weight": torch.ones(H, dtype=torch.bfloat16)}
    for i in range(cfg.num_hidden_layers):
        p = f"model.layers.{i}."
        sd[p + "self_attn.qkv_proj.weight_qkv"] = rnd((nq + 2 * nkv) * D, H)
        sd[p + "self_attn.o_proj.weight"] = rnd(H, nq * D, std=0.02 / (2 * cfg.num_hidden_layers) ** 0.5)
        sd[p + "mlp.gate_up_proj.weight"] = rnd(2 * I, H)
        sd[p + "mlp.down_proj.weight"] = rnd(H, I, std=0.02 / (2 * cfg.num_hidden_layers) ** 0.5)
        sd[p + "input_layernorm.weight"] = torch.ones(H, dtype=torch.bfloat16)
        sd[p + "post_attention_layernorm.weight"] = torch.ones(H, dtype=torch.bfloat16)
    if kind == "peaked":
        perm = torch.randperm(V, generator=torch.Generator().manual_seed(seed + 1))
        sd["lm_head.weight"] = sd["model.embed_tokens.weight"][torch.argsort(perm)].contiguous()
    else:
        sd["lm_head.weight"] = sd["model.embed_tokens.weight"]
    return sd


@pytest.mark.parametrize("kind", ["tiny", "llama3.2-1b", "peaked"])
def test_tp2_server_greedy_matches_tp1_on_gpu(kind):
    from neuronx_distributed_llama3_2_amd.inference.spmd_server import SpmdGenerationServer

    cfg = _cfg(kind)
    d = tempfile.mkdtemp()
    path = os.path.join(d, "full.pt")
    torch.save(_random_full_state(cfg, kind), path)
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 16))
    # deterministic: the TP=1 server skips the fp32-atomic fused attention + o_proj launch, so its
    # tokens do not vary from run to run
    kw = dict(batch_size=2, seq_len=128, max_context_length=96, deterministic=True)
    new = 64
    outs, servers = {}, {}
    try:
        for tp in (1, 2):
            servers[tp] = SpmdGenerationServer.from_full_state_dict(cfg.to_dict(), path, tp, kw, dtype="bfloat16")
            outs[tp] = servers[tp].generate(ids, max_new_tokens=new, eos_token_id=-1)
        a, b = outs[1], outs[2]
        assert a.shape == b.shape == (2, 16 + new)
        if kind == "peaked" or torch.equal(a, b):
            assert torch.equal(a, b), (a, b)
            return
        # first differing position: teacher-forced logits of both servers on TP=1's prefix
        diff = (a != b).any(0).nonzero()[0].item()
        assert diff >= 16
        prefix = a[:, :diff]
        la = servers[1].pool.call("_context_encode", prefix).float()
        lb = servers[2].pool.call("_context_encode", prefix).float()
        # bf16 TP=1 (fused decode kernels) vs TP=2 (unfused, all-reduced partials) over 16 layers:
        # the whole logit vector agrees to ~1 % (L2), single logits to a few % of the largest
        if la.dim() == 3:
            la, lb = la[:, -1], lb[:, -1]
        rel_l2 = (la - lb).norm() / la.norm()
        rel_max = (la - lb).abs().max() / la.abs().max()
        # distribution over 3 weight seeds x 6 prompts (profiles/r6_tp2_prefill_parity_distribution.jsonl):
        # Llama-3.2-1B rel_l2 p50 2.70e-2 / max 2.89e-2, rel_max p50 2.74e-2 / max 3.19e-2 (tiny model
        # <= 5.9e-3); the bound sits ~10 % above the largest.  These are PREFILL logits (TP=2 adds its
        # row-parallel partials in bf16), the bound on the prefix that decides the divergence
        print(f"{kind}: first differing token at {diff} ({diff - 16} new tokens identical); prefill logits "
              f"rel_l2 {float(rel_l2):.4f} rel_max {float(rel_max):.4f}")
        assert rel_l2 <= 3.5e-2 and rel_max <= 3.5e-2, (float(rel_l2), float(rel_max))
        # near-tie where the tokens differ: TP=1's preference for its token i1 over TP=2's token i2
        # must be within the two servers' logit differences AT THOSE TWO TOKENS (not over the vocab)
        margin = torch.tensor(0.0)
        for r in (a[:, diff] != b[:, diff]).nonzero().flatten().tolist():
            i1, i2 = int(a[r, diff]), int(b[r, diff])
            m = la[r, i1] - la[r, i2]
            slack = (la[r, i1] - lb[r, i1]).abs() + (la[r, i2] - lb[r, i2]).abs()
            # |m|: the tokens came from the decode kernels, la from the prefill ones (either may
            # rank the pair the other way inside the same noise)
            assert m.abs() <= slack, (diff, r, float(m), float(slack))
            margin = torch.maximum(margin, m.abs().cpu())
        print(f"{kind}: identical for {diff - 16} new tokens, then a near-tie (margin {float(margin):.4f})")
    finally:
        for s in servers.values():
            s.close()


def _teacher_forced(server, ids, P, steps, fused):
    """Prefill ids[:, :P], then `steps` eager decode calls fed ids[:, P + j] (teacher forcing):
    decode logits [B, steps, V] fp32."""
    B = ids.shape[0]
    server.pool.call("set_fused_decode", fused)
    server.pool.call("reset")
    server.pool.call("_context_encode", ids[:, :P])
    outs = []
    for j in range(steps):
        pos = torch.full((B, 1), P + j, dtype=torch.int64)
        outs.append(server.pool.call("_token_generate", ids[:, P + j:P + j + 1], None, pos).reshape(B, -1))
    return torch.stack(outs, 1)


@pytest.mark.parametrize("deterministic,batch", [(True, 2), (False, 2), (False, 4), (False, 8)])
def test_tp2_fused_decode_matches_unfused_like_tp1(deterministic, batch):
    """TP = 2 decode on the fused kernels with the one-shot peer all-reduce (two ranks on the GPU):
    against the same server's unfused decode (same prefill KV cache, so only the decode path differs)
    it differs no more than the TP = 1 fused decode does from the TP = 1 unfused one -- the two fused
    paths round identically; the TP=2 partials are summed in fp32.  deterministic=False (the serving
    default) takes the fp32-atomic attention + o_proj launch at batch <= 2 (its accumulator summed by
    the peer kernel with zero_in) and the MFMA row GEMVs with fp32 partials from batch 4."""
    from neuronx_distributed_llama3_2_amd.inference.spmd_server import SpmdGenerationServer

    cfg = _cfg("llama3.2-1b")
    d = tempfile.mkdtemp()
    path = os.path.join(d, "full.pt")
    torch.save(_random_full_state(cfg, "llama3.2-1b", seed=3), path)
    torch.manual_seed(9)
    P, steps = 24, 12
    ids = torch.randint(3, cfg.vocab_size, (batch, P + steps))
    kw = dict(batch_size=batch, seq_len=128, max_context_length=96, deterministic=deterministic, use_hip_graphs=False)
    rel = {}
    for tp in (1, 2):
        server = SpmdGenerationServer.from_full_state_dict(cfg.to_dict(), path, tp, kw, dtype="bfloat16")
        try:
            fused = _teacher_forced(server, ids, P, steps, True)
            plain = _teacher_forced(server, ids, P, steps, False)
        finally:
            server.close()
        rel[tp] = float((fused - plain).norm() / plain.norm())
        agree = float((fused.argmax(-1) == plain.argmax(-1)).float().mean())
        # (random-init logits are nearly tied everywhere: TP=1's own fused / unfused paths agree on
        # 87.5 % of the greedy picks, so agreement is reported, not asserted)
        print(f"TP={tp}: fused vs unfused decode logits rel_l2 {rel[tp]:.5f}, greedy agreement {agree:.3f}")
    assert rel[2] <= 2 * rel[1] + 2e-3, rel


def test_tp2_decode_hipgraph_on_peer_kernels():
    """TP = 2 over a gloo group (two ranks sharing the GPU): with every decode collective on the
    one-shot peer kernels (all-reduces and the vocabulary gather over IPC) the decode loop is captured
    in hipGraphs, and its greedy tokens equal the eager TP = 2 decode's."""
    from neuronx_distributed_llama3_2_amd.inference.spmd_server import SpmdGenerationServer

    cfg = _cfg("tiny")
    d = tempfile.mkdtemp()
    path = os.path.join(d, "full.pt")
    torch.save(_random_full_state(cfg, "tiny", seed=4), path)
    torch.manual_seed(11)
    ids = torch.randint(3, cfg.vocab_size, (2, 16))
    outs = {}
    for graphs in (True, False):
        kw = dict(batch_size=2, seq_len=128, max_context_length=96, deterministic=True, use_hip_graphs=graphs,
                  decode_graph_steps=8)
        server = SpmdGenerationServer.from_full_state_dict(cfg.to_dict(), path, 2, kw, dtype="bfloat16")
        try:
            assert server.pool.call("_decode_graphs_allowed") is graphs
            outs[graphs] = server.generate(ids, max_new_tokens=40, eos_token_id=-1)
        finally:
            server.close()
    assert torch.equal(outs[True], outs[False])


def test_tp2_decode_lost_peer_raises():
    """A TP = 2 rank that silently skips one decode all-reduce (NXD_PEER_AR_DROP, test hook): its peer's
    call sees the expected epoch with another call's signature (or times out), writes NaN and poisons
    its flags; generate() raises on the ranks instead of returning tokens."""
    from neuronx_distributed_llama3_2_amd.inference.spmd_server import SpmdGenerationServer

    cfg = _cfg("tiny")
    d = tempfile.mkdtemp()
    path = os.path.join(d, "full.pt")
    torch.save(_random_full_state(cfg, "tiny", seed=6), path)
    ids = torch.randint(3, cfg.vocab_size, (2, 16), generator=torch.Generator().manual_seed(2))
    kw = dict(batch_size=2, seq_len=128, max_context_length=96, deterministic=True, use_hip_graphs=False,
              decode_graph_steps=4)
    os.environ.update(NXD_PEER_AR_DROP="1:10", NXD_PEER_AR_SPIN_LIMIT="200000")
    try:
        server = SpmdGenerationServer.from_full_state_dict(cfg.to_dict(), path, 2, kw, dtype="bfloat16")
    finally:
        os.environ.pop("NXD_PEER_AR_DROP")
        os.environ.pop("NXD_PEER_AR_SPIN_LIMIT")
    try:
        with pytest.raises(RuntimeError, match="peer all-reduce"):
            server.generate(ids, max_new_tokens=24, eos_token_id=-1)
    finally:
        server.close()
