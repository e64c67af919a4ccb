"""Inference on MI355X: fused-kernel prefill vs fp32 CPU reference, hipGraph decode loop == eager
decode, sampling under graphs."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg():
    from transformers import LlamaConfig

    return LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                       num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                       rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)


def _model(cfg, sd, dtype, graphs=True, steps=8, device=None, seq_len=256, ctx=128):
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, LlamaForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd

    icfg = InferenceConfig(batch_size=2, seq_len=seq_len, max_context_length=ctx, use_hip_graphs=graphs,
                           decode_graph_steps=steps)
    m = LlamaForCausalLMInference(cfg, icfg, dtype=dtype, device=device, init_weights=False)
    m._load_full(hf_to_nxd(sd, cfg))
    return m


@pytest.fixture(scope="module")
def hf_sd():
    from transformers import LlamaForCausalLM as HF

    torch.manual_seed(0)
    cfg = _cfg()
    m = HF(cfg)
    return cfg, {k: v.detach().clone() for k, v in m.state_dict().items()}


def test_prefill_matches_cpu_reference(hf_sd):
    cfg, sd = hf_sd
    gpu = _model(cfg, sd, torch.bfloat16, device=torch.device("cuda"))
    cpu = _model(cfg, sd, torch.float32, device=torch.device("cpu"))
    torch.manual_seed(1)
    ids = torch.randint(3, cfg.vocab_size, (2, 100))
    mask = torch.ones_like(ids)
    mask[1, 70:] = 0
    lg = gpu._context_encode(ids, mask).cpu()
    lc = cpu._context_encode(ids, mask)
    err = (lg - lc).abs().max() / lc.abs().max()
    assert err < 3e-2, err
    # greedy top-1 agrees where the reference margin is comfortable
    top2 = lc.topk(2, -1).values
    ok = (top2[:, 0] - top2[:, 1]) > 0.05 * lc.abs().max()
    assert torch.equal(lg.argmax(-1)[ok], lc.argmax(-1)[ok])


def test_graph_decode_matches_eager(hf_sd):
    cfg, sd = hf_sd
    torch.manual_seed(2)
    ids = torch.randint(3, cfg.vocab_size, (2, 40))
    g = _model(cfg, sd, torch.bfloat16, graphs=True, steps=8, device=torch.device("cuda"))
    e = _model(cfg, sd, torch.bfloat16, graphs=False, steps=1, device=torch.device("cuda"))
    a = g.generate(ids, max_new_tokens=37, eos_token_id=-1)
    b = e.generate(ids, max_new_tokens=37, eos_token_id=-1)
    assert a.shape == (2, 77)
    # identical kernels; only hipBLASLt's stream-K prefill GEMMs may reorder fp32 sums run to run, which
    # can flip a near-tied argmax late in a random-weight model
    assert torch.equal(a[:, :60].cpu(), b[:, :60].cpu())
    assert (a.cpu() == b.cpu()).float().mean() > 0.95
    s1 = g.generate(ids, max_new_tokens=20, eos_token_id=-1, do_sample=True, top_k=20, seed=3)
    s2 = e.generate(ids, max_new_tokens=20, eos_token_id=-1, do_sample=True, top_k=20, seed=3)
    assert torch.equal(s1[:, :50].cpu(), s2[:, :50].cpu())
    assert not torch.equal(s1[:, 40:].cpu(), a[:, 40:60].cpu())  # sampling actually samples


def test_int8_inference_on_gpu(hf_sd):
    cfg, sd = hf_sd
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, LlamaForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd

    icfg = InferenceConfig(batch_size=2, seq_len=256, max_context_length=128, quantized=True,
                           quantization_type="per_channel_symmetric")
    q = LlamaForCausalLMInference(cfg, icfg, dtype=torch.bfloat16, device=torch.device("cuda"), init_weights=False)
    q._load_full(hf_to_nxd(sd, cfg))
    f = _model(cfg, sd, torch.bfloat16, device=torch.device("cuda"))
    ids = torch.randint(3, cfg.vocab_size, (2, 50))
    a, b = f._context_encode(ids), q._context_encode(ids)
    assert (a - b).abs().max() / a.abs().max() < 0.05
    out = q.generate(ids, max_new_tokens=20, eos_token_id=-1)
    assert out.shape == (2, 70)


def _greedy_consistent(model, ids_full, prompt_len, tol=0.08):
    """Every generated token is (within a small logit tolerance of) the target's argmax at its
    position, judged by ONE full causal forward over prompt + generation."""
    m = model.model
    B, T = ids_full.shape
    dev = model.device
    x = ids_full[:, :-1].to(dev)
    pos = torch.arange(T - 1, device=dev).unsqueeze(0).expand(B, T - 1)
    lg = m.forward_tokens(x, pos, torch.arange(B, device=dev), prefill=True).float()   # [B, T-1, V]
    lg = lg[:, prompt_len - 1:]
    chosen = lg.gather(-1, ids_full[:, prompt_len:].to(dev).unsqueeze(-1)).squeeze(-1)
    gap = lg.max(-1).values - chosen
    return float((gap <= tol * lg.abs().amax()).float().mean())


def test_speculative_decoding_gpu_graphs(hf_sd):
    """Device-resident speculation (hipGraph rounds) on MI355X: with a same-weights draft nearly
    every round accepts all K drafts, and the emitted tokens are the target's greedy choices."""
    cfg, sd = hf_sd
    dev = torch.device("cuda")
    tgt = _model(cfg, sd, torch.bfloat16, device=dev)
    tgt.config.speculation_length = 4
    draft = _model(cfg, sd, torch.bfloat16, device=dev)
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 40))
    out = tgt.generate(ids, max_new_tokens=48, eos_token_id=None, assistant_model=draft)
    assert out.shape == (2, 88)
    dec = next(iter(tgt._spec.values()))
    assert dec.last_stats["tokens_per_round"] > 3.0, dec.last_stats  # ~K+1 (bf16 ties may reject)
    ref = tgt.generate(ids, max_new_tokens=48, eos_token_id=None)
    # random-init weights give near-tied logits: judge greedy consistency, not token equality
    assert _greedy_consistent(tgt, ref, 40) > 0.97
    assert _greedy_consistent(tgt, out, 40) > 0.97


def test_expert_gemv_kernel_matches_fp32():
    """Expert-mode skinny GEMM (csrc/gemv.hip): pair p uses x row p // xdiv and expert eidx[p],
    with and without the fused SwiGLU epilogue, vs an fp32 PyTorch reference."""
    from neuronx_distributed_llama3_2_amd.ops import ext
    from neuronx_distributed_llama3_2_amd.ops.gemv import expert_linear

    torch.manual_seed(0)
    E, K, N, T, k = 8, 1024, 704, 3, 2
    w = (torch.randn(E, 2 * N, K, device="cuda") * 0.05).to(torch.bfloat16)
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    eidx = torch.randint(0, E, (T * k,), device="cuda", dtype=torch.int32)
    ext()   # the native kernel must be present on a GPU box
    y = expert_linear(x, w, eidx, xdiv=k, glu=True)
    rows = x.float()[torch.arange(T * k, device="cuda") // k]
    full = torch.einsum("pk,pnk->pn", rows, w.float()[eidx.long()])
    ref = torch.nn.functional.silu(full[:, :N]) * full[:, N:]
    assert (y.float() - ref).abs().max() < 2e-2 * ref.abs().max() + 1e-3
    y2 = expert_linear(x, w, eidx, xdiv=k, glu=False)
    assert (y2.float() - full).abs().max() < 2e-2 * full.abs().max() + 1e-3


def test_mixtral_inference_gpu_graphs_match_cpu():
    """Mixtral MoE inference on the GPU (bf16, hipGraph decode with selective-loading experts)
    vs the fp32 CPU path: prefill logits close, graph decode == eager decode."""
    from transformers import MixtralConfig, MixtralForCausalLM

    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, MixtralForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.mixtral.convert import mixtral_hf_to_nxd

    cfg = MixtralConfig(hidden_size=512, intermediate_size=768, num_hidden_layers=2, num_attention_heads=8,
                        num_key_value_heads=2, vocab_size=1000, max_position_embeddings=512, num_local_experts=8,
                        num_experts_per_tok=2, eos_token_id=2)
    torch.manual_seed(0)
    hf = MixtralForCausalLM(cfg)
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if "experts" in n:
                p.normal_(0.0, 0.05)
        hf.lm_head.weight.mul_(20.0)   # wide argmax margins: random-init logits are otherwise near-tied
    full = mixtral_hf_to_nxd({k: v.detach().clone() for k, v in hf.state_dict().items()}, cfg)

    def app(dtype, device, graphs):
        icfg = InferenceConfig(batch_size=1, seq_len=128, max_context_length=64, use_hip_graphs=graphs,
                               decode_graph_steps=4)
        m = MixtralForCausalLMInference(cfg, icfg, dtype=dtype, device=device, init_weights=False)
        m._load_full(full)
        return m

    gpu = app(torch.bfloat16, torch.device("cuda"), True)
    eager = app(torch.bfloat16, torch.device("cuda"), False)
    cpu = app(torch.float32, torch.device("cpu"), False)
    ids = torch.randint(3, cfg.vocab_size, (1, 40))
    lg, lc = gpu._context_encode(ids).cpu(), cpu._context_encode(ids)
    assert ((lg - lc).abs().max() / lc.abs().max()) < 3e-2
    a = gpu.generate(ids, max_new_tokens=12, eos_token_id=-1).cpu()
    b = eager.generate(ids, max_new_tokens=12, eos_token_id=-1).cpu()
    # same kernels; hipBLASLt stream-K prefill GEMMs may reorder fp32 sums run to run (see
    # test_graph_decode_matches_eager), so allow a late near-tie flip
    assert torch.equal(a[:, :46], b[:, :46]) and (a == b).float().mean() > 0.9, (a, b)


@pytest.mark.parametrize("hidden,heads", [(512, 8), (1024, 8)])   # head_dim 64 and 128
def test_fused_decode_matches_unfused(hidden, heads):
    """decode_fused.hip path (norm / RoPE / KV write / residual fused into the GEMVs) vs the
    unfused kernel chain: same greedy tokens, same KV cache, close logits."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF

    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=2, num_attention_heads=heads,
                      num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    f = _model(cfg, sd, torch.bfloat16, graphs=False, steps=1, device=torch.device("cuda"))
    u = _model(cfg, sd, torch.bfloat16, graphs=False, steps=1, device=torch.device("cuda"))
    u.model._decode_fused_ok = False
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 33))
    a = f.generate(ids, max_new_tokens=24, eos_token_id=-1)
    assert f.model._decode_fused_ok is True, "fused decode path was not taken"
    b = u.generate(ids, max_new_tokens=24, eos_token_id=-1)
    assert torch.equal(a[:, :43].cpu(), b[:, :43].cpu())
    assert (a.cpu() == b.cpu()).float().mean() > 0.9
    kf, ku = f.model.kv_cache[:, :, :, :, :50].float(), u.model.kv_cache[:, :, :, :, :50].float()
    assert ((kf - ku).abs().max() / ku.abs().max()).item() < 3e-2
    # one decode step on identical caches: logits agree
    f.model.kv_cache.copy_(u.model.kv_cache)
    last = b[:, -1:].cuda()
    pos = torch.full((2, 1), b.shape[1] - 1, dtype=torch.int64, device="cuda")
    sid = torch.arange(2, device="cuda")
    clen = torch.full((2,), b.shape[1], dtype=torch.int32, device="cuda")
    lf = f.model.forward_tokens(last, pos, sid, clen).float()
    lu = u.model.forward_tokens(last, pos, sid, clen).float()
    assert ((lf - lu).abs().max() / lu.abs().max()).item() < 3e-2


@pytest.mark.parametrize("hidden,heads,kv", [(512, 8, 2), (2048, 32, 8), (1024, 8, 2)])   # D = 64, 64, 128
def test_fused_attention_oproj_matches_two_launches(monkeypatch, hidden, heads, kv):
    """decode_attn.hip FUSE (attention + o_proj in one launch, o_proj rows added by float atomics
    into an fp32 accumulator that the GLU prologue / down epilogue fold into the residual) vs the
    attention launch + RESID o_proj GEMV: same greedy tokens, close logits, accumulator left zero."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base

    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=2, num_attention_heads=heads,
                      num_key_value_heads=kv, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 33))
    outs, models = [], []
    for on in (True, False):
        monkeypatch.setattr(model_base, "_ATTN_OPROJ", on)
        m = _model(cfg, sd, torch.bfloat16, graphs=True, steps=4, device=torch.device("cuda"))
        outs.append(m.generate(ids, max_new_tokens=24, eos_token_id=-1).cpu())
        models.append(m)
    assert models[0].model._decode_fused_ok is True
    buf = getattr(models[0].model, "_oacc_buf", None)
    assert buf is not None and int((buf != 0).sum()) == 0, "fused path not taken or accumulator not consumed"
    assert torch.equal(outs[0][:, :45], outs[1][:, :45]) and (outs[0] == outs[1]).float().mean() > 0.95
    # one decode step on identical caches: logits agree
    f, u = models[0].model, models[1].model
    f.kv_cache.copy_(u.kv_cache)
    last = outs[1][:, -1:].cuda()
    pos = torch.full((2, 1), outs[1].shape[1] - 1, dtype=torch.int64, device="cuda")
    sid = torch.arange(2, device="cuda")
    clen = torch.full((2,), outs[1].shape[1], dtype=torch.int32, device="cuda")
    monkeypatch.setattr(model_base, "_ATTN_OPROJ", True)
    lf = f.forward_tokens(last, pos, sid, clen).float()
    monkeypatch.setattr(model_base, "_ATTN_OPROJ", False)
    lu = u.forward_tokens(last, pos, sid, clen).float()
    assert ((lf - lu).abs().max() / lu.abs().max()).item() < 2e-2


@pytest.mark.parametrize("hidden,heads,kv", [(2048, 32, 8), (1024, 8, 2)])   # D = 64, 128
def test_fused_attention_oproj_long_context(monkeypatch, hidden, heads, kv):
    """The fused attention + o_proj launches on a cache past one 1,024-key split (the notebook config's
    2,048-token context + 256 new) -- every workgroup walking the whole cache; the default single launch
    whose workgroups each take a key split, wait for the head's partials and merge them; and the split
    attention launch whose partials the o_proj launch merges -- one decode step each against the split
    attention + merge + o_proj launches on identical caches."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base

    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=2, num_attention_heads=heads,
                      num_key_value_heads=kv, vocab_size=1000, max_position_embeddings=4096, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    torch.manual_seed(7)
    P = 1800
    ids = torch.randint(3, cfg.vocab_size, (2, P))
    m = _model(cfg, sd, torch.bfloat16, graphs=False, steps=1, device=torch.device("cuda"), seq_len=2304, ctx=2048)
    m.generate(ids, max_new_tokens=2, eos_token_id=-1)    # fills the cache with P + 1 positions
    f = m.model
    last = torch.randint(3, cfg.vocab_size, (2, 1), device="cuda")
    pos = torch.full((2, 1), P + 1, dtype=torch.int64, device="cuda")
    sid = torch.arange(2, device="cuda")
    clen = torch.full((2,), P + 2, dtype=torch.int32, device="cuda")
    saved = f.kv_cache.clone()
    from neuronx_distributed_llama3_2_amd.ops import ext as _native

    def step(fuse, maxl, sync=1):
        f.kv_cache.copy_(saved)
        monkeypatch.setattr(model_base, "_ATTN_OPROJ", fuse)
        _native().decode_attn_set_oproj_maxl(maxl)
        _native().decode_attn_set_sync(sync)
        try:
            out = f.forward_tokens(last, pos, sid, clen).float()
        finally:
            _native().decode_attn_set_oproj_maxl(int(os.environ.get("NXD_DECODE_ATTN_OPROJ_MAXL", "1024")))
            _native().decode_attn_set_sync(int(os.environ.get("NXD_DECODE_ATTN_SYNC", "0")))
        assert _native().decode_attn_sync_error(True) == 0
        if fuse:
            buf = getattr(f, "_oacc_buf", None)
            assert buf is not None and int((buf != 0).sum()) == 0, "fused path not taken or accumulator not consumed"
        return out

    lu = step(False, 1024)
    lf = step(True, 4096)    # one pass over the whole cache per workgroup
    ls = step(True, 1024, sync=1)   # one launch: key split per workgroup, in-launch merge, o_proj (opt-in)
    l2 = step(True, 1024, sync=0)   # split attention launch, partials merged inside the o_proj launch
    for got in (lf, ls, l2):
        assert ((got - lu).abs().max() / lu.abs().max()).item() < 2e-2


@pytest.mark.parametrize("hidden,heads,batch,split", [(512, 8, 2, 0), (1024, 8, 4, 0), (2048, 32, 8, 0), (2048, 32, 8, 1)])
def test_fused_decode_mfma_rows_match_valu(monkeypatch, hidden, heads, batch, split):   # D = 64, 128, 64, 64
    """decode_fused.hip dmm_kernel (2-8 activation rows on MFMA 16-row weight tiles: QKV + RoPE + KV
    write, SwiGLU, residual and plain epilogues, k split over waves and workgroups) vs the VALU GEMV
    body: same greedy tokens, same KV cache, close one-step logits."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base
    from neuronx_distributed_llama3_2_amd.ops import _ext

    C = _ext.ext()
    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=4 * hidden, num_hidden_layers=2, num_attention_heads=heads,
                      num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    torch.manual_seed(7)
    ids = torch.randint(3, cfg.vocab_size, (batch, 29))
    monkeypatch.setattr(model_base, "_ATTN_OPROJ", False)   # deterministic attention + o_proj
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, LlamaForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd

    outs, models = [], []
    C.decode_set_knob(8, split)   # K also split over workgroups
    try:
        for rows in (0, 2):   # VALU body, then MFMA from 2 rows
            C.decode_set_knob(7, rows)
            icfg = InferenceConfig(batch_size=batch, seq_len=256, max_context_length=128, use_hip_graphs=False,
                                   decode_graph_steps=1)
            m = LlamaForCausalLMInference(cfg, icfg, dtype=torch.bfloat16, device=torch.device("cuda"), init_weights=False)
            m._load_full(hf_to_nxd(sd, cfg))
            outs.append(m.generate(ids, max_new_tokens=20, eos_token_id=-1).cpu())
            assert m.model._decode_fused_ok is True
            models.append(m)
        # random-init weights have near-tied logits: greedy generation is judged for consistency
        # with one full prefill forward of the same model, not for token equality
        C.decode_set_knob(7, 2)
        assert _greedy_consistent(models[1], outs[1], 29) > 0.97
        # one decode step on identical caches: logits and the K / V rows it writes agree
        models[1].model.kv_cache.copy_(models[0].model.kv_cache)
        n = outs[0].shape[1]
        last = outs[0][:, -1:].cuda()
        pos = torch.full((batch, 1), n - 1, dtype=torch.int64, device="cuda")
        sid = torch.arange(batch, device="cuda")
        clen = torch.full((batch,), n, dtype=torch.int32, device="cuda")
        lg = []
        for rows, m in zip((0, 2), models):
            C.decode_set_knob(7, rows)
            lg.append(m.model.forward_tokens(last, pos, sid, clen).float())
        assert ((lg[0] - lg[1]).abs().max() / lg[0].abs().max()).item() < 2e-2
        kv = models[0].model.kv_cache[:, :, :, :, n - 1].float()
        km = models[1].model.kv_cache[:, :, :, :, n - 1].float()
        assert ((kv - km).abs().max() / kv.abs().max()).item() < 3e-2
    finally:
        C.decode_set_knob(7, 4)
        C.decode_set_knob(8, 0)


def test_fused_decode_weight_prefetch_is_exact(monkeypatch):
    """Spare attention workgroups streaming o_proj / gate_up into the Infinity Cache only read:
    decode tokens and logits are bit-identical with and without the prefetch."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=True, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 33))
    outs = []
    for mb in (0.0, 64.0):   # 64 MiB clamps to the whole gate_up weight
        monkeypatch.setattr(model_base, "_PREFETCH_MB", mb)
        m = _model(cfg, sd, torch.bfloat16, graphs=True, steps=4, device=torch.device("cuda"))
        outs.append(m.generate(ids, max_new_tokens=16, eos_token_id=-1).cpu())
        assert m.model._decode_fused_ok is True
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("batch", [1, 2])
def test_fused_decode_embedding_gather_is_exact(monkeypatch, batch):
    """The embedding gather folded into layer 0's QKV launch (xidx / xcopy) copies the same bf16
    rows the embedding kernel would: decode logits and tokens are bit-identical with and without it
    (bs = 1 takes the prologue-ahead path, bs = 2 the multi-row one)."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=False, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    torch.manual_seed(6)
    ids = torch.randint(3, cfg.vocab_size, (batch, 21))
    monkeypatch.setattr(model_base, "_ATTN_OPROJ", False)   # deterministic (no fp32 atomics)
    outs, logits = [], []
    n = ids.shape[1] + 12
    last = torch.randint(3, cfg.vocab_size, (batch, 1)).cuda()
    pos = torch.full((batch, 1), n, dtype=torch.int64, device="cuda")
    sid = torch.arange(batch, device="cuda")
    clen = torch.full((batch,), n + 1, dtype=torch.int32, device="cuda")
    for on in (False, True):
        monkeypatch.setattr(model_base, "_EMB_FUSED", on)
        m = _model(cfg, sd, torch.bfloat16, graphs=True, steps=4, device=torch.device("cuda"))
        outs.append(m.generate(ids, max_new_tokens=12, eos_token_id=-1).cpu())
        assert m.model._decode_fused_ok is True
        # one more (eager) decode step on the caches the generation left, then the same step with
        # out-of-range ids (pad -1, past the vocabulary): both paths embed a zero row for those
        steps = [m.model.forward_tokens(last, pos, sid, clen).float().cpu()]
        for bad in (-1, cfg.vocab_size + 5):
            steps.append(m.model.forward_tokens(torch.full_like(last, bad), pos, sid, clen).float().cpu())
        logits.append(steps)
    for a, b in zip(logits[0], logits[1]):
        assert torch.equal(a, b)
    assert not torch.equal(logits[0][0], logits[0][1])


def test_weight_layout_pass_on_gpu(hf_sd):
    """Measured layout pass at the prefill size: every weight gets a layout, packed copies are
    K-major, and prefill logits match the stored-layout model (forced-packed too)."""
    from neuronx_distributed_llama3_2_amd.trace import weight_layout as wl

    cfg, sd = hf_sd
    m = _model(cfg, sd, torch.bfloat16, device=torch.device("cuda"))
    torch.manual_seed(3)
    ids = torch.randint(3, cfg.vocab_size, (2, 100))
    ref = m._context_encode(ids).cpu()
    layouts = wl.choose_layouts(m.model, 256)
    names = [n for n, _ in wl._weights(m.model)]
    assert set(layouts) == set(names) and set(layouts.values()) <= {"nk", "kn"}
    for forced in (layouts, {n: "kn" for n in names}):
        wl.apply_layouts(m.model, forced)
        out = m._context_encode(ids).cpu()
        err = (out - ref).abs().max() / ref.abs().max()
        assert err < 1e-2, err


def test_prefill_graphs_match_eager(hf_sd):
    """Context encoding replayed from per-(batch, bucket) hipGraphs == the eager forward, across
    buckets and repeated calls; greedy generation after a graphed prefill is unchanged."""
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, LlamaForCausalLMInference
    from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd

    cfg, sd = hf_sd
    models = {}
    for graphs in (True, False):
        icfg = InferenceConfig(batch_size=2, seq_len=256, max_context_length=128, prefill_graphs=graphs)
        m = LlamaForCausalLMInference(cfg, icfg, dtype=torch.bfloat16, device=torch.device("cuda"), init_weights=False)
        m._load_full(hf_to_nxd(sd, cfg))
        models[graphs] = m
    torch.manual_seed(5)
    for T in (100, 30, 100):
        ids = torch.randint(3, cfg.vocab_size, (2, T))
        mask = torch.ones_like(ids)
        mask[1, T // 2:] = 0
        a = models[True]._context_encode(ids, mask)
        b = models[False]._context_encode(ids, mask)
        assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()
    assert len(models[True]._prefill_cache) == 1 and not models[False]._prefill_cache  # one (2, 128) bucket
    ids = torch.randint(3, cfg.vocab_size, (1, 40))
    ga = models[True].generate(ids, max_new_tokens=12, eos_token_id=-1)
    gb = models[False].generate(ids, max_new_tokens=12, eos_token_id=-1)
    assert torch.equal(ga, gb)
    assert len(models[True]._prefill_cache) == 2   # + (1, 128)


@pytest.mark.parametrize("V,dtype", [(128256, torch.bfloat16), (1001, torch.bfloat16), (5000, torch.float32)])
def test_greedy_advance_kernel(V, dtype):
    """Multi-workgroup argmax (ties -> lowest index, as torch.argmax) + decode-state feed-back."""
    from neuronx_distributed_llama3_2_amd import ops

    torch.manual_seed(V)
    B, S = 3, 8
    logits = torch.randn(B, V, device="cuda").to(dtype)
    logits[1, V // 3] = logits[1, V - 1] = 50.0          # tie: the first one wins
    logits[2] = -1.0                                      # all equal: index 0
    slot = torch.zeros(B, dtype=torch.int64, device="cuda")
    out = torch.zeros(B, S, dtype=torch.int64, device="cuda")
    step = torch.tensor([2], dtype=torch.int64, device="cuda")
    tokens = torch.zeros(B, 1, dtype=torch.int64, device="cuda")
    positions = torch.tensor([[5], [6], [7]], device="cuda")
    cache_len = torch.tensor([6, 7, 8], dtype=torch.int32, device="cuda")
    ops.greedy_advance_(logits, slot, out, step, tokens, positions, cache_len)
    ref = torch.argmax(logits.float(), dim=-1)
    assert torch.equal(tokens.view(-1), ref) and int(ref[1]) == V // 3 and int(ref[2]) == 0
    assert torch.equal(out[:, 2], ref) and int(out[:, [0, 1, 3]].abs().sum()) == 0
    assert int(step) == 3 and positions.view(-1).tolist() == [6, 7, 8] and cache_len.tolist() == [7, 8, 9]
    assert int(slot.abs().sum()) == 0


def test_greedy_fused_decode_matches_unfused(hf_sd):
    from neuronx_distributed_llama3_2_amd.inference import graphs

    cfg, sd = hf_sd
    m = _model(cfg, sd, torch.bfloat16, device=torch.device("cuda"))
    torch.manual_seed(9)
    ids = torch.randint(3, cfg.vocab_size, (2, 33))
    outs = []
    for fused in (True, False):
        graphs.GREEDY_FUSED = fused
        m._graphs.clear()
        try:
            outs.append(m.generate(ids, max_new_tokens=20, eos_token_id=-1))
        finally:
            graphs.GREEDY_FUSED = True
    assert torch.equal(outs[0], outs[1])


def test_decode_attention_phase_trace(monkeypatch):
    """The opt-in phase trace of the decode attention launches (decode_attn.hip Params::trace, the
    trailing field whose round-4 version aborted these tests while one launcher left it
    uninitialised): armed, each workgroup stamps entry <= exit; disarmed, decode output is unchanged."""
    from transformers import LlamaConfig, LlamaForCausalLM as HF
    from neuronx_distributed_llama3_2_amd.inference import model_base
    from neuronx_distributed_llama3_2_amd import _C

    cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=8,
                      num_key_value_heads=2, vocab_size=1000, max_position_embeddings=1024, rms_norm_eps=1e-5,
                      rope_theta=500000.0, tie_word_embeddings=False, eos_token_id=2)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in HF(cfg).state_dict().items()}
    m = _model(cfg, sd, torch.bfloat16, graphs=False, steps=1, device=torch.device("cuda"))
    ids = torch.randint(3, cfg.vocab_size, (1, 21))
    m.generate(ids, max_new_tokens=2, eos_token_id=-1)
    last = torch.randint(3, cfg.vocab_size, (1, 1)).cuda()
    pos = torch.full((1, 1), 23, dtype=torch.int64, device="cuda")
    sid = torch.arange(1, device="cuda")
    clen = torch.full((1,), 24, dtype=torch.int32, device="cuda")
    for fused in (True, False):
        monkeypatch.setattr(model_base, "_ATTN_OPROJ", fused)
        ref = m.model.forward_tokens(last, pos, sid, clen).float()
        tr = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
        _C.decode_attn_trace(tr)
        try:
            out = m.model.forward_tokens(last, pos, sid, clen).float()
        finally:
            _C.decode_attn_trace(None)
        torch.cuda.synchronize()
        t = tr.view(-1, 2).cpu()
        hit = t[:, 0] > 0
        assert hit.any() and bool((t[hit, 1] >= t[hit, 0]).all()), t[:8]
        if not fused:
            assert torch.equal(out, ref)
