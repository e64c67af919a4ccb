"""MoE on the MI355X: grouped-GEMM HIP kernels (forward, input grad, fp32 weight grad) against an
fp32 PyTorch reference on ragged / empty expert groups, and a dropless MoE layer's forward +
backward running with no device->host synchronisation."""

import os

import pytest
import torch

import neuronx_distributed_llama3_2_amd.ops as ops
from neuronx_distributed_llama3_2_amd.ops import _ext
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _native():
    assert _ext.ext_available(), "HIP extension must be built for GPU tests"
    torch.manual_seed(0)
    yield


def _offs(counts):
    o = [0]
    for c in counts:
        o.append(o[-1] + c)
    return torch.tensor(o, dtype=torch.int32, device=DEV)


def _ref_fwd(x, w, offs):
    b = offs.tolist()
    y = torch.zeros(x.shape[0], w.shape[2], device=DEV)
    for e in range(w.shape[0]):
        y[b[e]:b[e + 1]] = x[b[e]:b[e + 1]].float() @ w[e].float()
    return y


@pytest.mark.parametrize("counts,K,N", [
    ([300, 0, 17, 128, 1, 555, 0, 40], 256, 384),     # ragged + empty groups, 128-aligned dims
    ([64, 200, 0, 3], 264, 392),                       # k / n tails (multiples of 8 only)
    ([0, 0, 0, 0], 128, 128),                          # no rows at all
    ([4096], 512, 640),                                # one big group
    ([1000, 0, 37, 700, 3, 513], 512, 1056),           # 256-tile kernels: ragged rows, partial column tiles
])
def test_grouped_gemm_fwd_dgrad_wgrad(counts, K, N):
    E = len(counts)
    M = sum(counts)
    offs = _offs(counts)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, K, N, device=DEV) / K ** 0.5).to(torch.bfloat16)
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    C = ops.ext()
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    C.grouped_gemm(0, x, w, offs, y, False)
    ref = _ref_fwd(x, w, offs)
    if M:
        assert torch.isfinite(y.float()).all()
        assert ((y.float() - ref).abs().max() / (ref.abs().max() + 1e-6)).item() < 1e-2
    dx = torch.full((M, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    C.grouped_gemm(1, dy, w, offs, dx, False)
    ref_dx = _ref_fwd(dy, w.transpose(1, 2).contiguous(), offs)
    if M:
        assert ((dx.float() - ref_dx).abs().max() / (ref_dx.abs().max() + 1e-6)).item() < 1e-2
    dw = torch.full((E, K, N), 3.0, device=DEV)
    C.grouped_gemm(2, x, dy, offs, dw, True)      # accumulate onto 3.0
    b = offs.tolist()
    for e in range(E):
        r = x[b[e]:b[e + 1]].float().t() @ dy[b[e]:b[e + 1]].float() + 3.0
        err = (dw[e] - r).abs().max().item()
        assert err <= 1e-3 * (r.abs().max().item() + 1.0), (e, err)
    dw0 = torch.full((E, K, N), float("nan"), device=DEV)
    C.grouped_gemm(2, x, dy, offs, dw0, False)    # overwrite: empty groups get exact zeros
    for e in range(E):
        if b[e] == b[e + 1]:
            assert (dw0[e] == 0).all()
    assert torch.isfinite(dw0).all()


def test_grouped_gemm_asymmetric_exact():
    # small-integer operands: exact in bf16/fp32, catches any row/col swap of the C layout
    counts = [5, 130, 0, 77]
    E, K, N = 4, 64, 136
    offs = _offs(counts)
    M = sum(counts)
    x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    w = torch.randint(-3, 4, (E, K, N), device=DEV).to(torch.bfloat16)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.ext().grouped_gemm(0, x, w, offs, y, False)
    assert torch.equal(y.float(), _ref_fwd(x, w, offs))


def _single():
    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29641")
        dist.init_process_group("gloo", rank=0, world_size=1)
    if not ps.model_parallel_is_initialized():
        ps.initialize_model_parallel(1)


def _moe(E=8, k=2, H=512, I=768, dtype=torch.bfloat16):
    from neuronx_distributed_llama3_2_amd.modules.moe import MoE, ExpertMLPs, RouterTopK

    torch.manual_seed(1)
    r = RouterTopK(E, k, H)
    mlps = ExpertMLPs(E, k, H, I, "silu", True, None, normalize_top_k_affinities=True, dtype=dtype)
    return MoE(r, mlps, return_router_logits=True)


@pytest.mark.parametrize("backend", ["grouped", "loop"])
def test_dropless_moe_matches_fp32_and_has_no_host_sync(backend, monkeypatch):
    """Both expert-GEMM backends match fp32; the grouped one never reads a group size on the host."""
    monkeypatch.setattr(ops.grouped_gemm, "MOE_GEMM", backend)
    _single()
    layer = _moe()
    ref_layer = _moe(dtype=torch.float32)               # same init, fp32, CPU reference path
    ref_layer.load_state_dict({k: v.float() for k, v in layer.state_dict().items()})
    layer = layer.to(DEV)
    layer.train()
    ref_layer.train()
    x = torch.randn(1024, 1, 512).to(torch.bfloat16).float()   # identical router inputs on both paths
    xg = x.to(DEV).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    torch.cuda.synchronize()
    if backend == "grouped":
        torch.cuda.set_sync_debug_mode("error")           # any device->host sync raises
    try:
        out, _ = layer(xg.to(torch.bfloat16))
        out.float().square().mean().backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    out_r, _ = ref_layer(xr)
    out_r.square().mean().backward()
    o, r = out.float().cpu(), out_r.detach()
    assert ((o - r).abs().max() / r.abs().max()).item() < 3e-2
    gx, gr = xg.grad.float().cpu(), xr.grad
    assert ((gx - gr).abs().max() / gr.abs().max()).item() < 5e-2
    for name in ["expert_mlps.mlp_op.gate_up_proj.weight", "expert_mlps.mlp_op.down_proj.weight"]:
        g = dict(layer.named_parameters())[name].grad.float().cpu()
        g_ref = dict(ref_layer.named_parameters())[name].grad
        assert ((g - g_ref).abs().max() / g_ref.abs().max()).item() < 5e-2, name


def test_grouped_linear_loop_backend_matches_grouped():
    """NXD_MOE_GEMM=loop (per-expert hipBLASLt over host bounds) == the device-side grouped kernel:
    forward, input gradient and fp32 weight gradient, ragged and empty groups included."""
    import neuronx_distributed_llama3_2_amd.ops as ops

    torch.manual_seed(0)
    E, T, k, K, N = 6, 700, 2, 256, 384
    idx = torch.randint(0, E - 1, (T, k), device="cuda")          # expert E-1 stays empty
    order, inverse, offs = ops.moe_permutation(idx, E)
    bounds = offs.tolist()
    x = torch.randn(T * k, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(E, K, N, device="cuda") * 0.05).to(torch.bfloat16)
    dy = torch.randn(T * k, N, device="cuda", dtype=torch.bfloat16)
    outs = []
    for b in (None, bounds):
        xr = x.clone().requires_grad_(True)
        wr = w.clone().requires_grad_(True)
        y = ops.grouped_linear(xr, wr, offs, b)
        y.backward(dy)
        outs.append((y.float(), xr.grad.float(), wr.grad.float()))
    for a, b in zip(*outs):
        assert ((a - b).abs().max() / (b.abs().max() + 1e-6)).item() < 2e-2


@pytest.mark.parametrize("T,k,H", [(513, 2, 4096), (64, 1, 1024), (300, 8, 2056)])
def test_moe_unpermute_combine_and_dispatch_match_fp32(T, k, H):
    """csrc/moe_combine.hip: un-permute + affinity-weighted combine (fwd: out, bwd: d ys and fp32
    d aff) and the dispatch gather's backward (a gather-sum) against fp32 PyTorch."""
    torch.manual_seed(3)
    E = 8
    idx = torch.stack([torch.randperm(E, device=DEV)[:k] for _ in range(T)])
    order, inverse, offs = ops.moe_permutation(idx, E)
    ys = torch.randn(T * k, H, device=DEV).to(torch.bfloat16).requires_grad_(True)
    aff = torch.rand(T, k, device=DEV).requires_grad_(True)
    out = ops.moe_unpermute_combine(ys, inverse, aff)
    dout = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    out.backward(dout)
    ys_r = ys.detach().float().requires_grad_(True)
    aff_r = aff.detach().clone().requires_grad_(True)
    ref = torch.einsum("tkh,tk->th", ys_r.index_select(0, inverse).view(T, k, H), aff_r)
    ref.backward(dout.float())
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    assert (ys.grad.float() - ys_r.grad).abs().max().item() < 1e-2 * ys_r.grad.abs().max().item()
    assert torch.allclose(aff.grad, aff_r.grad, rtol=1e-3, atol=1e-3 * aff_r.grad.abs().max().item())

    x = torch.randn(T, H, device=DEV).to(torch.bfloat16).requires_grad_(True)
    xs = ops.moe_dispatch(x, order, inverse, k)
    assert torch.equal(xs, x.detach().index_select(0, order // k))
    dxs = torch.randn(T * k, H, device=DEV).to(torch.bfloat16)
    xs.backward(dxs)
    ref_dx = torch.zeros(T, H, device=DEV).index_add_(0, order // k, dxs.float())
    assert (x.grad.float() - ref_dx).abs().max().item() < 1e-2 * ref_dx.abs().max().item()


def test_mixtral_trains_with_flat_adamw_fp32_router():
    """Tiny Mixtral (fp32 router + bf16 experts) trains on the GPU under the flat fp32-master AdamW:
    the fp32 parameter buffer takes the master copy (no bf16 write-back), loss goes down."""
    from neuronx_distributed_llama3_2_amd.models.mixtral import MixtralForCausalLM, mixtral_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW

    _single()
    torch.manual_seed(0)
    cfg = mixtral_config("tiny", hidden_size=512, num_attention_heads=4, num_key_value_heads=2, intermediate_size=256)
    model = MixtralForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device(DEV))
    model.train()
    router = model.model.layers[0].block_sparse_moe.router.linear_router.weight
    assert router.dtype == torch.float32
    r0 = router.detach().clone()
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=3e-3)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    losses = []
    for _ in range(6):
        loss = model(ids, labels=ids).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]
    assert router.dtype == torch.float32 and not torch.equal(router.detach(), r0)


@pytest.mark.parametrize("H,I,E,k,T", [(1024, 1792, 8, 2, 777), (4096, 14336, 8, 2, 2048)])
def test_moe_inference_prefill_grouped_no_sync(H, I, E, k, T):
    """MoE inference prefill (inference/modeling_moe.py `_grouped`) on the training path's sync-free
    kernels: expert weights in the output-major storage `post_load` gives them, bf16 within tolerance
    of an fp32 per-expert reference, no device->host sync, and faster than the per-expert matmul
    loop it replaced (Mixtral-8x7B shape at 2k tokens last)."""
    import types

    from neuronx_distributed_llama3_2_amd.inference.modeling_moe import MoEInferenceModel

    g = torch.Generator(device=DEV).manual_seed(H + T)
    x = torch.randn(T, H, device=DEV, generator=g).to(torch.bfloat16)
    # logical [E, H, 2I] / [E, I, H] parameters stored output-major, as post_load lays them out
    w_gu = (torch.randn(E, 2 * I, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16).transpose(1, 2)
    w_d = (torch.randn(E, H, I, device=DEV, generator=g) * I ** -0.5).to(torch.bfloat16).transpose(1, 2)
    logits = torch.randn(T, E, device=DEV, generator=g)
    top_w, top_i = torch.softmax(logits, -1).topk(k, -1)
    top_w = top_w / top_w.sum(-1, keepdim=True)
    m = types.SimpleNamespace(num_experts=E)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = MoEInferenceModel._grouped_device(m, x, top_w, top_i, w_gu, w_d)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    ref = torch.zeros(T, H, device=DEV)
    for e in range(E):
        rows, slot = (top_i == e).nonzero(as_tuple=True)
        if rows.numel():
            gu = x[rows].float() @ w_gu[e].float()
            a = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
            ref.index_add_(0, rows, (a.to(torch.bfloat16).float() @ w_d[e].float()) * top_w[rows, slot, None])
    assert ((out.float() - ref).abs().max() / ref.abs().max()).item() < 2e-2

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    dev_ms = timed(lambda: MoEInferenceModel._grouped_device(m, x, top_w, top_i, w_gu, w_d))
    loop_ms = timed(lambda: _loop(m, x, top_w, top_i, w_gu, w_d))
    print(f"moe prefill H={H} I={I} T={T}: grouped {dev_ms:.3f} ms, per-expert loop {loop_ms:.3f} ms")
    if H == 4096:
        # measured 2.09 vs 2.14 ms (profiles/r5_moe_prefill_grouped_vs_loop.txt): a 2 % gap that run-to-run
        # noise can close; the gate is "not slower" within 10 % (the win is the removed host sync)
        assert dev_ms < 1.1 * loop_ms, (dev_ms, loop_ms)


def _loop(m, x, top_w, top_i, w_gu, w_d):
    """The per-expert matmul loop with a host read of the group sizes (the prefill path before)."""
    from neuronx_distributed_llama3_2_amd.ops import swiglu

    n, k = top_i.shape
    flat = top_i.reshape(-1)
    order = torch.argsort(flat, stable=True)
    tok = order // k
    counts = torch.bincount(flat, minlength=m.num_experts).tolist()
    xs = x.index_select(0, tok)
    ys = torch.empty((n * k, x.shape[1]), dtype=x.dtype, device=x.device)
    start = 0
    for e, c in enumerate(counts):
        if c:
            ys[start:start + c] = torch.matmul(swiglu(torch.matmul(xs[start:start + c], w_gu[e])), w_d[e])
            start += c
    ys = ys.float() * top_w.reshape(-1)[order].unsqueeze(1)
    out = torch.zeros((n, x.shape[1]), dtype=torch.float32, device=x.device)
    out.index_add_(0, tok, ys)
    return out.to(x.dtype)
